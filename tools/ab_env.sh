#!/bin/bash
# A/B of one environment toggle on one box (C2 bench unless WL is set):
#   bash tools/ab_env.sh VAR "a b" [bench args...]
set -e
VAR=$1; VALS=$2; shift 2
mkdir -p gpurun_out/ab
for rep in 1 2; do for v in $VALS; do
  env $VAR=$v timeout -k 10 200 python bench.py --steps 300 --warmup 30 --cpu-seconds 0 "$@" > gpurun_out/ab/${VAR}_$v.json
  python -c "import json; d=json.loads(open('gpurun_out/ab/${VAR}_$v.json').read().strip().splitlines()[-1]); print('$VAR=$v', d['ms_per_step'])"
done; done
