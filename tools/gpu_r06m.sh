#!/bin/bash
# Where does the driver command's short-run overhead come from: steps/warmup grid on one box.
set -uo pipefail
mkdir -p gpurun_out/r06m
for sw in "20 5" "20 50" "300 5" "20 5" "100 5" "300 50"; do
  set -- $sw
  timeout -k 10 300 python bench.py --steps $1 --warmup $2 --cpu-seconds 0 --entries 0 \
    > gpurun_out/r06m/b_$1_$2.json 2> gpurun_out/r06m/b_$1_$2.err || { tail -20 gpurun_out/r06m/b_$1_$2.err; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/r06m/b_$1_$2.json')); print('steps $1 warmup $2', d['value'], d['ms_per_step'])"
done
