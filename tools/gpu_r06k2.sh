#!/bin/bash
# A/B on one box: HIP_FORCE_DEV_KERNARG=1 (kernel arguments in device memory) vs the default
set -uo pipefail
OUT=gpurun_out/r06k2
mkdir -p $OUT
for rep in 1 2 3; do for v in dflt devk; do
  if [ $v = devk ]; then export HIP_FORCE_DEV_KERNARG=1; else unset HIP_FORCE_DEV_KERNARG; fi
  for w in c2 refcfg; do
    timeout -k 10 300 python bench.py --workload $w --steps 300 --warmup 50 --cpu-seconds 0 --entries 0 --no-kernel-timing > $OUT/${w}_${v}_$rep.json 2>$OUT/err || { tail $OUT/err; exit 1; }
    python -c "import json; d=json.loads(open('$OUT/${w}_${v}_$rep.json').read().strip().splitlines()[-1]); print('$w $v', d['ms_per_step'])"
  done
done; done
