#!/bin/bash
# A/B on one box: slab reduction with 4 columns per lane (default) vs 8 (half the workgroups)
set -uo pipefail
OUT=gpurun_out/r06y
mkdir -p $OUT
for rep in 1 2 3; do for v in c4 c8; do
  if [ $v = c4 ]; then LP=""; else LP=$GRAFT_REPO_ROOT/tools/ab/liblgnn_red8.so; fi
  for w in c2 c4; do
    LGNN_LIB_PATH=$LP timeout -k 10 200 python bench.py --workload $w --steps 300 --warmup 50 --cpu-seconds 0 --entries 0 --no-kernel-timing > $OUT/${w}_${v}_$rep.json 2>$OUT/err || { tail $OUT/err; exit 1; }
    python -c "import json; d=json.loads(open('$OUT/${w}_${v}_$rep.json').read().strip().splitlines()[-1]); print('$w cols=$v', d['ms_per_step'])"
  done
done; done
