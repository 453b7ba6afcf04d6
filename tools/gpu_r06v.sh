#!/bin/bash
# A/B on one box: layer-wise tile kernels' partial slots capped at 512 (default) vs 256
set -uo pipefail
OUT=gpurun_out/r06v
mkdir -p $OUT
for rep in 1 2; do for v in p512 p256; do
  if [ $v = p512 ]; then LP=""; else LP=$GRAFT_REPO_ROOT/tools/ab/liblgnn_p256.so; fi
  for w in c4 c5k16 c5k4; do
    LGNN_LIB_PATH=$LP timeout -k 10 200 python bench.py --workload $w --steps 200 --warmup 30 --cpu-seconds 0 --entries 0 > $OUT/${w}_${v}_$rep.json 2>$OUT/err || { tail $OUT/err; exit 1; }
    python -c "import json; d=json.loads(open('$OUT/${w}_${v}_$rep.json').read().strip().splitlines()[-1]); print('$w $v', d['ms_per_step'])"
  done
done; done
