#!/bin/bash
# round-6 box 2: what the three general-path build launches cost in the C2 step (ablation library
# without them on sorted input, same box), and the probe kernels' rocprof durations
set -uo pipefail
OUT=gpurun_out/r06b
mkdir -p $OUT
export TMPDIR=/tmp
for rep in 1 2; do
  timeout -k 10 200 python bench.py --steps 300 --warmup 30 --cpu-seconds 0 > $OUT/intree_$rep.json 2>$OUT/err || { tail $OUT/err; exit 1; }
  LGNN_LIB_PATH=$GRAFT_REPO_ROOT/tools/_abl/liblgnn_abl.so LGNN_ABL_SKIP_GENERAL=1 timeout -k 10 200 python bench.py --steps 300 --warmup 30 --cpu-seconds 0 > $OUT/skip_$rep.json 2>$OUT/err || { tail $OUT/err; exit 1; }
  for v in intree skip; do python -c "import json; d=json.loads(open('$OUT/${v}_$rep.json').read().strip().splitlines()[-1]); print('$v', d['ms_per_step'])"; done
done
cd /tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$OUT/probe -o trace -- python3 $GRAFT_REPO_ROOT/tools/launch_cost.py > $GRAFT_REPO_ROOT/$OUT/probe.txt 2>&1 || exit 1
S=$(find $GRAFT_REPO_ROOT/$OUT/probe -name "*kernel_stats.csv" | head -1)
cut -d, -f1-4 $S | head -12
