#!/bin/bash
# A/B: next-tile H_L rows issued at the first conv (new default) vs the last conv (late)
set -uo pipefail
OUT=gpurun_out/r06r
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
  tests/test_gpu_gcn.py tests/test_gpu_ce_fused.py > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
for rep in 1 2 3; do for v in new late; do
  if [ $v = new ]; then LP=""; else LP=$GRAFT_REPO_ROOT/tools/ab/liblgnn_late.so; fi
  for w in c2 sweep_gcn3; do
    LGNN_LIB_PATH=$LP timeout -k 10 200 python bench.py --workload $w --steps 300 --warmup 50 --cpu-seconds 0 --entries 0 > $OUT/${w}_${v}_$rep.json 2>$OUT/err || { tail $OUT/err; exit 1; }
    python -c "import json; d=json.loads(open('$OUT/${w}_${v}_$rep.json').read().strip().splitlines()[-1]); r=d.get('roofline') or {}; print('$w $v', d['ms_per_step'], r.get('avg_launch_ms'))"
  done
done; done
