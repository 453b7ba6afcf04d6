#!/bin/bash
# round-6 box: head-pipelined fused backward (HP): parity, then A/B vs the previous library
set -uo pipefail
OUT=gpurun_out/r06i
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_ce_fused.py tests/test_gpu_gcn.py tests/test_gpu_configs.py tests/test_gpu_s3.py tests/test_gpu_weight_planes.py tests/test_gpu_dist.py -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1
rc=$?
tail -2 $OUT/pytest.log; grep -E "^FAILED|^ERROR" $OUT/pytest.log | head -5
[ $rc -eq 0 ] || exit $rc
for rep in 1 2; do for v in new prev; do
  if [ $v = new ]; then LP=""; else LP=$GRAFT_REPO_ROOT/tools/_abl/liblgnn_prev.so; fi
  LGNN_LIB_PATH=$LP timeout -k 10 200 python bench.py --steps 300 --warmup 50 --cpu-seconds 0 > $OUT/${v}_$rep.json 2>$OUT/err || { tail $OUT/err; exit 1; }
  python -c "import json; d=json.loads(open('$OUT/${v}_$rep.json').read().strip().splitlines()[-1]); r=d['roofline']; print('$v', d['ms_per_step'], r['avg_launch_ms'], r['frac'])"
done; done
