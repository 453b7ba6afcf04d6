#!/bin/bash
# tile spmm: CSR block staged in LDS up to 640 entries (new) vs not (v1): tests, kernel time, A/B
set -uo pipefail
OUT=gpurun_out/r06z6
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_wide.py tests/test_gpu_sweep_space.py tests/test_gpu_gin.py > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
export TMPDIR=/tmp
( cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$OUT/prof -o t -- python3 $GRAFT_REPO_ROOT/bench.py --workload sweep_gin512 --steps 10 --warmup 3 --cpu-seconds 0 --no-kernel-timing > /dev/null 2>&1 ) || exit 1
S=$(find $OUT/prof -name "*kernel_stats.csv" | head -1)
grep -i "spmm" $S | cut -d, -f1-4
for rep in 1 2; do for v in new v1; do
  if [ $v = new ]; then LP=""; else LP=$GRAFT_REPO_ROOT/tools/ab/liblgnn_v1.so; fi
  LGNN_LIB_PATH=$LP timeout -k 10 300 python bench.py --workload sweep_gin512 --steps 40 --warmup 10 --cpu-seconds 0 --entries 0 --no-kernel-timing > $OUT/gin512_${v}_$rep.json 2>$OUT/err || { tail $OUT/err; exit 1; }
  python -c "import json; d=json.loads(open('$OUT/gin512_${v}_$rep.json').read().strip().splitlines()[-1]); print('gin512 $v', d['ms_per_step'])"
done; done
