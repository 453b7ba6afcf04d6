#!/bin/bash
# LDS-staged tile spmm: the wide-path tests, then a same-box A/B against the row kernel
set -uo pipefail
OUT=gpurun_out/r06z3
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_wide.py tests/test_gpu_gin.py tests/test_gpu_sweep_space.py tests/test_gpu_drgnet.py \
  tests/test_gpu_gcn.py > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
timeout -k 10 300 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_configs.py -k "gin512 or c4 or c2" > $OUT/pytest2.log 2>&1 || { tail -30 $OUT/pytest2.log; exit 1; }
tail -1 $OUT/pytest2.log
for rep in 1 2; do for v in tile rows; do
  if [ $v = tile ]; then LP=""; else LP=$GRAFT_REPO_ROOT/tools/ab/liblgnn_rows.so; fi
  LGNN_LIB_PATH=$LP timeout -k 10 300 python bench.py --workload sweep_gin512 --steps 40 --warmup 10 --cpu-seconds 0 --entries 0 --no-kernel-timing > $OUT/gin512_${v}_$rep.json 2>$OUT/err || { tail $OUT/err; exit 1; }
  python -c "import json; d=json.loads(open('$OUT/gin512_${v}_$rep.json').read().strip().splitlines()[-1]); print('gin512 $v', d['ms_per_step'])"
done; done
