#!/bin/bash
# three-conv fused backward (in_proj gradient outside): GCN tests, configs, then bench lines
set -uo pipefail
OUT=gpurun_out/r06q
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu \
  tests/test_gpu_gcn.py tests/test_gpu_configs.py tests/test_gpu_ce_fused.py tests/test_gpu_compile.py \
  tests/test_gpu_golden.py tests/test_gpu_s3.py > $OUT/pytest.log 2>&1 || { grep -E "FAILED|Error|error" $OUT/pytest.log | head -20; tail -30 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
for w in sweep_gcn3 c2; do
  timeout -k 10 300 python bench.py --workload $w --steps 200 --warmup 30 --cpu-seconds 0 > $OUT/$w.json 2> $OUT/$w.err || { tail -20 $OUT/$w.err; exit 1; }
  python -c "import json; d=json.load(open('$OUT/$w.json')); print('$w', d['value'], d['ms_per_step'], d['roofline']['frac'], d['roofline']['kernel'][:60])"
done
