#!/bin/bash
# round-6 close, box 1: the GPU suite, smoke, and the BASELINE-config bench lines
set -uo pipefail
OUT=gpurun_out/r06z
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread \
  > $OUT/pytest_gpu.log 2>&1 || { grep -E "FAILED|Error" $OUT/pytest_gpu.log | head; tail -20 $OUT/pytest_gpu.log; exit 1; }
tail -1 $OUT/pytest_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $OUT/smoke.log 2>&1 \
  || { tail -20 $OUT/smoke.log; exit 1; }
tail -1 $OUT/smoke.log
WL="c2_driver_cmd c2 c2_dist c4 c4_dist c5k4 c5k16 refcfg" bash tools/gpu_lines.sh r06z || exit 1
