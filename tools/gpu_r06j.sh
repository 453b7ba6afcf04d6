#!/bin/bash
# round-6 box: 8-head row-pipelined GAT kernels (HS = 2)
set -uo pipefail
OUT=gpurun_out/r06j
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_gat_pipe.py tests/test_gpu_gat.py -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1
rc=$?
tail -2 $OUT/pytest.log; grep -E "^FAILED|^ERROR|Error" $OUT/pytest.log | head -5
[ $rc -eq 0 ] || exit $rc
WL="sweep_gat128h8 refcfg c3" bash tools/gpu_lines.sh r06j || exit 1
