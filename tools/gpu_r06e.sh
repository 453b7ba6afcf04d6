#!/bin/bash
# round-6 box 5: the sorted transpose (source CSR / tmap of target-sorted builds)
set -uo pipefail
OUT=gpurun_out/r06e
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_graph_build.py -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest_build.log 2>&1
rc=$?
tail -3 $OUT/pytest_build.log; grep -E "^FAILED|^ERROR|Error" $OUT/pytest_build.log | head
[ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1
rc=$?
tail -3 $OUT/pytest_gpu.log; grep -E "^FAILED|^ERROR" $OUT/pytest_gpu.log | head
[ $rc -eq 0 ] || exit $rc
WL="c2 c4 c5k16 c5k4 refcfg c3" bash tools/gpu_lines.sh r06e || exit 1
