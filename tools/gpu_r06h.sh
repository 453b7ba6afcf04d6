#!/bin/bash
set -uo pipefail
OUT=gpurun_out/r06h
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_graph_build.py -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest_build.log 2>&1
rc=$?
tail -2 $OUT/pytest_build.log; grep -E "^FAILED|^ERROR|Error" $OUT/pytest_build.log | head -5
[ $rc -eq 0 ] || exit $rc
sed -i 's/for v in new nowin prev/for v in new prev/; s#r06g#r06h#' tools/gpu_r06g.sh
bash tools/gpu_r06g.sh
