#!/bin/bash
# round-6 box 4: closed tiles up to 2048 CSR entries (k <= 32 at 64 nodes)
set -uo pipefail
OUT=gpurun_out/r06d
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_gcn.py tests/test_gpu_graph_build.py tests/test_gpu_configs.py tests/test_gpu_s3.py tests/test_gpu_ce_fused.py -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1
rc=$?
tail -3 $OUT/pytest_gpu.log; grep -E "^FAILED|^ERROR" $OUT/pytest_gpu.log | head
[ $rc -eq 0 ] || exit $rc
WL="sweep_gcn_k32 sweep_gcn_k16 c2" bash tools/gpu_lines.sh r06d || exit 1
