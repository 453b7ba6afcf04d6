#!/bin/bash
# round-6 box 3: the GPU suite (sweep parity at 1024 graphs, C2 criterion at 1024), sweep lines
# with their rooflines, GIN-512 kernel trace + PMC passes
set -uo pipefail
OUT=gpurun_out/r06c
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1
rc=$?
tail -3 $OUT/pytest_gpu.log; grep -E "^FAILED|^ERROR" $OUT/pytest_gpu.log | head
[ $rc -eq 0 ] || exit $rc
WL="sweep_gcn3 sweep_gin512 sweep_gat128h8 sweep_gcn_k16 sweep_gcn_k32" bash tools/gpu_lines.sh r06c || exit 1
bash tools/prof_pmc.sh r06c/gin512 --workload sweep_gin512 || exit 1
