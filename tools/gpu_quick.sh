#!/bin/bash
# Quick GPU iteration: parity tests, one bench line, kernel-trace profile summary.
# Usage (on the GPU box, from the repo root): bash tools/gpu_quick.sh <tag> [bench args...]
set -euo pipefail
TAG=$1; shift
OUT=$GRAFT_REPO_ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1 || { tail -40 "$OUT/pytest_gpu.log"; exit 1; }
tail -1 "$OUT/pytest_gpu.log"
timeout -k 10 300 python bench.py --cpu-seconds 0 "$@" | tee "$OUT/bench.json"
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof" -o trace -- \
  python "$GRAFT_REPO_ROOT/bench.py" --steps 20 --warmup 5 --cpu-seconds 0 "$@" > /dev/null 2> "$OUT/prof.err" || { tail -20 "$OUT/prof.err"; exit 1; }
echo done
