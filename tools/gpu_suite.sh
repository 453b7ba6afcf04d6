#!/bin/bash
# GPU-box session: the whole -m gpu suite (not stopping at the first failure, each test under
# its own time limit), smoke(), and one default bench line.
# Usage (from the repo root, on the GPU box): bash tools/gpu_suite.sh <tag> [pytest selection...]
set -uo pipefail
TAG=${1:-run}; shift || true
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
SEL=${*:-tests}
timeout -k 10 900 python -u -m pytest $SEL -m gpu -v --timeout 120 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1
rc=$?
tail -3 "$OUT/pytest_gpu.log"
grep -E "^FAILED|^ERROR" "$OUT/pytest_gpu.log" | head -30
case $rc in 0|1) ;; *) echo "pytest rc=$rc: stopping"; exit $rc;; esac
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 || { cat "$OUT/smoke.log"; exit 1; }
tail -1 "$OUT/smoke.log"
timeout -k 10 600 python bench.py > "$OUT/bench.json" 2> "$OUT/bench.err" || { tail -30 "$OUT/bench.err"; exit 1; }
cat "$OUT/bench.json"
exit $rc
