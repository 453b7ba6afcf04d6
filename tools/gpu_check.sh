#!/bin/bash
# One GPU-box session: parity tests, smoke, bench, rocprofv3 kernel stats (+ optional PMC passes).
# Usage (from the repo root, on the GPU box): bash tools/gpu_check.sh [tag] [pmc]
# Every GPU step has its own time limit; the first failure ends the script.
set -euo pipefail
TAG=${1:-run}
PMC=${2:-}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
echo "== pytest -m gpu"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1 || { tail -40 "$OUT/pytest_gpu.log"; exit 1; }
tail -3 "$OUT/pytest_gpu.log"
echo "== smoke"
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 || { cat "$OUT/smoke.log"; exit 1; }
cat "$OUT/smoke.log"
echo "== bench"
timeout -k 10 600 python bench.py > "$OUT/bench.json" 2> "$OUT/bench.err" || { tail -30 "$OUT/bench.err"; exit 1; }
cat "$OUT/bench.json"
echo "== rocprofv3 kernel trace"
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof" -o trace -- \
  python bench.py --steps 20 --warmup 5 --cpu-seconds 0 > "$OUT/prof_bench.json" 2> "$OUT/prof.err" || { tail -30 "$OUT/prof.err"; exit 1; }
find "$OUT/prof" -name '*kernel_stats.csv' | head -n 3 || true
if [ -n "$PMC" ]; then
  for c in FETCH_SIZE WRITE_SIZE; do
    echo "== rocprofv3 --pmc $c"
    timeout -k 10 600 rocprofv3 --pmc $c --output-format csv -d "$OUT/pmc_$c" -o pmc -- \
      python bench.py --steps 5 --warmup 2 --cpu-seconds 0 > /dev/null 2> "$OUT/pmc_$c.err" || { tail -30 "$OUT/pmc_$c.err"; exit 1; }
  done
fi
echo "== done"
