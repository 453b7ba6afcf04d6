#!/bin/bash
# Kernel-trace stats + the two HBM PMC passes (separate runs) of one bench workload, laid out as
# tools/summarize_prof.py expects: bash tools/prof_pmc.sh <tag> [bench args...]
set -euo pipefail
TAG=$1; shift
OUT=$GRAFT_REPO_ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof" -o trace -- \
  python3 "$GRAFT_REPO_ROOT/bench.py" --steps 20 --warmup 5 --cpu-seconds 0 "$@" \
  > "$OUT/prof_bench.json" 2> "$OUT/prof.err" || { tail -20 "$OUT/prof.err"; exit 1; }
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 300 rocprofv3 --pmc $c --output-format csv -d "$OUT/pmc_$c" -o pmc -- \
    python3 "$GRAFT_REPO_ROOT/bench.py" --steps 5 --warmup 2 --cpu-seconds 0 "$@" \
    > /dev/null 2> "$OUT/pmc_$c.err" || { tail -20 "$OUT/pmc_$c.err"; exit 1; }
done
echo "prof + pmc done: $OUT"
