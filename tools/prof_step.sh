#!/bin/bash
# Kernel-trace profile of the default bench step (one GPU): rocprofv3 --kernel-trace --stats,
# summarised per kernel (tools/summarize_prof.py). Usage (GPU box, repo root):
#   bash tools/prof_step.sh <tag> [bench args...]     (env such as LGNN_BWD passes through)
set -euo pipefail
TAG=$1; shift
OUT=$GRAFT_REPO_ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof" -o trace -- \
  python3 "$GRAFT_REPO_ROOT/bench.py" --steps 20 --warmup 5 --cpu-seconds 0 "$@" \
  > "$OUT/bench.json" 2> "$OUT/prof.err" || { tail -20 "$OUT/prof.err"; exit 1; }
STATS=$(find "$OUT/prof" -name "*kernel_stats.csv" | head -1)
python3 - "$STATS" <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: -float(r["TotalDurationNs"]))
for r in rows[:28]:
    print(f'{r["Name"][:90]:90s} {int(r["Calls"]):5d} {float(r["AverageNs"])/1e3:9.2f} us')
PY
