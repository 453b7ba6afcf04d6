#!/bin/bash
# One SQ-counter pass (stall / MFMA-busy / LDS) of a bench workload: bash tools/pmc_sq.sh <tag> <workload>
# COUNTERS="..." overrides the counter set (at most 8 SQ_ counters: one hardware pass); SUB names
# the output subdirectory.
set -uo pipefail
TAG=$1; W=$2
OUT=$GRAFT_REPO_ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
cd /tmp
SUB=${SUB:-sq}
CNT=${COUNTERS:-"SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE"}
timeout -s KILL 240 rocprofv3 --pmc $CNT \
  --output-format csv -d "$OUT/$SUB" -o sq -- \
  python3 "$GRAFT_REPO_ROOT/bench.py" --workload $W --steps 5 --warmup 2 --cpu-seconds 0 \
  --no-kernel-timing > /dev/null 2> "$OUT/$SUB.err" || { tail -20 "$OUT/$SUB.err"; exit 1; }
F=$(find "$OUT/$SUB" -name "*counter_collection.csv" | head -1)
python3 - "$F" <<'PY'
import csv, sys, collections
agg = collections.defaultdict(lambda: collections.defaultdict(list))
for r in csv.DictReader(open(sys.argv[1])):
    agg[r["Kernel_Name"]][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, cs in sorted(agg.items(), key=lambda kv: -max(sum(v) for v in kv[1].values()))[:14]:
    m = {c: sum(v) / len(v) for c, v in cs.items()}
    print(k[:60], " ".join(f"{c.replace('SQ_','')}={m[c]:.3g}" for c in sorted(m)))
PY
