#!/bin/bash
# SQ / TA counter passes (one rocprofv3 --pmc run each) of tools/s3_micro.py --inproj:
#   bash tools/pmc_sq_micro.sh <tag>  -> gpurun_out/<tag>/pmc_<n>/ + a per-kernel summary
set -euo pipefail
OUT=$GRAFT_REPO_ROOT/gpurun_out/$1
mkdir -p "$OUT"
export TMPDIR=/tmp PYTHONPATH=$GRAFT_REPO_ROOT
cd /tmp
n=0
for set in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VMEM SQ_INSTS_LDS" \
           "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_VALU SQ_INSTS_MFMA SQ_WAVES TA_BUSY_avr TA_TA_BUSY_sum" \
           "FETCH_SIZE"; do
  n=$((n+1))
  timeout -s KILL 90 rocprofv3 --pmc $set --output-format csv -d "$OUT/pmc_$n" -o pmc -- \
    python3 "$GRAFT_REPO_ROOT/tools/s3_micro.py" --inproj > "$OUT/micro_$n.txt" 2> "$OUT/pmc_$n.err"
done
python3 - "$OUT" <<'PY'
import csv, glob, sys, collections
out = sys.argv[1]
agg = collections.defaultdict(lambda: collections.defaultdict(list))
for f in glob.glob(out + "/pmc_*/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        agg[r["Kernel_Name"][:60]][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, d in agg.items():
    print(k)
    for c, v in sorted(d.items()):
        print(f"   {c:28s} {sum(v)/len(v):.4g}  (n={len(v)})")
PY
