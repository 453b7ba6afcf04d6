#!/bin/bash
# HBM PMC passes (FETCH_SIZE, WRITE_SIZE: separate runs) of tools/s3_micro.py --inproj.
set -euo pipefail
OUT=$GRAFT_REPO_ROOT/gpurun_out/$1
mkdir -p "$OUT"
export TMPDIR=/tmp PYTHONPATH=$GRAFT_REPO_ROOT
cd /tmp
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 120 rocprofv3 --pmc $c --output-format csv -d "$OUT/pmc_$c" -o pmc -- \
    python3 "$GRAFT_REPO_ROOT/tools/s3_micro.py" --inproj > "$OUT/micro_$c.txt" 2> "$OUT/pmc_$c.err"
done
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof" -o trace -- \
  python3 "$GRAFT_REPO_ROOT/tools/s3_micro.py" --inproj > "$OUT/micro.txt" 2> "$OUT/prof.err"
echo done
