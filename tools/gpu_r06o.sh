#!/bin/bash
# C5 graph build alone under rocprofv3: target-sorted path on / off
set -uo pipefail
OUT=$GRAFT_REPO_ROOT/gpurun_out/r06o
mkdir -p $OUT
export TMPDIR=/tmp
cd /tmp
for cfg in "c5k16 gcn_lazy" "c5k4 gcn_lazy"; do
  set -- $cfg
  for v in 1 0; do
    timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/${1}_$v -o t -- python3 $GRAFT_REPO_ROOT/tools/build_probe.py $1 $2 20 $v > $OUT/${1}_$v.log 2>&1 || { tail $OUT/${1}_$v.log; exit 1; }
    S=$(find $OUT/${1}_$v -name "*kernel_stats.csv" | head -1)
    python3 - "$S" "$1 sorted=$v" <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
tot = 0
parts = []
for r in rows:
    n = r["Name"]
    if any(k in n for k in ("k_prep", "k_count", "k_scan", "k_fill", "k_finish", "k_tmap")):
        a = float(r["AverageNs"]) / 1e3
        tot += a
        parts.append(f'{n.split("::")[1].split("(")[0]} {a:.1f}')
print(sys.argv[2], f"sum {tot:.1f} us:", ", ".join(parts))
PY
  done
done
