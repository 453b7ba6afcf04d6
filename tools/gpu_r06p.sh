#!/bin/bash
# entry-parallel k_finish: graph-build + config parity, then the build kernels alone
set -uo pipefail
OUT=$GRAFT_REPO_ROOT/gpurun_out/r06p
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
  tests/test_gpu_graph_build.py tests/test_gpu_configs.py tests/test_gpu_gat.py tests/test_gpu_gin.py tests/test_gpu_golden.py tests/test_gpu_gcn.py \
  > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
export TMPDIR=/tmp
cd /tmp
for cfg in "c5k16 gcn_lazy 1" "c5k16 gcn_lazy 0" "c5k4 gcn_lazy 1" "c4 gin 1" "refcfg gat 1"; do
  set -- $cfg
  timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/${1}_$3 -o t -- python3 $GRAFT_REPO_ROOT/tools/build_probe.py $1 $2 20 $3 > $OUT/${1}_$3.log 2>&1 || { tail $OUT/${1}_$3.log; exit 1; }
  S=$(find $OUT/${1}_$3 -name "*kernel_stats.csv" | head -1)
  python3 - "$S" "$1 sorted=$3" <<'PY'
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
