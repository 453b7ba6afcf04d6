#!/bin/bash
# r03b: re-run the tests changed after r03a, short benches of the GAT workloads, kernel-trace
# profiles of refcfg / c3f32 / c3 (rocprofv3 --kernel-trace --stats).
set -uo pipefail
OUT=gpurun_out/r03b
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_s3gemm.py tests/test_gpu_gat.py tests/test_gpu_gin.py \
  -m gpu -q --timeout 120 --timeout-method thread > "$OUT/pytest.log" 2>&1
rc=$?; tail -3 "$OUT/pytest.log"; grep -E "^FAILED" "$OUT/pytest.log" | head
case $rc in 0|1) ;; *) exit $rc;; esac
for w in refcfg c3f32 c3; do
  timeout -k 10 300 python bench.py --workload $w --steps 100 --warmup 20 --cpu-seconds 0 \
    --no-kernel-timing > "$OUT/bench_$w.json" 2> "$OUT/bench_$w.err" || { tail -20 "$OUT/bench_$w.err"; exit 1; }
  python -c "import json,sys; d=json.load(open('$OUT/bench_$w.json')); print('$w', d['value'], d['ms_per_step'])"
done
for w in refcfg c3f32; do
  ( cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$GRAFT_REPO_ROOT/$OUT/prof_$w/prof" -o trace -- \
    python3 "$GRAFT_REPO_ROOT/bench.py" --workload $w --steps 20 --warmup 5 --cpu-seconds 0 --no-kernel-timing \
    > "$GRAFT_REPO_ROOT/$OUT/prof_$w.json" 2> "$GRAFT_REPO_ROOT/$OUT/prof_$w.err" ) || { tail -20 "$OUT/prof_$w.err"; exit 1; }
  STATS=$(find "$OUT/prof_$w/prof" -name "*kernel_stats.csv" | head -1)
  python3 - "$STATS" <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: -float(r["TotalDurationNs"]))
for r in rows[:22]:
    print(f'{r["Name"][:80]:80s} {int(r["Calls"]):5d} {float(r["AverageNs"])/1e3:9.2f} us')
PY
done
exit $rc
