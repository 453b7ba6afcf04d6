#!/bin/bash
# One GPU iteration: selected pytest files (-m gpu), short benches of selected workloads, and
# kernel-trace profiles (rocprofv3 --kernel-trace --stats) of selected workloads.
# Usage: TESTS="tests/a.py tests/b.py" BENCH="c2 c3f32" PROF="refcfg" bash tools/gpu_iter.sh <tag>
set -uo pipefail
TAG=$1
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
if [ -n "${TESTS:-}" ]; then
  timeout -k 10 600 python -u -m pytest $TESTS -m gpu -q --timeout 120 --timeout-method thread \
    > "$OUT/pytest.log" 2>&1
  rc=$?; tail -2 "$OUT/pytest.log"; grep -E "^FAILED|^ERROR" "$OUT/pytest.log" | head -20
  case $rc in 0|1) ;; *) echo "pytest rc=$rc"; exit $rc;; esac
fi
for w in ${BENCH:-}; do
  timeout -k 10 300 python bench.py --workload $w --steps ${STEPS:-200} --warmup 30 --cpu-seconds 0 \
    > "$OUT/bench_$w.json" 2> "$OUT/bench_$w.err" || { tail -20 "$OUT/bench_$w.err"; exit 1; }
  python -c "
import json; d=json.load(open('$OUT/bench_$w.json')); r=d.get('roofline') or {}
print('$w', d['value'], d['ms_per_step'], r.get('kernel','')[:40], r.get('avg_launch_ms'), r.get('frac'))"
done
for w in ${PROF:-}; do
  ( cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv \
    -d "$GRAFT_REPO_ROOT/$OUT/prof_$w/prof" -o trace -- \
    python3 "$GRAFT_REPO_ROOT/bench.py" --workload $w --steps 20 --warmup 5 --cpu-seconds 0 \
    --no-kernel-timing > "$GRAFT_REPO_ROOT/$OUT/prof_$w.json" 2> "$GRAFT_REPO_ROOT/$OUT/prof_$w.err" ) \
    || { tail -20 "$OUT/prof_$w.err"; exit 1; }
  STATS=$(find "$OUT/prof_$w/prof" -name "*kernel_stats.csv" | head -1)
  echo "== $w"
  python3 - "$STATS" <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: -float(r["TotalDurationNs"]))
for r in rows[:int(__import__("os").environ.get("TOPK", "16"))]:
    print(f'{r["Name"][:72]:72s} {int(r["Calls"]):5d} {float(r["AverageNs"])/1e3:9.2f} us')
PY
done
exit ${rc:-0}
