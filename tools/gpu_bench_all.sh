#!/bin/bash
# Every bench workload once (bounded CPU baselines), one JSON line each, into gpurun_out/<tag>/.
set -euo pipefail
TAG=$1; shift
OUT=$GRAFT_REPO_ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
for w in c2 c3 c3f32 c4 c5k4 c5k16; do
  timeout -k 10 300 python bench.py --workload $w --cpu-seconds ${CPU_SECONDS:-8} "$@" > "$OUT/bench_$w.json" 2> "$OUT/bench_$w.err" || { tail -20 "$OUT/bench_$w.err"; exit 1; }
  cut -c1-240 "$OUT/bench_$w.json"
done
