#!/bin/bash
# Final measurements of a round: kernel-trace + HBM PMC passes for the bench workloads, then one bench
# line per workload (with the CPU baseline leg). Usage: bash tools/gpu_final.sh <tag>
set -uo pipefail
TAG=$1
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
for w in ${WL:-c2 refcfg c3 c3f32}; do
  bash tools/prof_pmc.sh ${TAG}_$w --workload $w --no-kernel-timing || exit 1
done
for w in ${BW:-c2 refcfg c3 c3f32 c4 c5k4 c5k16}; do
  timeout -k 10 400 python bench.py --workload $w > "$OUT/bench_$w.json" 2> "$OUT/bench_$w.err" \
    || { tail -20 "$OUT/bench_$w.err"; exit 1; }
  python -c "import json; d=json.load(open('$OUT/bench_$w.json')); print('$w', d['value'], d['ms_per_step'], (d.get('cpu_baseline') or {}).get('value'))"
done
