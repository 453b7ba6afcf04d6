#!/bin/bash
# One bench line per workload (default steps, CPU baseline leg included), the driver's own C2
# command, and the N > 1 plans at world 1. Usage: WL="c2 c4 ..." bash tools/gpu_lines.sh <tag>
set -uo pipefail
TAG=$1
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
run() {  # name, args...
  local n=$1; shift
  timeout -k 10 400 python bench.py "$@" > "$OUT/bench_$n.json" 2> "$OUT/bench_$n.err" \
    || { tail -20 "$OUT/bench_$n.err"; exit 1; }
  python -c "import json; d=json.loads(open('$OUT/bench_$n.json').read().strip().splitlines()[-1]); print('$n', d['value'], d['ms_per_step'], (d.get('roofline') or {}).get('frac'), (d.get('cpu_baseline') or {}).get('value'))"
}
for w in ${WL:-c2}; do
  case $w in
    c2_driver_cmd) run $w --gpus 1 --steps 20 --warmup 5 ;;
    c2_dist) run $w --workload c2 --force-dist ;;
    c4_dist) run $w --workload c4 --force-dist --sync-bn on ;;
    *) run $w --workload $w ;;
  esac
done
