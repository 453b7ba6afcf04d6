#!/bin/bash
# A/B of one library path option on one box: bench.py --workload W with OPT=A, then OPT=B, twice
# each, interleaved. Usage: OPT=graph_sorted A=0 B=1 W="c2" bash tools/gpu_ab.sh <tag>
set -uo pipefail
TAG=$1
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
for w in $W; do
  for rep in 1 2; do
    for val in $A $B; do
      timeout -k 10 300 python bench.py --workload $w --steps ${STEPS:-200} --path-option "$OPT=$val" \
        --warmup 30 --cpu-seconds 0 > "$OUT/ab_${w}_${val}_$rep.json" 2> "$OUT/ab_${w}_${val}_$rep.err" \
        || { tail -20 "$OUT/ab_${w}_${val}_$rep.err"; exit 1; }
      python -c "
import json; d=json.load(open('$OUT/ab_${w}_${val}_$rep.json'))
print('$w $OPT=$val rep $rep', d['value'], d['ms_per_step'])"
    done
  done
done
