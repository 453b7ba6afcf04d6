#!/bin/bash
# A/B on one box: refcfg with the graph-breaking dropout scale (old) vs the plain-Python one (new)
set -uo pipefail
OUT=gpurun_out/r06u
mkdir -p $OUT
for rep in 1 2; do for v in new old; do
  if [ $v = new ]; then S=bench.py; else S=tools/ab_item_break.py; fi
  timeout -k 10 300 python $S --workload refcfg --cpu-seconds 0 --entries 0 > $OUT/${v}_$rep.json 2> $OUT/${v}_$rep.err || { tail -20 $OUT/${v}_$rep.err; exit 1; }
  python -c "import json; d=json.loads(open('$OUT/${v}_$rep.json').read().strip().splitlines()[-1]); print('$v', d['ms_per_step'], d['value'])"
  grep -c "Graph break" $OUT/${v}_$rep.err || true
done; done
