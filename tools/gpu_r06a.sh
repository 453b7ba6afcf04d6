#!/bin/bash
# round-6 first box: launch-cost probe, driver-command C2 line, C2 step under rocprofv3
set -uo pipefail
OUT=gpurun_out/r06a
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python -u tools/launch_cost.py > $OUT/launch_cost.txt 2>&1 || { tail -20 $OUT/launch_cost.txt; exit 1; }
cat $OUT/launch_cost.txt
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/bench_c2_drv.json 2> $OUT/bench_c2_drv.err || { tail -20 $OUT/bench_c2_drv.err; exit 1; }
python -c "import json; d=json.loads(open('$OUT/bench_c2_drv.json').read().strip().splitlines()[-1]); print('c2drv', d['value'], d['ms_per_step'], d['roofline']['frac'])"
bash tools/prof_step.sh r06a/prof_c2 || exit 1
