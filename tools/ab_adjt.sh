#!/bin/bash
# A/B of the forward -> backward Â^T plane handover (LGNN_ADJT) on one box, C2 bench
set -e
mkdir -p gpurun_out/ab
for v in 1 0 1 0; do
  LGNN_ADJT=$v timeout -k 10 200 python bench.py --steps 300 --warmup 30 --cpu-seconds 0 > gpurun_out/ab/adjt_$v.json
  python -c "import json; d=json.loads(open('gpurun_out/ab/adjt_$v.json').read().strip().splitlines()[-1]); print('adjt=$v', d['ms_per_step'], d['roofline']['avg_launch_ms'], d['roofline_next'][0]['avg_launch_ms'])"
done
