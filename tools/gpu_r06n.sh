#!/bin/bash
# Driver command after moving the diagnostics ahead of the warmup; c4 / refcfg lines still emit.
set -uo pipefail
mkdir -p gpurun_out/r06n
for i in 1 2; do
  timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r06n/c2_$i.json \
    2> gpurun_out/r06n/c2_$i.err || { tail -20 gpurun_out/r06n/c2_$i.err; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/r06n/c2_$i.json')); print('c2', d['value'], d['ms_per_step'], d['roofline']['frac'], d['roofline']['avg_launch_ms'])"
done
for w in c4 refcfg; do
  timeout -k 10 300 python bench.py --workload $w --steps 20 --warmup 5 --cpu-seconds 0 > gpurun_out/r06n/$w.json \
    2> gpurun_out/r06n/$w.err || { tail -20 gpurun_out/r06n/$w.err; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/r06n/$w.json')); print('$w', d['value'], d['ms_per_step'], d['roofline']['frac'])"
done
OPT=graph_sorted A=0 B=1 W="c5k16 c5k4 sweep_gcn_k16 sweep_gcn_k32" STEPS=100 bash tools/gpu_ab.sh r06n/ab || exit 1
