#!/bin/bash
# A/B of the in-tree library against another build of it (tools/_abl/liblgnn_<tag>.so), same box:
#   bash tools/ab_lib.sh <tag> [bench args...]
set -e
TAG=$1; shift
mkdir -p gpurun_out/ab
for rep in 1 2; do for v in intree $TAG; do
  if [ $v = intree ]; then LP=""; else LP=$GRAFT_REPO_ROOT/tools/_abl/liblgnn_$v.so; fi
  LGNN_LIB_PATH=$LP timeout -k 10 200 python bench.py --steps 300 --warmup 30 --cpu-seconds 0 "$@" > gpurun_out/ab/lib_$v.json
  python -c "import json; d=json.loads(open('gpurun_out/ab/lib_$v.json').read().strip().splitlines()[-1]); print('$v', d['ms_per_step'], d.get('roofline',{}).get('avg_launch_ms'))"
done; done
