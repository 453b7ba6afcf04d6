#!/bin/bash
# split-3 GEMM micro A/B on one box: the in-tree library against tools/_abl/liblgnn_s3f_base.so,
# twice each, interleaved (tools/s3_micro.py --wide). Usage: bash tools/gpu_micro_ab.sh <tag>
set -e
mkdir -p gpurun_out/micro
for rep in 1 2; do for v in new base; do
  if [ $v = new ]; then LP=""; else LP=$GRAFT_REPO_ROOT/tools/_abl/liblgnn_s3f_base.so; fi
  echo "== $v rep $rep"
  LGNN_LIB_PATH=$LP PYTHONPATH=$GRAFT_REPO_ROOT timeout -k 10 120 python tools/s3_micro.py --wide
done; done > gpurun_out/micro/$1.txt 2>&1
cat gpurun_out/micro/$1.txt
