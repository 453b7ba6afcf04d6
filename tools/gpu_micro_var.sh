#!/bin/bash
# split-3 GEMM micro timings of the in-tree library and every tools/_abl/liblgnn_v_*.so (timing
# ablations, tools/build_abl_s3g.sh), one box. Usage: bash tools/gpu_micro_var.sh <tag>
set -e
mkdir -p gpurun_out/micro
for v in intree $(cd tools/_abl && ls liblgnn_v_*.so 2>/dev/null); do
  if [ $v = intree ]; then LP=""; else LP=$GRAFT_REPO_ROOT/tools/_abl/$v; fi
  echo "== $v"
  PYTHONPATH=$GRAFT_REPO_ROOT LGNN_LIB_PATH=$LP timeout -k 10 120 python tools/s3_micro.py ${MICRO_ARGS:---wide} 2>&1 | grep -v amdgpu.ids
done > gpurun_out/micro/$1.txt 2>&1
cat gpurun_out/micro/$1.txt
