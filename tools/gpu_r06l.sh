#!/bin/bash
# Path-option migration: graph build + GAT pipe + lib tests, then the whole GPU suite.
set -uo pipefail
mkdir -p gpurun_out/r06l
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
  tests/test_gpu_graph_build.py tests/test_gpu_gat_pipe.py tests/test_lib.py \
  > gpurun_out/r06l/subset.log 2>&1 || { tail -30 gpurun_out/r06l/subset.log; exit 1; }
tail -3 gpurun_out/r06l/subset.log
timeout -k 10 900 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests \
  > gpurun_out/r06l/full.log 2>&1 || { tail -30 gpurun_out/r06l/full.log; exit 1; }
tail -3 gpurun_out/r06l/full.log
OPT=graph_sorted A=0 B=1 W="c2" STEPS=200 bash tools/gpu_ab.sh r06l/ab || exit 1
