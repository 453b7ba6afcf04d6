#!/bin/bash
# round-6 box 6: graph-build kernels, sorted transpose vs the previous library (rocprof, c5k16 / c4)
set -uo pipefail
OUT=gpurun_out/r06f
mkdir -p $OUT
export TMPDIR=/tmp
for wl in c5k16 c4; do
  bash tools/prof_step.sh r06f/new_$wl --workload $wl > $OUT/new_$wl.txt 2>&1 || { cat $OUT/new_$wl.txt; exit 1; }
  LGNN_LIB_PATH=$GRAFT_REPO_ROOT/tools/_abl/liblgnn_prev.so bash tools/prof_step.sh r06f/prev_$wl --workload $wl > $OUT/prev_$wl.txt 2>&1 || { cat $OUT/prev_$wl.txt; exit 1; }
  echo "== $wl new"; grep -E "k_finish|k_scan|k_fill|k_count|k_prep|k_tmap" $OUT/new_$wl.txt
  echo "== $wl prev"; grep -E "k_finish|k_scan|k_fill|k_count|k_prep|k_tmap" $OUT/prev_$wl.txt
done
