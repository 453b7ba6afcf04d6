#!/bin/bash
# Kernel-trace stats + separate FETCH_SIZE / WRITE_SIZE PMC passes of several workloads.
# Usage: WL="c2 c3 refcfg" bash tools/gpu_profset.sh <tag>
set -uo pipefail
TAG=$1
for w in ${WL:-c2}; do
  TAGW=${TAG}_$w
  bash tools/prof_pmc.sh $TAGW --workload $w --no-kernel-timing || exit 1
done
echo done
