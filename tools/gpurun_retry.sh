#!/bin/bash
# Run one gpurun call, retrying only while the pool has no free box (exit 3: nothing ran, nothing
# charged), at most 8 times, 2 minutes apart. Usage: bash tools/gpurun_retry.sh <log> <timeout> <cmd>
LOG=$1; TO=$2; CMD=$3
for i in 1 2 3 4 5 6 7 8; do
  /usr/local/graft/bin/gpurun --timeout "$TO" -- "$CMD" > "$LOG" 2>&1
  rc=$?
  grep -q "no free box\|slot(s) on this pod are busy\|backing off" "$LOG" || exit $rc
  sleep 120
done
exit $rc
