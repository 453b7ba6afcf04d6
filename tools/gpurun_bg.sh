#!/bin/bash
# usage: tools/gpurun_bg.sh <outfile> <timeout> <cmd>: one gpurun call, repeated only while the
# pool reports an infrastructure-side transient (no box, box lost while being prepared, back-off);
# waits as long as the back-off message asks.
OUT=$1; TO=$2; CMD=$3
for i in $(seq 1 12); do
  timeout $((TO + 900)) /usr/local/graft/bin/gpurun --timeout $TO -- "$CMD" > $OUT 2>&1
  if grep -q "status=transient\|stopped responding while being prepared\|no free box\|backing off" $OUT && ! grep -q "rc=[0-9]" $OUT; then
    w=$(grep -o "retry in [0-9]*s" $OUT | grep -o "[0-9]*" | tail -1)
    sleep $(( ${w:-90} + 10 )); continue
  fi
  break
done
echo "__done__" >> $OUT
