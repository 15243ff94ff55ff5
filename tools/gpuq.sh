#!/bin/bash
# retry a gpurun call only while the pool has no free slot/box (status=transient: nothing ran, nothing charged)
# usage: gpuq.sh OUTFILE TIMEOUT 'command'
OUT=$1; TO=$2; CMD=$3
for i in $(seq 1 30); do
  timeout $((TO + 900)) /usr/local/graft/bin/gpurun --timeout $TO -- "$CMD" > $OUT 2>&1
  if grep -q "status=transient" $OUT && ! grep -q "status=ok" $OUT; then sleep 150; continue; fi
  break
done
echo "gpuq done after $i attempt(s)" >> $OUT
