#!/bin/bash
# usage: gpurun_retry.sh <outfile> <timeout> <cmd>: retries only while gpurun reports no free slot/box (nothing ran, nothing charged)
out=$1; to=$2; cmd=$3
for i in $(seq 1 12); do
  /usr/local/graft/bin/gpurun --timeout $to -- "$cmd" > $out 2>&1
  rc=$?
  if grep -q "status=transient" $out; then sleep 150; continue; fi
  break
done
echo "[retry wrapper] attempts=$i rc=$rc" >> $out
