#!/bin/bash
# gpurun that waits out pool-side transients (no slot / no box / box lost while being prepared:
# nothing ran, nothing charged), honouring gpurun's own back-off.  Any run that started is
# reported as is, never repeated.  Usage: tools/gpurun_retry.sh <outfile> <timeout> <command>
out=$1; to=$2; cmd=$3
for i in $(seq 1 40); do
  /usr/local/graft/bin/gpurun --timeout $to -- "$cmd" > $out 2>&1
  rc=$?
  if grep -q "status=transient" $out; then
    w=$(grep -o "retry in [0-9]*s" $out | grep -o "[0-9]*" | tail -1)
    sleep $(( ${w:-150} + 15 ))
    continue
  fi
  break
done
echo "[retry wrapper] attempts=$i rc=$rc" >> $out
