#!/bin/bash
# usage: gpuq.sh OUTFILE TIMEOUT 'command' -- retries only while gpurun reports
# that no slot/box was available (exit 3: nothing ran, nothing charged)
out=$1; to=$2; cmd=$3
for i in $(seq 1 30); do
  timeout $((to + 900)) /usr/local/graft/bin/gpurun --timeout $to -- "$cmd" > $out 2>&1
  rc=$?
  if [ $rc -ne 3 ]; then echo "rc=$rc attempt=$i" >> $out; exit $rc; fi
  sleep 90
done
echo "gave up" >> $out
