#!/bin/bash
# Retry a gpurun call only while the pool has no free box (status "transient", nothing ran, nothing charged).
# usage: tools/gpurun_retry.sh LOG TIMEOUT 'command'
LOG=$1; TO=$2; shift 2
for i in $(seq 1 30); do
  /usr/local/graft/bin/gpurun --timeout $TO -- "$@" > $LOG 2>&1
  rc=$?
  if grep -q "status=transient" $LOG && grep -q "run 0.0s\|run Nones" $LOG; then sleep 90; continue; fi
  break
done
echo "rc=$rc tries=$i" >> $LOG
