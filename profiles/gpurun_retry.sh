#!/bin/bash
# usage: gpurun_retry.sh LOG TIMEOUT CMD  -- retries only when no box/slot is free (status=transient), every 240 s
LOG=$1; TO=$2; CMD=$3
for i in $(seq 1 20); do
  /usr/local/graft/bin/gpurun --timeout $TO -- "$CMD" > $LOG 2>&1
  rc=$?
  if grep -q "status=transient" $LOG; then echo "[retry $i: no box]" >> $LOG.retries; sleep 240; continue; fi
  break
done
echo "done rc=$rc" >> $LOG
