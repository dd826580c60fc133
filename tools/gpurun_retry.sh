#!/bin/bash
# usage: gpurun_retry.sh LOG TIMEOUT CMD  -- retries only when no box/slot is free (rc 3)
LOG=$1; TO=$2; shift 2
for i in $(seq 1 30); do
  /usr/local/graft/bin/gpurun --timeout "$TO" -- "$@" > "$LOG" 2>&1
  rc=$?
  if [ $rc -ne 3 ] && ! grep -q "status=transient" "$LOG"; then break; fi
  sleep 420
done
echo "RC=$rc" >> "$LOG"
