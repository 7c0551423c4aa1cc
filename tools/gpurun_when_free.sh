#!/bin/bash
# Retry a gpurun call while the pool has no free box (gpurun exit 3: nothing ran, nothing was
# charged); any other outcome -- success, a failure of the command, a refusal -- ends it.
#   tools/gpurun_when_free.sh LOG TIMEOUT 'command'
LOG=$1; TO=$2; CMD=$3
for i in $(seq 1 40); do
  /usr/local/graft/bin/gpurun --timeout "$TO" -- "$CMD" > "$LOG" 2>&1
  rc=$?
  if [ $rc -ne 3 ] && ! grep -q "status=transient" "$LOG"; then exit $rc; fi
  sleep 90
done
exit 3
