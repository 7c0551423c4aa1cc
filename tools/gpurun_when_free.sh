#!/bin/bash
# Starts one gpurun call, retrying ONLY while gpurun answers 3 ("no box or slot free right now":
# nothing ran, nothing charged); any other outcome (the command ran, or was refused) ends it.
#   tools/gpurun_when_free.sh LOG TIMEOUT 'command'
LOG=$1; TO=$2; CMD=$3
for i in $(seq 1 30); do
  /usr/local/graft/bin/gpurun --timeout "$TO" -- "$CMD" > "$LOG" 2>&1
  rc=$?
  [ $rc -ne 3 ] && { echo "gpurun rc=$rc" >> "$LOG"; exit $rc; }
  sleep 90
done
