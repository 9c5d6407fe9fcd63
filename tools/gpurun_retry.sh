#!/bin/bash
# gpurun with retries only while the pool has no free slot / box (nothing
# charged, nothing ran); any other outcome ends it.  usage:
#   tools/gpurun_retry.sh LOG TIMEOUT 'command'
LOG=$1; TO=$2; shift 2
for i in $(seq 1 30); do
  /usr/local/graft/bin/gpurun --timeout "$TO" -- "$@" > "$LOG" 2>&1
  rc=$?
  if grep -q "status=transient" "$LOG" && ! grep -q "charged=[1-9]" "$LOG"; then
    sleep 90
    continue
  fi
  exit $rc
done
exit 3
