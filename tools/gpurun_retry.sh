#!/bin/bash
# gpurun with retries only while the pool has no free slot / box (nothing
# charged, nothing ran); any other outcome ends it.  Waits as long as gpurun
# asks ("retry in Ns"), at least 90 s.  usage:
#   tools/gpurun_retry.sh LOG TIMEOUT 'command'
LOG=$1; TO=$2; shift 2
for i in $(seq 1 40); do
  /usr/local/graft/bin/gpurun --timeout "$TO" -- "$@" > "$LOG" 2>&1
  rc=$?
  if grep -q "status=transient" "$LOG" && ! grep -q "charged=[1-9]" "$LOG"; then
    w=$(grep -o "retry in [0-9]*s" "$LOG" | grep -o "[0-9]*" | tail -1)
    [ -z "$w" ] || [ "$w" -lt 90 ] && w=90
    sleep "$w"
    continue
  fi
  exit $rc
done
exit 3
