#!/bin/bash
# gpurun with retries while no box / slot is free (exit 3: nothing ran, nothing charged); any other
# exit ends it.  usage: tools/gpurun_retry.sh LOG TIMEOUT 'command'
LOG=$1; T=$2; shift 2
for i in $(seq 1 20); do
  /usr/local/graft/bin/gpurun --timeout "$T" -- "$@" > "$LOG" 2>&1
  rc=$?
  [ $rc -eq 3 ] || exit $rc
  grep -q "status=transient" "$LOG" || exit $rc
  sleep 120
done
exit 3
