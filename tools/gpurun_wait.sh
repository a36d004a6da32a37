#!/bin/bash
# Submit one gpurun call, waiting for a free GPU slot: resubmits ONLY while gpurun reports that
# nothing ran (status "transient" / exit 3: no slot or box free, nothing charged).  Any call
# that actually ran -- passed or failed -- ends the loop; a failed GPU step is never retried.
#   tools/gpurun_wait.sh LOG TIMEOUT 'command'
LOG=$1; TO=$2; CMD=$3
for i in $(seq 1 30); do
  /usr/local/graft/bin/gpurun --timeout "$TO" -- "$CMD" > "$LOG" 2>&1
  rc=$?
  if [ $rc -eq 3 ] || grep -q "status=transient" "$LOG"; then
    sleep 120
    continue
  fi
  exit $rc
done
exit 3
