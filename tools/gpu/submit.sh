#!/bin/bash
# submit one gpurun call; when no box / slot is free (gpurun exit 3: nothing ran, nothing charged) wait and submit
# it again, at most 12 times.  Any other outcome (success, failure, refusal) is final.
# usage: tools/gpu/submit.sh LOG TIMEOUT 'command'
LOG=$1; T=$2; shift 2
for i in $(seq 1 12); do
  /usr/local/graft/bin/gpurun --timeout "$T" -- "$@" > "$LOG" 2>&1
  rc=$?
  if [ $rc -ne 3 ] && ! grep -q "status=transient" "$LOG"; then echo "rc=$rc" >> "$LOG"; exit $rc; fi
  sleep 120
done
echo "gave up after 12 transient attempts" >> "$LOG"
exit 3
