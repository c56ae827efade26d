#!/bin/bash
# Local helper (runs in the build container, never on the GPU box): submit one gpurun call and,
# while the pool answers "no slot / no box free" (exit 3, nothing charged), wait and submit it again.
# Any other outcome -- success, failure, refusal -- ends the loop.
#   tools/gpurun_retry.sh <timeout_s> '<command>' <log>
T=$1; CMD=$2; LOG=$3
for attempt in $(seq 1 20); do
    /usr/local/graft/bin/gpurun --timeout "$T" -- "$CMD" > "$LOG" 2>&1
    rc=$?
    if [ $rc -ne 3 ] && ! grep -q "status=transient" "$LOG"; then exit $rc; fi
    echo "attempt $attempt: no slot, waiting" >> "$LOG.retries"
    sleep 120
done
exit 3
