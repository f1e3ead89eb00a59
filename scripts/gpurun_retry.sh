#!/bin/bash
# Run one gpurun call, asking again only when the pool reports an infrastructure-side transient
# (no box / slot free, box lost while being prepared: nothing ran, nothing charged).  A command
# that ran on a box -- whatever its exit status -- is never repeated.
# usage: scripts/gpurun_retry.sh <timeout_s> <log> '<command>'
T=$1; LOG=$2; CMD=$3
for attempt in 1 2 3 4 5 6 7 8; do
  /usr/local/graft/bin/gpurun --timeout "$T" -- "$CMD" > "$LOG" 2>&1
  rc=$?
  if grep -q "status=transient\|taken away by the GPU service\|no free box\|are busy\|backing off" "$LOG" \
     && ! grep -q "run [1-9][0-9]*\.[0-9]*s of limit" "$LOG"; then
    echo "attempt $attempt: transient, waiting" >&2
    sleep $((60 * attempt))
    continue
  fi
  exit $rc
done
exit 3
