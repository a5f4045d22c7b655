#!/bin/bash
# Re-submit a gpurun call only when the pool reports a transient infrastructure failure
# (box not prepared: nothing ran, nothing charged).  Any result from the command itself
# (pass or fail) ends the loop.  Usage: tools/gpurun_retry.sh LOG TIMEOUT 'command'
LOG=$1; TMO=$2; CMD=$3
for attempt in 1 2 3 4 5 6; do
  /usr/local/graft/bin/gpurun --timeout "$TMO" -- "$CMD" > "$LOG" 2>&1
  if grep -q "status=transient\|backing off" "$LOG"; then
    echo "[retry] transient attempt $attempt" >> "$LOG.retries"; sleep 30; continue
  fi
  break
done
