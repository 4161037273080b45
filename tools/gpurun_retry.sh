#!/bin/bash
# Resubmit a gpurun call only while the pool reports a transient provisioning failure (nothing ran).
# usage: tools/gpurun_retry.sh LOG TIMEOUT 'command'
LOG=$1; TO=$2; CMD=$3
for i in 1 2 3 4 5 6 7 8; do
  /usr/local/graft/bin/gpurun --timeout "$TO" -- "$CMD" > "$LOG" 2>&1
  if grep -q "status=transient" "$LOG" && grep -q "run 0.0s\|run Nones" "$LOG"; then
    echo "attempt $i transient: $(grep -o 'the [a-zA-Z ]*' "$LOG" | head -1)" >> "$LOG.attempts"
    sleep 200
    continue
  fi
  break
done
