#!/bin/bash
# Retry a gpurun call while the service reports a transient infrastructure
# failure (box not ready / taken away: status=transient, nothing charged).
# Never retries a command that ran and failed.  Usage: tools/run_cmd_retry.sh <log> <timeout> <cmd>
LOG=$1; T=$2; shift 2
for i in 1 2 3 4 5 6; do
  timeout $((T + 900)) /usr/local/graft/bin/gpurun --timeout "$T" -- "$@" > "$LOG" 2>&1
  if grep -q "status=transient\|backing off" "$LOG"; then sleep 45; continue; fi
  break
done
