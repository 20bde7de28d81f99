#!/bin/bash
# Run one gpurun call; when the infrastructure reports a transient failure (nothing ran, nothing
# charged) wait and submit the same call again, at most 3 times. A call that ran is never repeated.
# Usage: tools/gpurun_retry.sh LOGFILE TIMEOUT 'command'
log=$1; to=$2; shift 2
for a in 1 2 3; do
    /usr/local/graft/bin/gpurun --timeout "$to" -- "$@" > "$log" 2>&1
    grep -q "status=transient" "$log" || exit 0
    sleep 60
done
