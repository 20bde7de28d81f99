#!/bin/bash
# Same-box A/B of the closure under concurrent host threads (tools/closure_threads_probe.py):
# alternating runs of two libmaxcover builds, calls/s at 1, 4 and 16 native threads.
# Usage: tools/closure_ab.sh path/to/libA.so path/to/libB.so [rounds]
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out/cab
A=$1; B=$2; R=${3:-2}
for r in $(seq 1 "$R"); do
  for v in A B; do
    lib=$A; [ "$v" = B ] && lib=$B
    MAXCOVER_CL_STATS=1 MAXCOVER_LIB=$lib timeout -k 10 120 python tools/closure_threads_probe.py > gpurun_out/cab/$v$r.log 2>&1 || exit $?
    echo "== $v$r"; grep -E "^[0-9]+ |closure batches" gpurun_out/cab/$v$r.log | cut -c1-260
  done
done
