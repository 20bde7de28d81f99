#!/bin/bash
# The closure under concurrent host threads (tools/closure_threads_probe.py) for several settings of
# the combiner (same box): MAXCOVER_CL_LEADERS (batches launched at once) x MAXCOVER_CL_READSPIN
# (pause-spins before a waiting caller yields its CPU).
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out/csw
for r in 1 2; do
  for cfg in "2 64" "2 100000000" "4 64" "2 0"; do
    set -- $cfg
    MAXCOVER_CL_LEADERS=$1 MAXCOVER_CL_READSPIN=$2 MAXCOVER_CL_STATS=1 timeout -k 10 120 python tools/closure_threads_probe.py > gpurun_out/csw/L$1.S$2.$r.log 2>&1 || exit $?
    echo "== leaders $1 readspin $2 run $r"; grep -E "^[0-9]+ |closure batches" gpurun_out/csw/L$1.S$2.$r.log | sed 's/"mismatches.*vs_1_thread": [0-9.]*}//' | cut -c1-200
  done
done
