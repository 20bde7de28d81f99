#!/bin/bash
# The closure under concurrent host threads (tools/closure_threads_probe.py) for several settings of
# the combiner (same box): MAXCOVER_CL_LEADERS (batches launched at once) x MAXCOVER_CL_READSPIN
# (pause-spins before a caller waiting for its slot yields its CPU) x MAXCOVER_CL_SPIN (pause-spins
# before a queued caller sleeps on its futex) x MAXCOVER_CL_LEAD (batches one thread launches in a row).
# Usage: tools/closure_sweep.sh [rounds] ["leaders readspin spin lead" ...]
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out/csw
R=${1:-2}; shift || true
CFGS=("$@"); [ ${#CFGS[@]} -eq 0 ] && CFGS=("2 64 64 1" "2 64 64 16" "1 64 64 16" "4 64 64 16")
for r in $(seq 1 "$R"); do
  for cfg in "${CFGS[@]}"; do
    set -- $cfg
    f=gpurun_out/csw/L$1.S$2.W$3.D$4.$r.log
    MAXCOVER_CL_LEADERS=$1 MAXCOVER_CL_READSPIN=$2 MAXCOVER_CL_SPIN=$3 MAXCOVER_CL_LEAD=$4 MAXCOVER_CL_STATS=1 \
      timeout -k 10 120 python tools/closure_threads_probe.py > $f 2>&1 || exit $?
    echo "== leaders $1 readspin $2 spin $3 lead $4 run $r"; grep -E "^[0-9]+ |closure |cpu.max" $f | sed 's/"mismatches.*vs_1_thread": [0-9.]*}//' | cut -c1-320
  done
done
