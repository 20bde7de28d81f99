#!/bin/bash
# Same-box A/B of two builds: config-4 bench (ms per poll, chain) and the host enqueue time of one
# device poll (tools/host_overhead.py), alternating.
set -u
cd "$(dirname "$0")/.."
A=$1; B=$2; R=${3:-3}
tools/ab.sh "$A" "$B" "$R" || exit $?
for r in $(seq 1 "$R"); do
  for v in A B; do
    lib=$A; [ "$v" = B ] && lib=$B
    echo -n "$v host: "; MAXCOVER_LIB=$lib timeout -k 10 120 python tools/host_overhead.py 2>/dev/null | grep '^{' || exit 1
  done
done
