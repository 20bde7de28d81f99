#!/bin/bash
# Same-box A/B of two builds of libmaxcover on the config-4 poll: alternates A and B runs of
# bench.py (no CPU baseline, no extras) and prints each run's chain and ms per poll.
# Usage: tools/ab.sh path/to/libA.so path/to/libB.so [rounds]
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out/ab
A=$1; B=$2; R=${3:-3}
for r in $(seq 1 "$R"); do
  for v in A B; do
    lib=$A; [ "$v" = B ] && lib=$B
    MAXCOVER_LIB=$lib timeout -k 10 120 python bench.py --no-cpu --no-extras --steps 40 > gpurun_out/ab/$v$r.log 2>&1 || exit $?
    python3 - "$v" "gpurun_out/ab/$v$r.log" <<'PY'
import json, sys
line = [l for l in open(sys.argv[2]) if l.startswith("{")][0]
d = json.loads(line)
print(sys.argv[1], "chain_us %.1f" % (d["roofline"]["chain_ms"] * 1e3), "ms_per_poll %.4f" % d["ms_per_step"],
      {k: round(v * 1e3, 1) for k, v in d["roofline"]["split_ms_per_poll"].items()})
PY
  done
done
