#!/bin/bash
# Same-box A/B of one libmaxcover build under two environment settings on the config-4 poll:
# alternating runs of bench.py (no CPU baseline, no extras), each run's chain, kernels and ms per poll.
# Usage: tools/ab_env.sh 'VAR=a' 'VAR=b' [rounds] [extra bench args]
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out/abe
A=$1; B=$2; R=${3:-3}; shift 3; EXTRA="$*"
for r in $(seq 1 "$R"); do
  for v in A B; do
    e=$A; [ "$v" = B ] && e=$B
    env $e timeout -k 10 120 python bench.py --no-cpu --no-extras --steps 100 $EXTRA > gpurun_out/abe/$v$r.log 2>&1 || exit $?
    python3 - "$v $e" "gpurun_out/abe/$v$r.log" <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[2]) if l.startswith("{")][0])
print(sys.argv[1], "chain_us %.1f" % (d["roofline"]["chain_ms"] * 1e3), "ms_per_poll %.4f" % d["ms_per_step"],
      {k: round(v["avg_us"], 1) for k, v in d["roofline"]["kernels"].items()})
PY
  done
done
