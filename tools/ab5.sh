#!/bin/bash
# Same-box A/B of two builds on the config-5 MPC loop (3 steps each, alternating).
# Usage: tools/ab5.sh libA.so libB.so [rounds]
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out/ab5
A=$1; B=$2; R=${3:-2}
for r in $(seq 1 "$R"); do
  for v in A B; do
    lib=$A; [ "$v" = B ] && lib=$B
    MAXCOVER_LIB=$lib timeout -k 10 200 python bench.py --config 5 --no-cpu > gpurun_out/ab5/$v$r.log 2>&1 || exit $?
    python3 - "$v" "gpurun_out/ab5/$v$r.log" <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[2]) if l.startswith("{")][0])
print(sys.argv[1], "ms_per_step %.2f" % d["ms_per_step"], "chain_us %.1f" % (d["roofline"]["chain_ms"] * 1e3),
      {k: round(v["avg_us"], 1) for k, v in d["roofline"]["kernels"].items()})
PY
  done
done
