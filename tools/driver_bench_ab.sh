#!/bin/bash
# The driver's bench command (python3 bench.py --gpus 1 --steps 20 --warmup 5) beside the default
# run (200 timed polls after 20 warmup, no extras), alternating on one box: ms per poll and chain.
set -u
cd "$(dirname "$0")/.."
for r in 1 2 3; do
  timeout -k 10 200 python3 bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/drv$r.log 2>&1 || exit $?
  python3 - gpurun_out/drv$r.log <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[1]) if l.startswith("{")][0])
print("steps20", round(d["ms_per_step"], 4), round(d["roofline"]["chain_ms"] * 1e3, 1), d.get("check_timed_poll_vs_scan"))
PY
  timeout -k 10 200 python3 bench.py --no-cpu --no-extras > gpurun_out/drvd$r.log 2>&1 || exit $?
  python3 - gpurun_out/drvd$r.log <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[1]) if l.startswith("{")][0])
print("default", round(d["ms_per_step"], 4), round(d["roofline"]["chain_ms"] * 1e3, 1), d["steps"], d["warmup"])
PY
done
