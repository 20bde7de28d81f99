#!/bin/bash
# Same-box A/B of the host-pointer poll's staging threads (MAXCOVER_STAGE_THREADS): bench.py's
# host_poll_ms (the 37.7-MB matrix from host memory, and the basis form), alternating.
set -u
cd "$(dirname "$0")/.."
for r in 1 2; do
  for t in 1 8 16; do
    MAXCOVER_STAGE_THREADS=$t timeout -k 10 300 python bench.py --no-cpu --steps 20 > gpurun_out/stage_ab.log 2>&1 || exit $?
    python3 - $t gpurun_out/stage_ab.log <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[2]) if l.startswith("{")][0])
h = d["host_poll_ms"]
print("threads", sys.argv[1], "matrix_ms %.3f" % h["matrix_ms"], "basis_ms %.3f" % h["basis_ms"], "agree", h["agree"])
PY
  done
done
