#!/bin/bash
# Same-box A/B of two builds on the closure under 1/4/16 native threads (tools/closure_threads_probe.py,
# in-kernel stamps off), alternating. Usage: tools/closure_ab_lib.sh libA.so libB.so [rounds]
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out/clab
A=$1; B=$2; R=${3:-3}
for r in $(seq 1 "$R"); do
  for v in A B; do
    lib=$A; [ "$v" = B ] && lib=$B
    MAXCOVER_LIB=$lib CL_PROBE_PROFILE=0 timeout -k 10 120 python tools/closure_threads_probe.py > gpurun_out/clab/$v$r.log 2>&1 || exit $?
    python3 - "$v" gpurun_out/clab/$v$r.log <<'PY'
import json, sys
out = {}
for l in open(sys.argv[2]):
    if l[:1].isdigit() and "{" in l:
        t, js = l.split(" ", 1)
        d = json.loads(js)
        out[t] = round(d[t]["calls_per_s"] / 1e3, 1)
print(sys.argv[1], out, round(out["16"] / out["1"], 2))
PY
  done
done
