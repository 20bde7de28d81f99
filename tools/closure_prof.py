"""The single-candidate closure path (mac_area_f64, src/TDM_STATIC_opt.jl:125: one objective call
per trial point) at config 4: host-side latency per call, for rocprofv3 --kernel-trace --stats.
    python tools/closure_prof.py [--calls 200]"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import __graft_entry__ as ge  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--calls", type=int, default=200)
ap.add_argument("--config", type=int, default=4)
a = ap.parse_args()
pkg = ge.load_package()
x, y, w, C, rmax = pkg.workloads.make_config(a.config)
ctx = pkg.Context(0)
ctx.set_points(x, y, w)
c0 = C[1].copy()
for _ in range(20):
    ctx.area(c0)
t = time.perf_counter()
for _ in range(a.calls):
    v = ctx.area(c0)
dt = (time.perf_counter() - t) / a.calls
t = time.perf_counter()
for _ in range(a.calls):
    o = ctx.poll_best(C[:1], rmax)
dt2 = (time.perf_counter() - t) / a.calls
print(json.dumps({"mac_area_f64_us": dt * 1e6, "mac_poll_best_f64_K1_us": dt2 * 1e6, "area": v}))
