"""Probe: mac_area_f64 from 1 / 4 / 16 native host threads (bench.closure_threads) at config 4,
with the combined launches' kernel time (in-kernel stamps) beside the calls/s; run with
MAXCOVER_CL_STATS=1 for the batch sizes."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import __graft_entry__ as ge  # noqa: E402
import bench  # noqa: E402

pkg = ge.load_package()
x, y, w, C, rmax = pkg.workloads.make_config(4)
for T in (1, 4, 16):
    ctx = pkg.Context(0)
    ctx.set_points(x, y, w)
    ctx.profile(True)
    ctx.profile_read(reset=True)
    r = bench.closure_threads(ctx, C, (T,), seconds=0.5)
    k_ms, k_launches, k_cands, _ = ctx.profile_read(reset=True)
    ctx.profile(False)
    r["kernel_us_per_launch"] = k_ms / max(k_launches, 1) * 1e3
    r["candidates_per_launch"] = k_cands / max(k_launches, 1)
    print(T, json.dumps(r), flush=True)
    ctx.close()
