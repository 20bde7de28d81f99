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


def cpu_stat():
    """The cgroup's CPU accounting (cgroup v2 cpu.stat: usage and throttling), {} if absent."""
    try:
        return {k: int(v) for k, v in (ln.split() for ln in open("/sys/fs/cgroup/cpu.stat"))}
    except OSError:
        return {}


try:
    print("cpu.max", open("/sys/fs/cgroup/cpu.max").read().strip(), "affinity", len(os.sched_getaffinity(0)),
          flush=True)
except OSError:
    pass
for T in [int(t) for t in os.environ.get("CL_PROBE_THREADS", "1,4,16").split(",")]:
    ctx = pkg.Context(0)
    ctx.set_points(x, y, w)
    prof = os.environ.get("CL_PROBE_PROFILE", "1") == "1"   # in-kernel stamps (as bench.py: off)
    ctx.profile(prof)
    ctx.profile_read(reset=True)
    c0 = cpu_stat()
    r = bench.closure_threads(ctx, C, (T,), seconds=0.5)
    c1 = cpu_stat()
    if c0 and c1:   # CPU-seconds per wall second (includes the probe's setup), throttled periods
        r["cgroup"] = {k: c1.get(k, 0) - c0.get(k, 0) for k in ("usage_usec", "nr_throttled", "throttled_usec")}
    k_ms, k_launches, k_cands, _ = ctx.profile_read(reset=True)
    ctx.profile(False)
    r["kernel_us_per_launch"] = k_ms / max(k_launches, 1) * 1e3
    r["candidates_per_launch"] = k_cands / max(k_launches, 1)
    print(T, json.dumps(r), flush=True)
    ctx.close()
