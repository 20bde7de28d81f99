"""Native MADS driver (mac_mads_run) on a config: evaluations per second of the whole loop,
host round trip per iteration included (every poll depends on the previous one)."""
import argparse
import json
import math
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import __graft_entry__ as ge  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", type=int, default=4)
    ap.add_argument("--iters", type=int, default=30)
    a = ap.parse_args()
    pkg = ge.load_package()
    wl = pkg.workloads
    cfg = wl.CONFIGS[a.config]
    x, y, w = wl.grid_points(cfg["G"])
    rng = wl.SplitMix64(wl.SEED)
    x0 = wl.uniform_disks(cfg["N"], cfg["G"], rng)
    N = cfg["N"]
    r_max = np.full(N, 30.0 * math.tan(100 / 180 * math.pi / 2))
    ctx = pkg.Context(0)
    ctx.set_points(x, y, w)
    ctx.mads_run(x0, r_max, n_iter=2, ell0=2, ell_max=6)        # warm-up (allocations)
    xo, st = ctx.mads_run(x0, r_max, prev=x0, d_lim=np.full(N, 10.0),
                          tan_half_fov=math.tan(100 / 180 * math.pi / 2), n_iter=a.iters,
                          ell0=2, ell_max=6)
    st["evals_per_s"] = st["evaluations"] / st["seconds"]
    st["ms_per_iteration"] = st["seconds"] / max(st["iterations"], 1) * 1e3
    st["config"] = a.config
    print(json.dumps(st))


if __name__ == "__main__":
    main()
