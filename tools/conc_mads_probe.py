"""Probe: how much two native MADS runs (config 5's, mac_mads_run: the five-launch chain per
iteration) slow each other when they run at once on one GPU from two host threads (each on its
own lane and stream), against one after the other: the bound on speculating over a failure
branch on the same device."""
import json
import os
import sys
import threading
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import __graft_entry__ as ge  # noqa: E402


def main():
    import torch
    pkg = ge.load_package()
    wl = pkg.workloads
    rng = wl.SplitMix64(20250216)
    fire_kw, x0 = wl.config5_setup(rng, 4096, 512, 512)
    ctx = pkg.Context(0)
    D = pkg.DynamicArea.DynamicArea(**fire_kw, seed=20250216, device=0)
    sim = pkg.FullSimulation.Simulation(ctx, x0, fire=D, N_iter=100, seed=20250216)
    for _ in range(3):
        sim.step()
    torch.cuda.synchronize()
    xin = sim.outputs[-1]
    kw = dict(prev=sim.x_prev, d_lim=sim.d_lim, tan_half_fov=sim.tan, n_iter=sim.N_iter,
              ell0=sim.ell0, ell_max=sim.ell_max, seed=sim.seed + 99)
    run = lambda: ctx.mads_run(xin, sim.r_max, 1e5, **kw)   # noqa: E731
    run()
    out = {}
    for rep in range(3):
        t = time.perf_counter()
        run()
        run()
        seq = time.perf_counter() - t
        th = [threading.Thread(target=run) for _ in range(2)]
        t = time.perf_counter()
        for h in th:
            h.start()
        for h in th:
            h.join()
        conc = time.perf_counter() - t
        t = time.perf_counter()
        run()
        one = time.perf_counter() - t
        out[rep] = {"one_ms": one * 1e3, "two_sequential_ms": seq * 1e3, "two_concurrent_ms": conc * 1e3,
                    "concurrent_over_one": conc / one}
        print(json.dumps(out[rep]), flush=True)
    ctx.close()


if __name__ == "__main__":
    main()
