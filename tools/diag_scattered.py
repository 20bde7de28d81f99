"""Diagnostic: the chain and walk AUTO takes for a scattered batch (64 unrelated 8-disk layouts) on
a fresh context, call by call (tests/test_gpu_parity.py test_walk_choice_scattered_batch)."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import __graft_entry__ as ge  # noqa: E402

pkg = ge.load_package()
wl = pkg.workloads
rng = wl.SplitMix64(4244)
G, N, K = 512, 8, 64
x, y, w = wl.grid_points(G)
C = np.stack([wl.uniform_disks(N, G, rng) for _ in range(K)])
with pkg.Context(0) as c:
    c.set_points(x, y, w)
    for i in range(6):
        c.profile(True)
        c.profile_read(reset=True)
        c.area_batch(C)
        kern = {k: n for k, (ms, n) in c.profile_kernels().items() if n}
        walk = c.profile_read(reset=True)[3]
        c.profile(False)
        print(i, walk, sorted(kern), flush=True)
