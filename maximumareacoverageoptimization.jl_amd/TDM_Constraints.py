"""Mirror of the extreme constraints the driver passes to MADS (src/TDM_Constraints.jl):
``cons1`` (:9-19, always true) and ``create_cons3`` (:54-75, per-UAV 3-D displacement limit).
The returned ``cons3`` evaluates on the host with the reference's arithmetic and also carries
its data (``prev``, ``d_lim``, ``tan_half_fov``) so the batched GPU poll can apply the same
test inside libmaxcover (finalize kernel, exact threshold form)."""
from __future__ import annotations

import math

import numpy as np


def cons1(x) -> bool:
    """src/TDM_Constraints.jl:9-19 — the body is commented out; always feasible."""
    return True


def create_cons3(pre_optimized_circles_MADS, FOV: float, d_lim):
    """src/TDM_Constraints.jl:54-75. ``pre_optimized_circles_MADS``: list of Circle or [x;y;R]."""
    from .AreaCoverageCalculation import make_MADS
    pre = pre_optimized_circles_MADS
    if len(pre) and not isinstance(pre[0], (float, int, np.floating, np.integer)):
        prev = make_MADS(pre)
    else:
        prev = np.asarray(pre, dtype=np.float64)
    prev = np.ascontiguousarray(prev, dtype=np.float64)
    dl = np.ascontiguousarray(np.asarray(d_lim, dtype=np.float64))
    t = math.tan(FOV / 2)

    def cons3(x) -> bool:
        xx = np.asarray(x, dtype=np.float64)
        N = xx.size // 3
        for i in range(N):
            x1, y1, z1 = float(prev[i]), float(prev[N + i]), float(prev[2 * N + i]) / t
            x2, y2, z2 = float(xx[i]), float(xx[N + i]), float(xx[2 * N + i]) / t
            if math.sqrt((x1 - x2) * (x1 - x2) + (y1 - y2) * (y1 - y2) + (z1 - z2) * (z1 - z2)) \
                    > dl[i]:
                return False
        return True

    cons3.prev = prev
    cons3.d_lim = dl
    cons3.tan_half_fov = t
    return cons3
