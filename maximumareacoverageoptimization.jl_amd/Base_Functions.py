"""Mirror of the parts of src/Base_Functions.jl the hot path touches: the ``Circle`` record
(:37-41) and ``allocate_even_circles`` (:44-65), the driver's initial swarm placement
(src/FullSimulation.jl:803). Plotting and the legacy analytic-area geometry are out of scope."""
from __future__ import annotations

import math
from dataclasses import dataclass

import numpy as np


@dataclass
class Circle:
    """src/Base_Functions.jl:37-41 — mutable struct Circle x, y, R."""
    x: float
    y: float
    R: float


def allocate_even_circles(r_centering_cir: float, N: int, r_uav: float, center_x: float,
                          center_y: float) -> np.ndarray:
    """src/Base_Functions.jl:44-65: N UAVs evenly on a ring; returns [x; y; R] (3N)."""
    xs, ys, rs = [], [], []
    for i in range(1, N + 1):
        ref_angle = 2 * math.pi / N * (i - 1)
        xs.append(r_centering_cir * math.cos(ref_angle) + center_x)
        ys.append(r_centering_cir * math.sin(ref_angle) + center_y)
        rs.append(float(r_uav))
    return np.array(xs + ys + rs, dtype=np.float64)
