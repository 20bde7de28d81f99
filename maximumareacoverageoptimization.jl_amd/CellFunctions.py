"""Mirror of src/CellFunctions.jl: the fire-point list state between MADS calls.

``initialise_POI`` (:20-57) and ``update_POI`` (:59-79) restate the INTENDED semantics of the
dynamic mode (as committed it cannot run: undefined globals, a Windows path, XLSX not imported —
SURVEY.md §3.3): rows 1..10 of the FirePoints table as flat 5-tuples, then row t+10 appended
for t != 1. ``rmvCoveredPOI`` (:81-108) runs on the GPU (covered flags + order-preserving
compaction, like ``deleteat!``)."""
from __future__ import annotations

import math

import numpy as np

from .AreaCoverageCalculation import DevicePointList, createPOI


class Cells:
    """src/CellFunctions.jl:5-16."""

    def __init__(self, points_of_interest=None, fire_point_xy_ccordinates=None):
        self.points_of_interest = (np.zeros((0, 5)) if points_of_interest is None
                                   else np.asarray(points_of_interest, dtype=np.float64))
        self.fire_point_xy_ccordinates = (np.zeros((0, 2)) if fire_point_xy_ccordinates is None
                                          else np.asarray(fire_point_xy_ccordinates))
        self.device = None  # DevicePointList once uploaded


def _high_interest(new_point, box, h_max, FOV):
    x_LB, x_UB, y_LB, y_UB = box
    check = [(new_point[0] < xu) and (new_point[0] > xl) and (new_point[1] < yu) and
             (new_point[1] > yl) for xl, xu, yl, yu in zip(x_LB, x_UB, y_LB, y_UB)]
    if any(check):                                       # :42-45 / :68-72
        new_point[3] = (h_max * math.tan(FOV / 2)) ** 2 * math.pi
    return new_point


def initialise_POI(self: Cells, environment_type: str, firepoints=None,
                   box=([2500], [3500], [1000], [2000]), h_max: float = 30.0,
                   FOV: float = 100 / 180 * math.pi) -> Cells:
    """src/CellFunctions.jl:20-57. ``firepoints``: list of (n_i x 5) rows (workloads.load_firepoints)."""
    if environment_type == "dynamic":
        if firepoints is None:
            raise ValueError("dynamic environment needs the FirePoints table")
        pts = []
        for row in range(min(10, len(firepoints))):       # :35
            for p in firepoints[row]:
                pts.append(_high_interest(np.array(p, dtype=np.float64), box, h_max, FOV))
        self.points_of_interest = np.array(pts, dtype=np.float64).reshape(-1, 5)
        self.fire_point_xy_ccordinates = self.points_of_interest[:, :2].copy()
    else:
        self.points_of_interest = createPOI(5.0, 5.0, 100.0, 100.0)   # :53
    self.device = None
    return self


def update_POI(self: Cells, t: int, firepoints, box=([2500], [3500], [1000], [2000]),
               h_max: float = 30.0, FOV: float = 100 / 180 * math.pi) -> Cells:
    """src/CellFunctions.jl:59-79: append row t+10 (1-based) for t != 1."""
    if t != 1 and t % 1 == 0:
        r = int(t / 1 + 10) - 1
        if r < len(firepoints):
            new = [_high_interest(np.array(p, dtype=np.float64), box, h_max, FOV)
                   for p in firepoints[r]]
            if new:
                self.points_of_interest = np.concatenate(
                    [self.points_of_interest, np.array(new).reshape(-1, 5)], axis=0)
                self.fire_point_xy_ccordinates = self.points_of_interest[:, :2].copy()
                self.device = None
    return self


def rmvCoveredPOI(self: Cells, circles) -> Cells:
    """src/CellFunctions.jl:81-108, on the GPU."""
    dev = DevicePointList(self.points_of_interest)
    self.points_of_interest = dev.remove_covered(np.asarray(circles, dtype=np.float64))
    self.device = dev
    return self
