"""Mirror of src/AreaCoverageCalculation.jl on the MI355X path.

``calculateArea`` keeps the reference signature ``calculateArea(circles, points)`` and its
semantics (src/AreaCoverageCalculation.jl:63-78): covered weight (record column 4) of the
point list under the union of the N disks ``circles = [x_1..x_N; y_1..y_N; r_1..r_N]``,
strict ``sqrt(d^2) < r`` in fp64, duplicates counted per entry. The evaluation runs in
libmaxcover's HIP kernels; there is no CPU path here.

``points`` may be a ``DevicePointList`` (resident on the GPU, the fast path the objective
closure uses) or a host array of records (M x >=4, uploaded for the call, the literal drop-in).
"""
from __future__ import annotations

import numpy as np

from ._lib import Context, InexactError, default_context
from .Base_Functions import Circle

__all__ = ["createPOI", "make_circles", "make_MADS", "calculateArea", "rmvCoveredPOI",
           "DevicePointList"]


def createPOI(dx: float, dy: float, x_length: float, y_length: float) -> np.ndarray:
    """src/AreaCoverageCalculation.jl:11-21: rows [i*dx-dx/2, j*dy-dy/2, dx*dy, dx*dy, false],
    i over 1:x_length (outer), j over 1:y_length (inner)."""
    nx = int(np.floor(x_length)) if x_length >= 1 else 0
    ny = int(np.floor(y_length)) if y_length >= 1 else 0
    i = np.arange(1, nx + 1, dtype=np.float64)
    j = np.arange(1, ny + 1, dtype=np.float64)
    out = np.empty((nx * ny, 5), dtype=np.float64)
    out[:, 0] = np.repeat(i * dx - dx / 2, ny)
    out[:, 1] = np.tile(j * dy - dy / 2, nx)
    out[:, 2] = dx * dy
    out[:, 3] = dx * dy
    out[:, 4] = 0.0
    return out


def _n_circles(arr) -> int:
    n3 = len(arr)
    if n3 % 3:
        raise InexactError(2, f"InexactError: Int64({n3}/3)")  # :34 / :65
    return n3 // 3


def make_circles(arr) -> list:
    """src/AreaCoverageCalculation.jl:33-45: [x;y;R] -> Vector{Circle}."""
    a = np.asarray(arr, dtype=np.float64)
    N = _n_circles(a)
    return [Circle(float(a[i]), float(a[N + i]), float(a[2 * N + i])) for i in range(N)]


def make_MADS(circles) -> np.ndarray:
    """src/AreaCoverageCalculation.jl:48-59: Vector{Circle} -> [x;y;R]."""
    return np.array([c.x for c in circles] + [c.y for c in circles] + [c.R for c in circles],
                    dtype=np.float64)


class DevicePointList:
    """A fire-point list resident in HBM (one libmaxcover context), plus the host copy of the
    full 5-column records so rmvCoveredPOI can return them in list order."""

    def __init__(self, records, ctx: Context | None = None):
        r = np.asarray(records, dtype=np.float64)
        if r.ndim == 1:
            r = r.reshape(-1, 5)
        self.records = np.ascontiguousarray(r)
        self.ctx = ctx or default_context()
        self.ctx.set_points_records(self.records)

    def __len__(self) -> int:
        return self.records.shape[0]

    def area(self, circles) -> float:
        return self.ctx.area(circles)

    def remove_covered(self, circles) -> np.ndarray:
        kept = self.ctx.remove_covered(circles)
        self.records = self.records[kept]
        return self.records


def calculateArea(circles, points) -> float:
    """src/AreaCoverageCalculation.jl:63-110."""
    c = np.asarray(circles, dtype=np.float64)
    _n_circles(c)
    if isinstance(points, DevicePointList):
        return points.area(c)
    ctx = default_context()
    ctx.set_points_records(np.asarray(points, dtype=np.float64).reshape(-1, 5)
                           if np.asarray(points).ndim == 1 else points)
    return ctx.area(c)


def rmvCoveredPOI(circles, points):
    """src/AreaCoverageCalculation.jl:113-137 (legacy) / src/CellFunctions.jl:81-108: delete,
    order-preserving, every entry covered by ``circles``; returns the remaining records."""
    c = np.asarray(circles, dtype=np.float64)
    _n_circles(c)
    if isinstance(points, DevicePointList):
        return points.remove_covered(c)
    recs = np.asarray(points, dtype=np.float64)
    if recs.ndim == 1:
        recs = recs.reshape(-1, 5)
    ctx = default_context()
    ctx.set_points_records(recs)
    kept = ctx.remove_covered(c)
    return recs[kept]
