"""TEST INFRASTRUCTURE ONLY — the checker, never the thing measured or shipped.

Only tests/, ``__graft_entry__.smoke()`` and bench.py's ``cpu_baseline`` leg may import this
module. The product path (libmaxcover + the package) never does.

Three independent restatements of the reference's area-coverage path:

1. ``libref_cpu.so`` (oracle/ref_cpu.c): plain C, statement-by-statement restatement of
   ``calculateArea`` (src/AreaCoverageCalculation.jl:63-78), the objective
   (src/TDM_STATIC_opt.jl:82-100), ``rmvCoveredPOI`` (src/CellFunctions.jl:81-108),
   ``createPOI`` (src/AreaCoverageCalculation.jl:11-21), ``cons3``
   (src/TDM_Constraints.jl:54-75), built -O2 -ffp-contract=off, no fast-math.
2. numpy (this file, ``np_*``): vectorised over points, same fp64 rounding sequence
   (``dx*dx + dy*dy`` without FMA, IEEE sqrt, strict ``<``), sequential sum via
   ``np.add.accumulate`` so the summation order is the list order (:67, :72).
3. Exact integer lattice counting (``lattice_count``) for half-integer lattices with integer
   disks, independent of floating point.

Parity status: the reference is Julia and Julia is absent here, so the reference cannot be run;
its own tests pin nothing on this path (test/runtests.jl:4-6). The oracle is pinned by (a) the
integer KATs, (b) agreement of the C and numpy restatements, (c) the FirePoints.xlsx data
(tests/golden/firepoints.csv). DirectSearch.jl's candidate sequence is parity-unpinned.
"""
from __future__ import annotations

import ctypes
import math
import os
import subprocess
from fractions import Fraction

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB = None

_dp = ctypes.POINTER(ctypes.c_double)
_i64p = ctypes.POINTER(ctypes.c_int64)


def build() -> str:
    """Compile oracle/ref_cpu.c -> oracle/libref_cpu.so (gcc)."""
    subprocess.run(["make", "-s", "-C", _HERE], check=True)
    return os.path.join(_HERE, "libref_cpu.so")


def lib() -> ctypes.CDLL:
    global _LIB
    if _LIB is None:
        path = os.path.join(_HERE, "libref_cpu.so")
        src = os.path.join(_HERE, "ref_cpu.c")
        if not os.path.exists(path) or os.path.getmtime(path) < os.path.getmtime(src):
            build()
        L = ctypes.CDLL(path)
        L.ref_calculate_area_rec.argtypes = [_dp, ctypes.c_int64, _dp, ctypes.c_int64,
                                             ctypes.c_int64, _dp]
        L.ref_calculate_area_rec.restype = ctypes.c_int
        L.ref_calculate_area_ptrs.argtypes = [_dp, ctypes.c_int64, ctypes.c_void_p,
                                              ctypes.c_int64, _dp]
        L.ref_calculate_area_ptrs.restype = ctypes.c_int
        L.ref_objective_ptrs.argtypes = [_dp, ctypes.c_int64, ctypes.c_void_p, ctypes.c_int64,
                                         _dp, ctypes.c_double, _dp]
        L.ref_objective_ptrs.restype = ctypes.c_int
        L.ref_points_alloc.argtypes = [_dp, ctypes.c_int64, ctypes.c_int64]
        L.ref_points_alloc.restype = ctypes.c_void_p
        L.ref_points_free.argtypes = [ctypes.c_void_p, ctypes.c_int64]
        L.ref_points_free.restype = None
        L.ref_area_batch_ptrs.argtypes = [_dp, ctypes.c_int64, ctypes.c_int64, ctypes.c_void_p,
                                          ctypes.c_int64, _dp, ctypes.c_int]
        L.ref_area_batch_ptrs.restype = ctypes.c_int
        L.ref_max_threads.argtypes = []
        L.ref_max_threads.restype = ctypes.c_int
        L.ref_remove_covered_rec.argtypes = [_dp, ctypes.c_int64, _dp, ctypes.c_int64,
                                             ctypes.c_int64, _i64p, _i64p]
        L.ref_remove_covered_rec.restype = ctypes.c_int
        L.ref_create_poi.argtypes = [ctypes.c_double] * 4 + [_dp]
        L.ref_create_poi.restype = ctypes.c_int64
        L.ref_cons3.argtypes = [_dp, _dp, ctypes.c_int64, _dp, ctypes.c_double]
        L.ref_cons3.restype = ctypes.c_int
        L.ref_allocate_even_circles.argtypes = [ctypes.c_double, ctypes.c_int64, ctypes.c_double,
                                                ctypes.c_double, ctypes.c_double, _dp]
        L.ref_allocate_even_circles.restype = None
        _u8 = ctypes.POINTER(ctypes.c_uint8)
        L.ref_fire_thresholds.argtypes = [ctypes.c_double] * 3 + [_dp]
        L.ref_fire_thresholds.restype = None
        L.ref_fire_init.argtypes = [_u8, ctypes.c_int64, ctypes.c_int64, ctypes.c_double,
                                    ctypes.c_uint64] + [ctypes.c_int64] * 4
        L.ref_fire_init.restype = None
        L.ref_fire_step.argtypes = [_u8, _u8, ctypes.c_int64, ctypes.c_int64, _dp, ctypes.c_double,
                                    ctypes.c_double, ctypes.c_uint64, ctypes.c_uint64, _dp,
                                    ctypes.c_int64]
        L.ref_fire_step.restype = ctypes.c_int64
        L.ref_lattice_count_batch.argtypes = [_dp, ctypes.c_int64, ctypes.c_int64, ctypes.c_int64,
                                              ctypes.c_int64, _i64p, ctypes.c_int]
        L.ref_lattice_count_batch.restype = ctypes.c_int
        L.ref_violation_batch.argtypes = [_dp, ctypes.c_int64, ctypes.c_int64, _dp, _dp]
        L.ref_violation_batch.restype = None
        L.ref_cons3_batch.argtypes = [_dp, _dp, ctypes.c_int64, ctypes.c_int64, _dp, ctypes.c_double,
                                      ctypes.POINTER(ctypes.c_uint8)]
        L.ref_cons3_batch.restype = None
        _LIB = L
    return _LIB


def _p(a: np.ndarray):
    return a.ctypes.data_as(_dp)


def _f64(a) -> np.ndarray:
    return np.ascontiguousarray(np.asarray(a, dtype=np.float64))


class InexactError(ValueError):
    """Julia's Int(length(circles)/3) failure (src/AreaCoverageCalculation.jl:65)."""


# ----------------------------------------------------------------------------- C oracle

def ref_area(circles, rec) -> float:
    """calculateArea(circles, points) over M x >=4 records (C restatement)."""
    c = _f64(circles)
    r = _f64(rec)
    if r.ndim != 2:
        r = r.reshape(-1, 5)
    out = ctypes.c_double()
    rc = lib().ref_calculate_area_rec(_p(c), c.size, _p(r), r.shape[0], r.shape[1],
                                      ctypes.byref(out))
    if rc == 2:
        raise InexactError(f"length(circles)={c.size} is not a multiple of 3")
    return out.value


def ref_objective(x, rec, r_max, penalty: float = 1e5) -> float:
    """AreaMaxObjective(x) (src/TDM_STATIC_opt.jl:82-100), C restatement."""
    x = _f64(x)
    rm = _f64(r_max)
    area = ref_area(x, rec)
    N = x.size // 3
    violation = 0.0
    for i in range(N):  # :90-93, sequential
        violation += abs(float(x[i + 2 * N]) - float(rm[i]))
    return -area + violation * penalty


class PointerList:
    """Vector{Vector{Float64}} mirror in C memory (one malloc per entry), for the CPU baseline."""

    def __init__(self, rec):
        r = _f64(rec)
        if r.ndim != 2:
            r = r.reshape(-1, 5)
        self.M = r.shape[0]
        self._h = lib().ref_points_alloc(_p(r), self.M, r.shape[1])
        if not self._h and self.M:
            raise MemoryError("ref_points_alloc failed")

    def area_batch(self, cands, nthreads: int = 0) -> np.ndarray:
        c = _f64(cands)
        K, three_n = c.shape
        out = np.zeros(K, dtype=np.float64)
        rc = lib().ref_area_batch_ptrs(_p(c), three_n, K, self._h, self.M, _p(out), nthreads)
        if rc == 2:
            raise InexactError("three_n not a multiple of 3")
        return out

    def close(self):
        if getattr(self, "_h", None):
            lib().ref_points_free(self._h, self.M)
            self._h = None

    def __del__(self):
        self.close()


def ref_max_threads() -> int:
    return int(lib().ref_max_threads())


def ref_remove_covered(circles, rec) -> np.ndarray:
    """rmvCoveredPOI (src/CellFunctions.jl:81-108): kept 0-based indices, in list order."""
    c = _f64(circles)
    r = _f64(rec)
    kept = np.zeros(max(r.shape[0], 1), dtype=np.int64)
    m = ctypes.c_int64()
    rc = lib().ref_remove_covered_rec(_p(c), c.size, _p(r), r.shape[0], r.shape[1],
                                      kept.ctypes.data_as(_i64p), ctypes.byref(m))
    if rc == 2:
        raise InexactError("three_n not a multiple of 3")
    return kept[: m.value].copy()


def ref_create_poi(dx: float, dy: float, x_length: float, y_length: float) -> np.ndarray:
    n = lib().ref_create_poi(dx, dy, x_length, y_length, None)
    out = np.zeros((n, 5), dtype=np.float64)
    lib().ref_create_poi(dx, dy, x_length, y_length, _p(out))
    return out


def ref_cons3(prev, x, d_lim, tan_half_fov: float) -> bool:
    p = _f64(prev)
    xx = _f64(x)
    d = _f64(d_lim)
    return bool(lib().ref_cons3(_p(p), _p(xx), xx.size, _p(d), tan_half_fov))


def ref_allocate_even_circles(r_centering, N, r_uav, cx, cy) -> np.ndarray:
    out = np.zeros(3 * N, dtype=np.float64)
    lib().ref_allocate_even_circles(r_centering, N, r_uav, cx, cy, _p(out))
    return out


# ----------------------------------------------------------------------------- numpy oracle

def np_covered(circles, x, y) -> np.ndarray:
    """Per-entry covered flag, same rounding as src/AreaCoverageCalculation.jl:70."""
    c = _f64(circles)
    if c.size % 3:
        raise InexactError("three_n not a multiple of 3")
    N = c.size // 3
    x = _f64(x)
    y = _f64(y)
    cov = np.zeros(x.shape, dtype=bool)
    with np.errstate(invalid="ignore", over="ignore"):
        for i in range(N):
            dx = x - c[i]
            dy = y - c[N + i]
            a = dx * dx + dy * dy          # two roundings + one, no FMA
            cov |= np.sqrt(a) < c[2 * N + i]
    return cov


def np_area(circles, x, y, w) -> float:
    """calculateArea with the list-order sequential sum (np.add.accumulate is sequential)."""
    cov = np_covered(circles, x, y)
    vals = _f64(w)[cov]
    if vals.size == 0:
        return 0.0
    return float(np.add.accumulate(vals)[-1])


# ----------------------------------------------------------------------------- exact KATs

def lattice_count(circles_int, G: int, pitch: int = 5) -> int:
    """Exact integer count of lattice entries ((i-1/2)p, (j-1/2)p), i,j in 1..G, lying strictly
    inside at least one disk with integer centre (cx, cy) and integer radius R.

    For such inputs fl(sqrt(d^2)) < R <=> d^2 < R^2 exactly: d^2 is an exact quarter-integer
    = 2q + 1/2 (odd^2 + odd^2 = 2 mod 8, over 4), R^2 is an integer, and the rounding band of
    sqrt near R (~R^2 * 2^-52) contains no such value for R < 2^20.
    """
    c = [int(v) for v in circles_int]
    N = len(c) // 3
    total = 0
    # twice the coordinates: X = (2i-1)*p
    for i in range(1, G + 1):
        X = (2 * i - 1) * pitch
        for j in range(1, G + 1):
            Y = (2 * j - 1) * pitch
            for k in range(N):
                dx = X - 2 * c[k]
                dy = Y - 2 * c[N + k]
                if dx * dx + dy * dy < 4 * c[2 * N + k] * c[2 * N + k]:
                    total += 1
                    break
    return total


def lattice_count_np(circles_int, G: int, pitch: int = 5) -> int:
    """Vectorised integer version of lattice_count (int64 exact)."""
    c = np.asarray(circles_int, dtype=np.int64)
    N = c.size // 3
    i = np.arange(1, G + 1, dtype=np.int64)
    X = ((2 * i - 1) * pitch)[:, None]
    Y = ((2 * i - 1) * pitch)[None, :]
    cov = np.zeros((G, G), dtype=bool)
    for k in range(N):
        dx = X - 2 * c[k]
        dy = Y - 2 * c[N + k]
        cov |= (dx * dx + dy * dy) < 4 * c[2 * N + k] * c[2 * N + k]
    return int(cov.sum())


def exact_threshold(r: float) -> float:
    """Largest double T with (fl(sqrt(a)) < r) <=> (a <= T) for all doubles a >= 0, computed
    with exact rationals (independent of the library's integer-bit implementation)."""
    if not (r > 0.0):
        return -1.0
    if math.isinf(r):
        return float(np.finfo(np.float64).max)
    pred = math.nextafter(r, 0.0)
    m = (Fraction(pred) + Fraction(r)) / 2
    m2 = m * m
    dmax = float(np.finfo(np.float64).max)
    if m2 >= Fraction(dmax):
        return dmax
    # round m2 down to a double
    t = float(m2)                       # round to nearest (int/int is correctly rounded)
    if Fraction(t) > m2:
        t = math.nextafter(t, 0.0)
    if math.isinf(t):
        t = float(np.finfo(np.float64).max)
    return t


def lattice_count_batch(cands, G: int, pitch: int = 5, nthreads: int = 0) -> np.ndarray:
    """lattice_count for every row of cands (K x 3N integer-valued disks) on the G x G lattice of
    pitch `pitch`: the exact number of covered entries (C, ref_lattice_count_batch, OpenMP)."""
    c = _f64(np.atleast_2d(cands))
    out = np.zeros(c.shape[0], dtype=np.int64)
    rc = lib().ref_lattice_count_batch(_p(c), c.shape[1], c.shape[0], int(G), int(pitch),
                                       out.ctypes.data_as(_i64p), int(nthreads))
    if rc == 2:
        raise InexactError("three_n not a multiple of 3")
    if rc != 0:
        raise MemoryError("ref_lattice_count_batch: mask allocation failed")
    return out


def violation_batch(cands, r_max) -> np.ndarray:
    """sum_i |x[2N+i] - r_max[i]| per row, accumulated sequentially (src/TDM_STATIC_opt.jl:89-93)."""
    c = _f64(np.atleast_2d(cands))
    rm = _f64(r_max)
    out = np.zeros(c.shape[0])
    lib().ref_violation_batch(_p(c), c.shape[1], c.shape[0], _p(rm), _p(out))
    return out


def cons3_batch(prev, cands, d_lim, tan_half_fov: float) -> np.ndarray:
    """ref_cons3 per row (src/TDM_Constraints.jl:54-75): True = feasible."""
    c = _f64(np.atleast_2d(cands))
    pv, dl = _f64(prev), _f64(d_lim)
    out = np.zeros(c.shape[0], dtype=np.uint8)
    lib().ref_cons3_batch(_p(pv), _p(c), c.shape[1], c.shape[0], _p(dl), float(tan_half_fov),
                          out.ctypes.data_as(ctypes.POINTER(ctypes.c_uint8)))
    return out.astype(bool)


def lattice_count_fast(circles_int, G: int, pitch: int = 5) -> int:
    """lattice_count for large G: each disk only touches the cells of its bounding box; the
    union is accumulated in a G x G boolean mask with exact int64 tests."""
    c = np.asarray(circles_int, dtype=np.int64)
    N = c.size // 3
    cov = np.zeros((G, G), dtype=bool)
    for k in range(N):
        cx, cy, R = int(c[k]), int(c[N + k]), int(c[2 * N + k])
        if R <= 0:
            continue
        # lattice index i has 2x = (2i-1)*pitch; |x - cx| < R  =>  i in a small window
        i0 = max(1, (2 * (cx - R)) // (2 * pitch))
        i1 = min(G, (2 * (cx + R)) // (2 * pitch) + 2)
        j0 = max(1, (2 * (cy - R)) // (2 * pitch))
        j1 = min(G, (2 * (cy + R)) // (2 * pitch) + 2)
        if i0 > i1 or j0 > j1:
            continue
        ii = np.arange(i0, i1 + 1, dtype=np.int64)
        jj = np.arange(j0, j1 + 1, dtype=np.int64)
        dx = ((2 * ii - 1) * pitch - 2 * cx)[:, None]
        dy = ((2 * jj - 1) * pitch - 2 * cy)[None, :]
        cov[i0 - 1:i1, j0 - 1:j1] |= (dx * dx + dy * dy) < 4 * R * R
    return int(cov.sum())


class RefFire:
    """src/DynamicArea.jl restated in C (ref_fire_*): the CPU checker of the GPU fire generator."""

    def __init__(self, nx, ny, dx=5.0, dy=5.0, forest_density=0.7, prob_spread=0.5, wind_speed=4.0,
                 wind_direction=math.radians(270), ignition=(40, 60, 69, 71), seed=20250216):
        self.nx, self.ny, self.dx, self.dy, self.seed = int(nx), int(ny), float(dx), float(dy), seed
        self.p9 = np.zeros(9)
        lib().ref_fire_thresholds(wind_speed, wind_direction, prob_spread, _p(self.p9))
        self.grid = np.zeros(self.nx * self.ny, dtype=np.uint8)
        ix0, ix1, iy0, iy1 = ignition
        lib().ref_fire_init(self.grid.ctypes.data_as(ctypes.POINTER(ctypes.c_uint8)), self.nx,
                            self.ny, forest_density, seed, ix0, ix1, iy0, iy1)
        self.t = 0

    def step(self) -> np.ndarray:
        """One update_grid (:52-72); returns the pushed points as (n, 5) records."""
        self.t += 1
        gn = np.empty_like(self.grid)
        u8 = ctypes.POINTER(ctypes.c_uint8)
        n = lib().ref_fire_step(self.grid.ctypes.data_as(u8), gn.ctypes.data_as(u8), self.nx,
                                self.ny, _p(self.p9), self.dx, self.dy, self.seed, self.t, None, 0)
        rec = np.zeros((max(n, 1), 5))
        lib().ref_fire_step(self.grid.ctypes.data_as(u8), gn.ctypes.data_as(u8), self.nx, self.ny,
                            _p(self.p9), self.dx, self.dy, self.seed, self.t, _p(rec), n)
        self.grid = gn
        return rec[:n]
