"""Synthetic workloads of SURVEY.md §8(d) / BASELINE.md, reproducible from a splitmix64 seed.

Points: G x G lattice, pitch 5 m (the reference pitch, src/CellFunctions.jl:53), entry
((i-1/2)*5, (j-1/2)*5), i outer / j inner (createPOI order, src/AreaCoverageCalculation.jl:11-21),
weight 25.0. Disks: integer centres uniform over [0, 5G]^2, R = 36 (what the reference iterates
converge to: z = 30.2076 <=> R = 36 in Quadrotor_Targets.xlsx). Candidates: k = 0 incumbent,
k = 1..n: x0 + delta*b_k, k = n+1..2n: x0 - delta*b_k, b_k the columns of an LTMADS-style
integer basis (lower triangular, diagonal +-2^l, sub-diagonal in (-2^l, 2^l), random row and
column permutation), l = 2, delta = 1; n = 3N, K = 2n + 1 = 6N + 1.
"""
from __future__ import annotations

import numpy as np

SEED = 20250216
PITCH = 5.0
RADIUS = 36.0

# BASELINE.json configs 2..5 (config 1 is the FirePoints fixture).
CONFIGS = {
    2: dict(G=1024, N=32, K=1, name="32 UAVs, 1M-cell synthetic fire grid, fp64, single eval"),
    3: dict(G=2048, N=128, K=769, name="128 UAVs, 4M-cell grid, full MADS poll batch"),
    4: dict(G=4096, N=512, K=3073, name="512 UAVs, 16M-cell grid, full MADS poll batch"),
    # config 5: src/DynamicArea.jl's automaton on a 4096 x 4096 grid of 5 m cells, a central
    # 512 x 512-cell ignition block, 512 UAVs over the burning block, MPC steps of FullSimulation
    5: dict(G=4096, N=512, K=3072, ignition=512,
            name="512 UAVs, CA fire on a 4096^2 grid streamed per MPC step, end-to-end loop"),
}


def config5_setup(rng: "SplitMix64", G: int = 4096, N: int = 512, ignition: int = 512):
    """(fire kwargs for DynamicArea, starting circles [x;y;R]) of config 5."""
    c0 = G // 2 - ignition // 2 + 1
    fire = dict(X=G * PITCH, Y=G * PITCH, dx=PITCH, dy=PITCH,
                x_start1=c0 * PITCH, x_start2=(c0 + ignition - 1) * PITCH,
                y_start1=c0 * PITCH, y_start2=(c0 + ignition - 1) * PITCH)
    lo = (c0 - 1) * PITCH
    span = ignition * PITCH
    cx = np.round(lo + rng.uniform(N) * span)
    cy = np.round(lo + rng.uniform(N) * span)
    return fire, np.concatenate([cx, cy, np.full(N, RADIUS)])

_M64 = np.uint64(0xFFFFFFFFFFFFFFFF)


class SplitMix64:
    """splitmix64 stream (Steele, Lea, Flood 2014), vectorised; identical to the C++ form."""

    def __init__(self, seed: int = SEED):
        self.state = np.uint64(seed & 0xFFFFFFFFFFFFFFFF)

    def next_u64(self, n: int) -> np.ndarray:
        with np.errstate(over="ignore"):
            inc = np.uint64(0x9E3779B97F4A7C15)
            steps = np.arange(1, n + 1, dtype=np.uint64)
            z = self.state + steps * inc
            self.state = self.state + np.uint64(n) * inc
            z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
            z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
            return z ^ (z >> np.uint64(31))

    def uniform(self, n: int) -> np.ndarray:
        """U[0, 1) doubles from the top 53 bits."""
        return (self.next_u64(n) >> np.uint64(11)).astype(np.float64) * (1.0 / 9007199254740992.0)

    def integers(self, lo: int, hi: int, n: int) -> np.ndarray:
        """Uniform integers in [lo, hi] (inclusive)."""
        span = hi - lo + 1
        return lo + np.floor(self.uniform(n) * span).astype(np.int64)

    def permutation(self, n: int) -> np.ndarray:
        keys = self.next_u64(n)
        return np.argsort(keys, kind="stable")


def grid_points(G: int, pitch: float = PITCH, weight: float | None = None):
    """createPOI(pitch, pitch, G, G) as SoA arrays (x, y, w)."""
    c = (np.arange(1, G + 1, dtype=np.float64) * pitch - pitch / 2)
    x = np.repeat(c, G)
    y = np.tile(c, G)
    w = np.full(G * G, pitch * pitch if weight is None else weight, dtype=np.float64)
    return x, y, w


def uniform_disks(N: int, G: int, rng: SplitMix64, pitch: float = PITCH,
                  radius: float = RADIUS) -> np.ndarray:
    """[x; y; R] with integer centres uniform over [0, pitch*G]^2."""
    L = int(round(pitch * G))
    cx = rng.integers(0, L, N).astype(np.float64)
    cy = rng.integers(0, L, N).astype(np.float64)
    return np.concatenate([cx, cy, np.full(N, radius)])


def clustered_disks(N: int, G: int, rng: SplitMix64, pitch: float = PITCH,
                    radius: float = RADIUS) -> np.ndarray:
    """Integer centres within sqrt(N)*40 m of the domain centre (overlapping footprints)."""
    L = pitch * G
    half = min(np.sqrt(N) * 40.0, L / 2)
    c0 = L / 2
    cx = np.round(c0 + (rng.uniform(N) * 2 - 1) * half)
    cy = np.round(c0 + (rng.uniform(N) * 2 - 1) * half)
    return np.concatenate([cx, cy, np.full(N, radius)])


def ltmads_basis(n: int, ell: int, rng: SplitMix64) -> np.ndarray:
    """n x n integer LTMADS-style basis: lower-triangular L with diagonal +-2^ell and strictly
    lower entries uniform in (-2^ell, 2^ell), rows and columns randomly permuted (Audet & Dennis
    2006, LTMADS). Column k is poll direction b_k."""
    Lm, rp, cp = ltmads_basis_parts(n, ell, rng)
    return Lm[rp][:, cp]


def ltmads_basis_parts(n: int, ell: int, rng: SplitMix64):
    """(L, rp, cp) with ltmads_basis's draws (the same rng stream): B = L[rp][:, cp] — the basis
    form mac_poll_basis_f64 takes (L lower triangular, rp / cp permutations)."""
    b = 2 ** ell
    Lm = np.zeros((n, n), dtype=np.int64)
    signs = np.where(rng.uniform(n) < 0.5, -1, 1)
    Lm[np.arange(n), np.arange(n)] = signs * b
    il = np.tril_indices(n, -1)
    if il[0].size:
        Lm[il] = rng.integers(-b + 1, b - 1, il[0].size)
    rp = rng.permutation(n)
    cp = rng.permutation(n)
    return Lm, rp, cp


def poll_candidates(x0: np.ndarray, rng: SplitMix64, ell: int = 2, delta: float = 1.0,
                    include_incumbent: bool = True) -> np.ndarray:
    """K x 3N candidate matrix (row k = candidate k): [x0, x0 + delta*B, x0 - delta*B]."""
    n = x0.size
    B = ltmads_basis(n, ell, rng).astype(np.float64)
    plus = x0[None, :] + delta * B.T
    minus = x0[None, :] - delta * B.T
    parts = ([x0[None, :]] if include_incumbent else []) + [plus, minus]
    return np.ascontiguousarray(np.concatenate(parts, axis=0))


def make_config(cfg: int, seed: int = SEED, disks: str = "uniform"):
    """(x, y, w, cands, r_max) for BASELINE config 2..4."""
    c = CONFIGS[cfg]
    rng = SplitMix64(seed)
    x, y, w = grid_points(c["G"])
    gen = uniform_disks if disks == "uniform" else clustered_disks
    x0 = gen(c["N"], c["G"], rng)
    if c["K"] == 1:
        cands = x0[None, :].copy()
    else:
        cands = poll_candidates(x0, rng)
        assert cands.shape[0] == c["K"], (cands.shape, c["K"])
    r_max = np.full(c["N"], 30.0 * np.tan(100 / 180 * np.pi / 2))
    return x, y, w, cands, r_max


def shuffled_with_duplicates(x, y, w, rng: SplitMix64, dup_frac: float = 0.05):
    """Parity variant: the list shuffled, with dup_frac of its entries duplicated."""
    M = x.size
    nd = int(M * dup_frac)
    extra = rng.integers(0, M - 1, nd) if nd and M else np.zeros(0, dtype=np.int64)
    idx = np.concatenate([np.arange(M), extra])
    perm = rng.permutation(idx.size)
    idx = idx[perm]
    return x[idx].copy(), y[idx].copy(), w[idx].copy()


def load_firepoints(path: str):
    """FirePoints table (tests/golden/firepoints.csv, converted from src/FirePoints.xlsx):
    one line per xlsx row = timestep, flat groups of 5 [x, y, area, importance, covered]
    (src/DynamicArea.jl:100-108, read as in src/CellFunctions.jl:36-41). Returns a list of
    (n_i x 5) arrays (firepoints.read_csv)."""
    from .firepoints import read_csv
    return read_csv(path)
