"""Mirror of src/TDM_STATIC_opt.jl: the objective factory the solver calls and the MADS wrapper.

``createObjective(cells, N, r_max)`` (:82-100) packs ``cells.points_of_interest`` into the
device list ONCE per MPC step and returns ``AreaMaxObjective(x)`` with the reference closure
signature; ``AreaMaxObjective.batch(X)`` evaluates a whole poll (K x 3N) in one launch.

``optimize(input, obj, cons_ext, cons_prog, N_iter)`` (:118-222) stands in for DirectSearch's
``Optimize!`` (third-party, not vendored, version unpinned — SURVEY.md §8c): a granular MADS with
LTMADS-style integer poll directions (maximal basis, 2n trial points), extreme-barrier
constraints and a complete poll evaluated as one GPU batch. Its candidate sequence is NOT
DirectSearch's (parity unpinned); per-candidate objective values and the poll argmin are.
Returns ``(result, runtime_seconds)`` like the reference (:219-220).
"""
from __future__ import annotations

import time

import numpy as np

from ._lib import Context, InexactError, default_context
from .workloads import SplitMix64, ltmads_basis

PENALTY = 1e5  # :97


def createObjective(cells, N: int, r_max, ctx: Context | None = None):
    """src/TDM_STATIC_opt.jl:82-100. ``r_max`` is read at call time (the reference closure
    captures the array by reference; src/FullSimulation.jl:64-76 mutates it between steps)."""
    ctx = ctx or default_context()
    pts = getattr(cells, "points_of_interest", cells)
    recs = np.asarray(pts, dtype=np.float64)
    if recs.ndim == 1:
        recs = recs.reshape(-1, 5)
    ctx.set_points_records(recs)

    def AreaMaxObjective(x) -> float:
        xx = np.asarray(x, dtype=np.float64)
        if xx.size % 3:
            raise InexactError(2, f"InexactError: Int64({xx.size}/3)")
        area_covered = ctx.area(xx)                     # :85-87
        violation = 0.0                                 # :89
        rm = np.asarray(r_max, dtype=np.float64)
        for i in range(N):                              # :90-93
            violation += abs(float(xx[i + 2 * N]) - float(rm[i]))
        return -area_covered + violation * PENALTY      # :97

    def batch(X) -> np.ndarray:
        Xa = np.asarray(X, dtype=np.float64)
        if Xa.ndim != 2 or Xa.shape[1] != 3 * N:
            raise ValueError("batch expects K x 3N")
        return ctx.objective_batch(Xa, np.asarray(r_max, dtype=np.float64), PENALTY)

    def poll(X, cons3=None):
        """(best_obj, best_idx, objectives) with cons3 applied on the device."""
        Xa = np.asarray(X, dtype=np.float64)
        kw = {}
        if cons3 is not None and hasattr(cons3, "prev"):
            kw = dict(prev=cons3.prev, d_lim=cons3.d_lim, tan_half_fov=cons3.tan_half_fov)
        return ctx.poll_best(Xa, np.asarray(r_max, dtype=np.float64), PENALTY, want_all=True,
                             **kw)

    AreaMaxObjective.batch = batch
    AreaMaxObjective.poll = poll
    AreaMaxObjective.ctx = ctx
    AreaMaxObjective.N = N
    return AreaMaxObjective


class Status:
    def __init__(self):
        self.runtime_total = 0.0
        self.iteration = 0
        self.function_evaluations = 0
        # poll candidates passing cons3 (mac_mads_stats.feasible_evaluations: every candidate
        # without cons3) and polls where none does (a superset of mac_mads_stats.rejected_polls,
        # which counts the polls rejected by their diagonal steps alone)
        self.cons3_passed = 0
        self.cons3_empty_polls = 0
        self.successes = 0   # polls that moved the incumbent (mac_mads_stats.successes)
        self.optimization_status = "Unoptimized"


class MADSResult:
    """What the driver reads back: x (feasible best) or i (infeasible best), status."""

    def __init__(self):
        self.x = None
        self.i = None
        self.x_cost = np.inf
        self.status = Status()


def mads(input, obj, cons_ext=(), N_iter: int = 100, ell0: int = 2, ell_max: int = 6,
         seed: int = 20250216) -> MADSResult:
    """Granular MADS, complete poll over D = [B, -B] (B an LTMADS-style integer basis whose
    entries are bounded by 2^ell), extreme barrier on cons_ext. Success: ell <- min(ell+1,
    ell_max) (larger steps); failure: ell <- ell-1; stop when ell < 0 (below the granularity
    1.0 of every variable, src/TDM_STATIC_opt.jl:131-137) or after N_iter iterations (:126)."""
    t0 = time.perf_counter()
    res = MADSResult()
    x = np.asarray(input, dtype=np.float64).copy()
    n = x.size
    rng = SplitMix64(seed)
    cons = list(cons_ext)

    def feasible(v) -> bool:
        return all(bool(c(v)) for c in cons)

    cons3 = next((c for c in cons if hasattr(c, "prev")), None)
    others = [c for c in cons if c is not cons3]
    f = obj(x) if feasible(x) else np.inf
    res.status.function_evaluations += 1
    ell = ell0
    it = 0
    while it < N_iter and ell >= 0:
        it += 1
        B = ltmads_basis(n, ell, rng).astype(np.float64)
        X = np.concatenate([x[None, :] + B.T, x[None, :] - B.T], axis=0)
        n3 = sum(bool(cons3(v)) for v in X) if cons3 is not None else X.shape[0]
        res.status.cons3_passed += n3
        res.status.cons3_empty_polls += n3 == 0
        if hasattr(obj, "poll"):
            mask = np.array([all(bool(c(v)) for c in others) for v in X]) if others else None
            if mask is not None and not mask.any():
                bo, bi = np.inf, -1
            else:
                Xe = X if mask is None else X[mask]
                bo, bi, _ = obj.poll(Xe, cons3)
                if mask is not None and bi >= 0:
                    bi = int(np.flatnonzero(mask)[bi])
            res.status.function_evaluations += X.shape[0]
        else:
            bo, bi = np.inf, -1
            for k, v in enumerate(X):
                if not feasible(v):
                    continue
                fv = obj(v)
                res.status.function_evaluations += 1
                if fv < bo:
                    bo, bi = fv, k
        if bi >= 0 and bo < f:
            x, f = X[bi].copy(), bo
            ell = min(ell + 1, ell_max)
            res.status.successes += 1
        else:
            ell -= 1
    res.status.iteration = it
    res.status.runtime_total = time.perf_counter() - t0
    res.status.optimization_status = "MeshPrecisionLimit" if ell < 0 else "IterationLimit"
    if np.isfinite(f):
        res.x, res.x_cost = x, f
    else:
        res.i = x
    return res


class PollStepper:
    """Host mirror of the native stepper (mac_mads_begin / _poll / _update, include/maxcover.h),
    driven by ``dist.mads_loop``: the poll sequence of ``mads`` (same stream, same update rule),
    of which this stepper evaluates only the shard [lo, hi) of every poll's 2n candidates, through
    ``poll_fn(X_shard) -> (best_obj, best_local_index)`` (index -1: nothing feasible). Every rank
    draws the whole basis, so all ranks stay at the same stream position."""

    def __init__(self, x0, f0: float, poll_fn, N_iter: int = 100, ell0: int = 2,
                 ell_max: int = 6, seed: int = 20250216, shard=None):
        self.x = np.asarray(x0, dtype=np.float64).copy()
        self.n = self.x.size
        self.f = float(f0)
        self.poll_fn = poll_fn
        self.N_iter, self.ell, self.ell_max = N_iter, ell0, ell_max
        self.rng = SplitMix64(seed)
        self.it = 0
        self.evals = 1
        self.lo, self.hi = (0, 2 * self.n) if shard is None else (int(shard[0]), int(shard[1]))
        self._X = None

    def poll(self):
        if self.it >= self.N_iter or self.ell < 0:
            return True, np.inf, -1
        self.it += 1
        B = ltmads_basis(self.n, self.ell, self.rng).astype(np.float64)
        self._X = np.concatenate([self.x[None, :] + B.T, self.x[None, :] - B.T], axis=0)
        Xs = self._X[self.lo:self.hi]
        if Xs.shape[0] == 0:
            return False, np.inf, -1
        bo, bi = self.poll_fn(Xs)
        return False, float(bo), (self.lo + int(bi) if bi >= 0 else -1)

    def update(self, best_obj: float, best_idx: int) -> None:
        self.evals += 2 * self.n
        if best_idx >= 0 and best_obj < self.f:
            self.x = self._X[best_idx].copy()
            self.f = float(best_obj)
            self.ell = min(self.ell + 1, self.ell_max)
        else:
            self.ell -= 1

    # speculation over failure branches (mac_mads_poll_ahead / mac_mads_advance)
    def _draws(self) -> int:
        n = self.n
        return n + n * (n - 1) // 2 + 2 * n   # ltmads_basis's stream values per iteration

    def _poll_matrix(self, ahead: int):
        rng = SplitMix64()
        with np.errstate(over="ignore"):
            rng.state = self.rng.state + np.uint64(ahead * self._draws()) * np.uint64(0x9E3779B97F4A7C15)
        B = ltmads_basis(self.n, self.ell - ahead, rng).astype(np.float64)
        return np.concatenate([self.x[None, :] + B.T, self.x[None, :] - B.T], axis=0)

    def poll_ahead(self, ahead: int):
        """(done, best_obj, best_idx, feasible): feasible is not tracked here (0)."""
        if self.it + ahead >= self.N_iter or self.ell - ahead < 0:
            return True, np.inf, -1, 0
        Xs = self._poll_matrix(ahead)[self.lo:self.hi]
        if Xs.shape[0] == 0:
            return False, np.inf, -1, 0
        bo, bi = self.poll_fn(Xs)
        return False, float(bo), (self.lo + int(bi) if bi >= 0 else -1), 0

    def advance(self, best_obj: float, best_idx: int) -> bool:
        X = self._poll_matrix(0)
        self.rng.next_u64(self._draws())   # the iteration's stream values
        self.it += 1
        self.evals += 2 * self.n
        if best_idx >= 0 and best_obj < self.f:
            self.x = X[best_idx].copy()
            self.f = float(best_obj)
            self.ell = min(self.ell + 1, self.ell_max)
            return True
        self.ell -= 1
        return False

    def result(self):
        return self.x.copy(), {"f": self.f, "iterations": self.it, "evaluations": self.evals,
                               "status": 0 if self.ell < 0 else 1}


def optimize(input, obj, cons_ext, cons_prog, N_iter: int):
    """src/TDM_STATIC_opt.jl:118-222: returns (p.x if feasible else p.i, runtime_total)."""
    p = mads(input, obj, cons_ext, N_iter)
    result = p.i if p.x is None else p.x                # :165-169
    return result, p.status.runtime_total               # :219-220
