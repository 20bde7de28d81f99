"""CPU: the whole-poll cons3 rejection (k_prep.h diag_rejects, used by maxcover.hip poll_rejected
on the host and by the prep launch on the device) is exact: whenever every variable's diagonal
step +-2^ell alone puts its UAV's own cons3 term above the threshold, the C oracle's cons3
(src/TDM_Constraints.jl:54-75, oracle/ref_cpu.c ref_cons3) rejects every candidate of the
LTMADS poll, for any permutations and lower entries. The numpy form below restates diag_rejects
operation for operation (no FMA: numpy float64 scalar ops round each step)."""
import math

import numpy as np
import pytest

TAN50 = math.tan(100 / 180 * math.pi / 2)


def dlim_threshold(d):
    """predicate.h dlim_threshold: the largest s with fl(sqrt(s)) <= d."""
    d = float(d)
    if d != d or math.isinf(d):
        return math.inf
    if d < 0:
        return -1.0
    s = d * d
    while math.sqrt(s) > d:
        s = np.nextafter(s, -np.inf)
    while True:
        t = np.nextafter(s, np.inf)
        if math.sqrt(t) <= d:
            s = t
        else:
            break
    return float(s)


def diag_rejects(v, b, p, q, tan, T3):
    for c in (v + b, v - b):
        if q < 2:
            d = p - c
        else:
            d = p / tan - c / tan
        if not (d * d > T3):
            return False
    return True


def poll_rejected(x, prev, d_lim, tan, b):
    n = x.size
    N = n // 3
    return all(diag_rejects(float(x[v]), float(b), float(prev[v]), v // N, tan,
                            dlim_threshold(d_lim[v % N])) for v in range(n))


def test_rejection_implies_every_candidate_fails(pkg, orc):
    wl = pkg.workloads
    rng = wl.SplitMix64(4242)
    N = 7
    seen = 0
    for trial in range(120):
        prev = np.concatenate([np.round(500 + rng.uniform(N) * 300),
                               np.round(500 + rng.uniform(N) * 300), np.full(N, 30.0)])
        d_lim = np.full(N, 10.0) if trial % 2 == 0 else 6.0 + rng.uniform(N) * 8.0
        # an incumbent inside cons3 (small integer moves), or off it
        x = prev + np.round((rng.uniform(3 * N) - 0.5) * (4.0 if trial % 3 else 14.0))
        for ell in range(0, 7):
            B = wl.ltmads_basis(3 * N, ell, rng).astype(np.float64)
            X = np.concatenate([x[None, :] + B.T, x[None, :] - B.T], axis=0)
            if poll_rejected(x, prev, d_lim, TAN50, 2 ** ell):
                seen += 1
                feas = orc.cons3_batch(prev, X, d_lim, TAN50)
                assert not np.any(feas), (trial, ell)
    assert seen > 50


@pytest.mark.parametrize("ell", [5, 6])
def test_large_steps_always_rejected_from_a_feasible_incumbent(pkg, ell):
    """With d_lim = 10 and FOV 100 deg, a poll at ell >= 5 around any incumbent that itself
    passes cons3 is rejected whole (|e| <= 10 per axis, 2^ell - |e| > 10; radius: |e_r| <= 11.9,
    (2^ell - |e_r|) / tan > 10)."""
    wl = pkg.workloads
    rng = wl.SplitMix64(99 + ell)
    N = 9
    prev = np.concatenate([np.round(rng.uniform(N) * 800), np.round(rng.uniform(N) * 800),
                           np.full(N, 30.0)])
    d_lim = np.full(N, 10.0)
    for _ in range(50):
        u = rng.uniform(N) * 2 * math.pi
        rad = rng.uniform(N) * 10.0 / math.sqrt(3.0)
        x = prev.copy()
        x[:N] += np.round(rad * np.cos(u))
        x[N:2 * N] += np.round(rad * np.sin(u))
        x[2 * N:] += np.round((rng.uniform(N) - 0.5) * 10.0)
        assert poll_rejected(x, prev, d_lim, TAN50, 2 ** ell)


def test_small_steps_not_rejected(pkg):
    """ell = 0..2 from the incumbent prev itself: some candidate passes, nothing is skipped."""
    N = 5
    prev = np.concatenate([np.arange(N) * 50.0, np.arange(N) * 40.0, np.full(N, 30.0)])
    for ell in range(3):
        assert not poll_rejected(prev.copy(), prev, np.full(N, 10.0), TAN50, 2 ** ell)
