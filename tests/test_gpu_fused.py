"""GPU: the fused poll chain (k_fiw.h: prep -> fiw -> fin2) against the C oracle and the exact
lattice counts, and against the five-launch chain (prep, index, set-up, walk, finalize), each forced
with MAC_OPT_CHAIN. The fused chain decides ownership with superset boxes (candidate 0's disk and one
poll-wide displacement bound), the five-launch chain with the exact union regions: different entry
sets take the shared pass, the same entries are credited. Reference: src/AreaCoverageCalculation.jl
:63-78 (calculateArea), src/TDM_STATIC_opt.jl:82-100 (the objective), src/TDM_Constraints.jl:54-75
(cons3)."""
import math

import numpy as np
import pytest

from test_gpu_parity import _full_poll_check, recs
from test_gpu_parity import test_poll_walk_stress as _stress
from test_gpu_parity import test_cons3_failures_not_evaluated as _cons3
from test_gpu_parity import test_native_mads_pipelined_matches_stepper as _pipelined

pytestmark = pytest.mark.gpu
TAN50 = math.tan(100 / 180 * math.pi / 2)
CHAINS = ("fused", "five")


@pytest.fixture
def chain(ctx, request):
    ctx.set_chain(request.param)
    yield request.param
    ctx.set_chain("auto")
    ctx.set_algo("auto")


def _walks(ctx, C):
    """(areas, {kernel: launches}) of one batch: which chain ran."""
    ctx.profile(True)
    ctx.profile_read(reset=True)
    area = ctx.area_batch(C)
    kern = {k: n for k, (ms, n) in ctx.profile_kernels().items() if n}
    ctx.profile_read(reset=True)
    ctx.profile(False)
    return area, kern


@pytest.mark.parametrize("chain", CHAINS, indirect=True)
def test_config4_full_poll_chain(ctx, pkg, orc, chain):
    """The bench workload (512 UAVs x 16.8M cells, K = 3073) through each chain: every area == 25 x
    the exact lattice count, objectives and argmin bit-exact with and without cons3."""
    x, y, w, C, rmax = pkg.workloads.make_config(4)
    ctx.set_points(x, y, w)
    _full_poll_check(ctx, orc, C, rmax, 4096, ["poll"], "config4-" + chain)
    _, kern = _walks(ctx, C)
    assert ("fiw_kernel" in kern) == (chain == "fused"), kern


@pytest.mark.parametrize("chain", CHAINS, indirect=True)
def test_config4_clustered_full_poll_chain(ctx, pkg, orc, chain):
    """SURVEY 8(d)'s clustered variant at full size (most disks overlap lower-index ones: the fused
    chain's per-disk shared pass carries much of every area) through each chain."""
    x, y, w, C, rmax = pkg.workloads.make_config(4, disks="clustered")
    ctx.set_points(x, y, w)
    _full_poll_check(ctx, orc, C, rmax, 4096, ["poll"], "config4-clustered-" + chain)


@pytest.mark.parametrize("chain", CHAINS, indirect=True)
@pytest.mark.parametrize("disks", ["uniform", "clustered"])
def test_cons3_failures_chain(ctx, pkg, orc, chain, disks):
    """ell = 3 polls with about half the candidates failing cons3 (left out of the walks, +inf):
    through each chain (the fused chain's displacement bound covers the feasible candidates only)."""
    _cons3(ctx, pkg, orc, disks)


@pytest.mark.parametrize("chain", CHAINS, indirect=True)
@pytest.mark.parametrize("case", ["real_clustered", "big_radius", "mixed_weights", "pythagorean",
                                  "crowded", "lattice_mixed", "key_mix", "key_escape"])
def test_poll_walk_stress_chain(ctx, pkg, orc, chain, case):
    """The poll walk's rare paths (band decisions, ownership between overlapping disks, large
    regions, weights, escaped keys: the fused chain takes one position per candidate there) through
    each chain; test_gpu_parity.test_poll_walk_stress describes the cases."""
    _stress(ctx, pkg, orc, case)


@pytest.mark.parametrize("chain", CHAINS, indirect=True)
@pytest.mark.parametrize("N,n_iter,ell0,ell_max,cons3,stall", [
    (40, 60, 2, 5, True, False),
    (40, 200, 2, 4, False, True),
    (300, 25, 3, 6, True, False),
])
def test_native_mads_pipelined_chain(ctx, pkg, chain, N, n_iter, ell0, ell_max, cons3, stall):
    """The pipelined native MADS loop (generated candidates, device-side update) == the stepper,
    through each chain."""
    _pipelined(ctx, pkg, N, n_iter, ell0, ell_max, cons3, stall)


def test_fused_equals_five_on_mads_sequence(ctx, pkg):
    """A native MADS run under each forced chain: the same iterate, objective and counts bit for
    bit (the chains share no kernel past the prep)."""
    wl = pkg.workloads
    rng = wl.SplitMix64(5151)
    N = 64
    x, y, w = wl.grid_points(400)
    ctx.set_points(x, y, w)
    x0 = np.concatenate([np.round(300 + rng.uniform(N) * 1200), np.round(300 + rng.uniform(N) * 1200),
                         np.full(N, 30.0)])
    r_max = np.full(N, 30.0 * TAN50)
    kw = dict(prev=x0, d_lim=np.full(N, 10.0), tan_half_fov=TAN50, n_iter=40, ell0=2, ell_max=5,
              seed=77)
    out = {}
    try:
        for c in CHAINS:
            ctx.set_chain(c)
            out[c] = ctx.mads_run(x0, r_max, 1e5, **kw)
    finally:
        ctx.set_chain("auto")
    (xa, sa), (xb, sb) = out["fused"], out["five"]
    assert np.array_equal(xa, xb)
    for key in ("f", "iterations", "evaluations", "status", "feasible"):
        assert sa[key] == sb[key], key


def test_fused_nan_and_inf_candidates(ctx, pkg, orc):
    """Non-finite candidate values in a poll the fused chain takes (NaN / inf centres and radii,
    r <= 0): the displacement bound turns into a whole-grid box (NaN / inf differences), and every
    area and objective still equals the C oracle's."""
    wl = pkg.workloads
    rng = wl.SplitMix64(606)
    G, N = 200, 12
    x, y, w = wl.grid_points(G)
    ctx.set_points(x, y, w)
    x0 = wl.uniform_disks(N, G, rng)
    C = wl.poll_candidates(x0, rng)
    K = C.shape[0]
    C[5, 3] = np.nan
    C[9, N + 2] = np.inf
    C[11, 2 * N + 4] = np.nan
    C[13, 2 * N + 5] = -3.0
    C[17, 2 * N + 6] = np.inf
    C[21, 7] = -np.inf
    rmax = np.full(N, 30.0)
    rec = recs(x, y, w)
    want = orc.PointerList(rec).area_batch(C)
    want_obj = np.array([orc.ref_objective(c, rec, rmax) for c in C])
    ctx.set_chain("fused")
    try:
        got = ctx.area_batch(C)
        bo, bi, objs = ctx.poll_best(C, rmax, want_all=True)
    finally:
        ctx.set_chain("auto")
    assert np.array_equal(got, want), np.flatnonzero(got != want)[:5]
    assert np.array_equal(objs, want_obj, equal_nan=True)
    assert K >= 64


@pytest.mark.parametrize("extra", [-1, 0, 4, 11])
def test_fused_prep_candidate_remainders(ctx, pkg, orc, extra):
    """The fused chain's matrix-source prep takes 6 candidates per workgroup and hands the remainder
    K mod 6 to the first workgroups one each (k_prep.h prep_x_kernel): polls of K = 6N + 1 + extra
    candidates (extra < 0: the last dropped; > 0: shifted copies of the first appended), against
    the exact lattice counts, with and without cons3."""
    wl = pkg.workloads
    rng = wl.SplitMix64(4242 + extra)
    G, N = 600, 40
    x, y, w = wl.grid_points(G)
    ctx.set_points(x, y, w)
    x0 = wl.uniform_disks(N, G, rng)
    C = wl.poll_candidates(x0, rng)
    if extra < 0:
        C = C[:extra]
    elif extra > 0:
        add = C[1:1 + extra].copy()
        add[:, :N] += 1.0   # (integer shifts: still on the lattice's mesh)
        C = np.concatenate([C, add])
    K = C.shape[0]
    assert K == 6 * N + 1 + extra
    rmax = np.full(N, 30.0 * TAN50)
    ctx.set_chain("fused")
    try:
        _full_poll_check(ctx, orc, C, rmax, G, ["poll"], f"remainder{extra}")
        _, kern = _walks(ctx, C)
    finally:
        ctx.set_chain("auto")
    assert "fiw_kernel" in kern, kern


@pytest.mark.parametrize("chain", CHAINS, indirect=True)
def test_large_counts_overflow_the_16bit_rows(ctx, pkg, orc, chain):
    """Disks of R = 820 m on a 1024^2 grid at 5 m (about 84,000 entries each, more than a 16-bit
    row holds): the fused chain's count rows carry 0xFFFF and the 32-bit overflow row (k_fiw.h),
    and every area still equals 25 x the exact lattice count, with and without cons3, through
    each chain."""
    wl = pkg.workloads
    rng = wl.SplitMix64(4242)
    G, N = 1024, 16
    x, y, w = wl.grid_points(G)
    ctx.set_points(x, y, w)
    x0 = wl.uniform_disks(N, G, rng, radius=820.0)
    C = wl.poll_candidates(x0, rng, ell=2)
    assert C.shape[0] >= 64
    _full_poll_check(ctx, orc, C, np.full(N, 820.0), G, ["poll"], "r820-" + chain)
    _, kern = _walks(ctx, C)
    assert ("fiw_kernel" in kern) == (chain == "fused"), kern


@pytest.mark.parametrize("disks", ["clustered", "uniform"])
@pytest.mark.parametrize("where", ["device", "host"])
def test_first_matrix_poll_routes_from_the_poll(pkg, orc, disks, where):
    """A context's first matrix poll (DirectSearch's, handed over as a candidate matrix) routes
    from the poll before any chain has reported (maxcover.hip seed_route: candidate 0's disks
    overlap-tested on the host): a crowded incumbent (clustered disks) runs the five-launch chain
    from the first poll on — no fused launch — and an uncrowded one keeps the fused chain. The
    objectives equal the C oracle's either way."""
    import torch
    wl = pkg.workloads
    G, N = 512, 64
    x, y, w = wl.grid_points(G)
    rng = wl.SplitMix64(617 if disks == "clustered" else 618)
    x0 = (wl.clustered_disks if disks == "clustered" else wl.uniform_disks)(N, G, rng)
    C = wl.poll_candidates(x0, rng)
    r_max = np.full(N, 30.0 * TAN50)
    want = -orc.PointerList(recs(x, y, w)).area_batch(C) + orc.violation_batch(C, r_max) * 1e5
    with pkg.Context(0) as c2:   # (a fresh context: no routing history)
        c2.set_points(x, y, w)
        c2.profile(True)
        c2.profile_read(reset=True)
        if where == "host":
            _, _, obj = c2.poll_best(C, r_max, 1e5, want_all=True)
        else:
            dev = torch.device("cuda", 0)
            dC = torch.from_numpy(np.ascontiguousarray(C)).to(dev)
            dR = torch.from_numpy(r_max).to(dev)
            dB = torch.empty(2, dtype=torch.float64, device=dev)
            dO = torch.empty(C.shape[0], dtype=torch.float64, device=dev)
            c2.poll_best_dev(dC, 3 * N, C.shape[0], dR, dB, d_obj=dO)
            torch.cuda.synchronize()
            obj = dO.cpu().numpy()
        kern = {k: n for k, (ms, n) in c2.profile_kernels().items() if n}
    assert np.array_equal(obj, want)
    if disks == "clustered":
        assert "fiw_kernel" not in kern and kern.get("coverage_poll_kernel", 0) > 0, kern
    else:
        assert kern.get("fiw_kernel", 0) > 0, kern


@pytest.mark.parametrize("disks", ["clustered", "uniform"])
def test_native_mads_routes_from_the_poll(ctx, pkg, disks):
    """The native MADS driver routes its generated polls from the poll (maxcover.hip
    host_crowded_disks: the fused chain's superset boxes around the incumbent at the run's first
    mesh step): a crowded layout (clustered disks, many disks with lower-index neighbours) runs
    every poll through the five-launch chain from the first one — no fused launch, not even before
    AUTO's history exists — and an uncrowded one (uniform disks) keeps the fused chain. Both end on
    the same iterate as the same run forced through the five-launch chain."""
    wl = pkg.workloads
    G, N = 512, 64
    x, y, w = wl.grid_points(G)
    rng = wl.SplitMix64(515 if disks == "clustered" else 516)
    x0 = (wl.clustered_disks if disks == "clustered" else wl.uniform_disks)(N, G, rng)
    r_max = np.full(N, 30.0 * TAN50)
    kw = dict(prev=x0, d_lim=np.full(N, 10.0), tan_half_fov=TAN50, n_iter=20, ell0=2, ell_max=5, seed=77)
    with pkg.Context(0) as c2:   # (a fresh context: no routing history)
        c2.set_points(x, y, w)
        c2.profile(True)
        c2.profile_read(reset=True)
        xa, sa = c2.mads_run(x0, r_max, 1e5, **kw)
        kern = {k: n for k, (ms, n) in c2.profile_kernels().items() if n}
        c2.profile_read(reset=True)
        c2.set_chain("five")
        xb, sb = c2.mads_run(x0, r_max, 1e5, **kw)
    assert np.array_equal(xa, xb) and sa["f"] == sb["f"]
    if disks == "clustered":
        assert "fiw_kernel" not in kern and kern.get("coverage_poll_kernel", 0) > 0, kern
    else:
        assert kern.get("fiw_kernel", 0) > 0, kern
