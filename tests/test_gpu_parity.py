"""GPU parity: libmaxcover (HIP, gfx950) against the oracle, through the C-ABI.

Bar: bit-exact coverage decisions everywhere, and bit-exact areas/objectives whenever the
partial sums are exact (every reference input: weight 25.0 on every entry). For arbitrary real
weights the library sums in a fixed tile order instead of list order; the covered SET is still
checked exactly (mac_covered_flags_f64) and the area within rtol 1e-12 (north star: 1e-9 rel).
"""
import hashlib
import math
import threading

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

ALGOS = ("tiled", "scan", "poll")
TAN50 = math.tan(100 / 180 * math.pi / 2)


def recs(x, y, w):
    return np.stack([x, y, w * 2, w, np.zeros_like(x)], axis=1)


def both(ctx, fn):
    out = {}
    for a in ALGOS:
        ctx.set_algo(a)
        out[a] = fn()
    ctx.set_algo("auto")
    return out


# ---------------------------------------------------------------------------- golden vectors

def test_golden_static_grid(ctx, pkg, golden, orc):
    poi = pkg.AreaCoverageCalculation.createPOI(5.0, 5.0, 100.0, 100.0)
    ctx.set_points_records(poi)
    for a, got in both(ctx, lambda: ctx.area_batch(golden["A_cands"])).items():
        assert np.array_equal(got, golden["A_area"]), a
    for a, got in both(ctx, lambda: ctx.objective_batch(golden["A_cands"], golden["A_rmax"])).items():
        assert np.array_equal(got, golden["A_obj"]), a
    # poll with cons3 on the device == oracle's extreme barrier + argmin
    feas = golden["A_cons3"].astype(bool)
    want = np.where(feas, golden["A_obj"], np.inf)
    k = int(np.argmin(want))
    for a, (bo, bi, objs) in both(ctx, lambda: ctx.poll_best(
            golden["A_cands"], golden["A_rmax"], 1e5, prev=golden["A_prev"],
            d_lim=golden["A_dlim"], tan_half_fov=float(golden["A_tan"][0]), want_all=True)).items():
        assert np.array_equal(objs, want), a
        assert bi == k and bo == want[k], a


def test_reference_mads_outputs_device_cons3(ctx, pkg, orc, quadrotor_steps):
    """The reference's recorded MADS outputs (UAV 1 of its static N = 5 run, tests/golden/
    quadrotor_run.csv) through the device poll: per step, a batch of the target, the start and a
    point 10.5 m from the start, with prev = the step's start and d_lim = 10 m. The device's
    cons3 keeps the target and the start and rejects the far point (+inf), and the feasible
    objectives equal the oracle's on the reference static grid (createPOI(5, 5, 100, 100))."""
    steps, tan = quadrotor_steps
    poi = pkg.AreaCoverageCalculation.createPOI(5.0, 5.0, 100.0, 100.0)
    ctx.set_points_records(poi)
    rmax = np.array([30 * tan])
    for prev, tgt in steps:
        cand = np.array([tgt[0], tgt[1], float(round(tgt[2]))])
        far = np.array([prev[0] + 10.5, prev[1], prev[2]])
        C = np.stack([cand, prev, far])
        bo, bi, objs = ctx.poll_best(C, rmax, 1e5, prev=prev, d_lim=np.array([10.0]),
                                     tan_half_fov=tan, want_all=True)
        assert np.isinf(objs[2]) and objs[2] > 0
        for k in (0, 1):
            assert objs[k] == orc.ref_objective(C[k], poi, rmax), (k, objs[k])
        assert bi == int(np.argmin(objs[:2])) and bo == objs[bi]


def test_golden_firepoints(ctx, golden, firepoints):
    fp10 = np.concatenate(firepoints[:10])
    fpall = np.concatenate(firepoints)
    for rec, key in ((fp10, "B_area10"), (fpall, "B_area_all")):
        ctx.set_points_records(rec)
        for a, got in both(ctx, lambda: ctx.area_batch(golden["B_cands"])).items():
            assert np.array_equal(got, golden[key]), (a, key)


def test_golden_removal(ctx, pkg, golden, firepoints):
    poi = pkg.AreaCoverageCalculation.createPOI(5.0, 5.0, 100.0, 100.0)
    ctx.set_points_records(poi)
    kept = ctx.remove_covered(golden["A_rmv_cand"])
    assert np.array_equal(kept, golden["A_rmv_kept"])
    assert ctx.num_points == kept.size
    x, y, w = ctx.get_points()
    assert np.array_equal(x, poi[kept, 0]) and np.array_equal(y, poi[kept, 1])
    fpall = np.concatenate(firepoints)
    ctx.set_points_records(fpall)
    assert np.array_equal(ctx.remove_covered(golden["B_rmv_cand"]), golden["B_rmv_kept"])


def test_golden_synthetic_real_weights(ctx, pkg, golden, orc):
    wl = pkg.workloads
    rngC = wl.SplitMix64(303)
    M = 20000
    xc = rngC.uniform(M) * 400.0 - 50.0
    yc = rngC.uniform(M) * 300.0 + 10.0
    wc = rngC.uniform(M) * 10.0 + 0.5
    xc, yc, wc = wl.shuffled_with_duplicates(xc, yc, wc, rngC, 0.05)
    h = hashlib.sha256()
    for a in (xc, yc, wc):
        h.update(np.ascontiguousarray(a).tobytes())
    assert h.hexdigest() == str(golden["C_sha"][0]), "generator drifted from the fixture"
    ctx.set_points(xc, yc, wc)
    for a, got in both(ctx, lambda: ctx.area_batch(golden["C_cands"])).items():
        np.testing.assert_allclose(got, golden["C_area"], rtol=1e-12, atol=0, err_msg=a)
    for c in golden["C_cands"]:
        assert np.array_equal(ctx.covered_flags(c), orc.np_covered(c, xc, yc))


def test_golden_lattice_kats(ctx, pkg, golden):
    x, y, w = pkg.workloads.grid_points(64)
    ctx.set_points(x, y, w)
    for k, c in enumerate(golden["D_cands"]):
        cc = c[: 3 * int(golden["D_N"][k])]
        for a, got in both(ctx, lambda: ctx.area(cc)).items():
            assert got == 25.0 * golden["D_count"][k], (a, k)


# ---------------------------------------------------------------------------- edge cases

def test_empty_and_size_errors(ctx, pkg):
    ctx.set_points(np.zeros(0), np.zeros(0), np.zeros(0))
    for a in ALGOS:
        ctx.set_algo(a)
        assert ctx.area(np.array([1.0, 2.0, 3.0])) == 0.0
        assert np.array_equal(ctx.area_batch(np.zeros((3, 6))), np.zeros(3))
    ctx.set_algo("auto")
    assert ctx.remove_covered(np.array([0.0, 0.0, 10.0])).size == 0
    x, y, w = pkg.workloads.grid_points(10)
    ctx.set_points(x, y, w)
    assert ctx.area(np.zeros(0)) == 0.0          # no UAV: nothing covered
    with pytest.raises(pkg.InexactError):
        ctx.area(np.zeros(4))                   # Int(4/3): InexactError
    assert ctx.area_batch(np.zeros((0, 6))).size == 0


def test_special_values(ctx, orc):
    x = np.array([0.0, 1.0, np.nan, np.inf, -np.inf, 2.0, 2.0, 1e300, -3.0, 0.5])
    y = np.array([0.0, 1.0, 1.0, 0.0, 5.0, np.nan, 2.0, 0.0, -3.0, 0.25])
    w = np.array([1.0, 2.0, 4.0, 8.0, 16.0, 32.0, 64.0, 128.0, 256.0, 512.0])
    ctx.set_points(x, y, w)
    rec = recs(x, y, w)
    cases = [
        [0.0, 0.0, 1.5],                       # plain
        [0.0, 0.0, math.sqrt(2.0)],            # point (1,1) exactly on the boundary
        [0.0, 0.0, np.inf],                    # infinite radius: every finite point
        [0.0, 0.0, 0.0], [0.0, 0.0, -1.0],     # covers nothing
        [np.nan, 0.0, 5.0], [0.0, 0.0, np.nan],
        [np.inf, 0.0, 5.0],
        [1.0, 1.0, 1e308],                     # huge finite radius
        [0.0, 1.0, 0.0, 1.0, 1.0, 1.0],        # two disks, overlapping
        [0.0, 0.0, 0.0, 0.0, 2.0, 2.0],        # identical disks
        [0.5, -3.0, 0.25, -3.0, 5e-324, 1e-300],
    ]
    for c in cases:
        c = np.array(c, dtype=float)
        want = orc.ref_area(c, rec)
        for a, got in both(ctx, lambda: ctx.area(c)).items():
            assert got == want, (a, c, got, want)
        assert np.array_equal(ctx.covered_flags(c), orc.np_covered(c, x, y)), c


def test_degenerate_point_sets(ctx, orc):
    rng = np.random.default_rng(9)
    sets = [
        (np.full(500, 3.0), np.full(500, 4.0)),                    # all entries identical
        (np.linspace(0, 100, 700), np.full(700, 7.0)),             # collinear (H = 0)
        (np.full(300, -2.0), np.linspace(-50, 50, 300)),           # collinear (W = 0)
        (np.array([1.0]), np.array([1.0])),                        # single entry
        (rng.normal(0, 1e6, 2000), rng.normal(0, 1e-3, 2000)),     # extreme aspect ratio
    ]
    for x, y in sets:
        w = np.full(x.size, 25.0)
        ctx.set_points(x, y, w)
        rec = recs(x, y, w)
        for _ in range(5):
            N = int(rng.integers(1, 6))
            c = np.concatenate([rng.choice(x, N) + rng.normal(0, 2, N),
                                rng.choice(y, N) + rng.normal(0, 2, N), rng.uniform(0, 20, N)])
            want = orc.ref_area(c, rec)
            for a, got in both(ctx, lambda: ctx.area(c)).items():
                assert got == want, (a, c)


# ---------------------------------------------------------------------------- fuzz

@pytest.mark.parametrize("seed", range(12))
def test_fuzz_vs_oracle(ctx, pkg, orc, seed):
    wl = pkg.workloads
    rng = wl.SplitMix64(1000 + seed)
    lattice = seed % 2 == 0
    if lattice:
        G = int(rng.integers(8, 120, 1)[0])
        x, y, w = wl.grid_points(G)
        x, y, w = wl.shuffled_with_duplicates(x, y, w, rng, 0.05)
    else:
        M = int(rng.integers(1, 30000, 1)[0])
        x = rng.uniform(M) * 500 - 100
        y = rng.uniform(M) * 300
        w = np.full(M, 25.0)
    ctx.set_points(x, y, w)
    rec = recs(x, y, w)
    N = int(rng.integers(1, 300, 1)[0])
    span = float(np.nanmax(x) - np.nanmin(x)) + 10
    x0 = np.concatenate([np.round(rng.uniform(N) * span), np.round(rng.uniform(N) * 300),
                         np.round(rng.uniform(N) * 40)])
    K = int(rng.integers(1, 40, 1)[0])
    C = np.concatenate([x0[None, :], wl.poll_candidates(x0, rng, ell=2)[: K - 1]], axis=0)
    want = orc.PointerList(rec).area_batch(C)
    for a, got in both(ctx, lambda: ctx.area_batch(C)).items():
        assert np.array_equal(got, want), (a, seed, np.flatnonzero(got != want)[:5])


def test_many_uavs_single_candidate(ctx, pkg, orc):
    """N = 2100 UAVs, above the per-candidate walk's LDS limit (2048 disks): AUTO and 'tiled' take
    the poll walk (one workgroup per disk; K = 1), 'scan' the brute force; all == the oracle."""
    wl = pkg.workloads
    rng = wl.SplitMix64(55)
    x, y, w = wl.grid_points(60)
    ctx.set_points(x, y, w)
    N = 2100   # above the tiled kernel's LDS limit
    c = np.concatenate([rng.uniform(N) * 300, rng.uniform(N) * 300, rng.uniform(N) * 3])
    for a, got in both(ctx, lambda: ctx.area(c)).items():
        assert got == orc.ref_area(c, recs(x, y, w)), a


def test_determinism_and_slicing(ctx, pkg):
    """Same inputs -> bit-identical results; the multi-workgroup-per-candidate path (small K)
    equals the one-workgroup path (large K)."""
    wl = pkg.workloads
    rng = wl.SplitMix64(8)
    x, y, w = wl.grid_points(300)
    ctx.set_points(x, y, w)
    x0 = wl.clustered_disks(64, 300, rng)
    C = wl.poll_candidates(x0, rng)
    ctx.set_algo("tiled")
    a1 = ctx.area_batch(C)
    a2 = ctx.area_batch(C)
    singles = np.array([ctx.area(c) for c in C[:20]])
    ctx.set_algo("auto")
    assert np.array_equal(a1, a2)
    assert np.array_equal(a1[:20], singles)


def test_concurrent_host_threads(ctx, pkg):
    wl = pkg.workloads
    rng = wl.SplitMix64(21)
    x, y, w = wl.grid_points(200)
    ctx.set_points(x, y, w)
    x0 = wl.uniform_disks(20, 200, rng)
    C = wl.poll_candidates(x0, rng)
    want = ctx.area_batch(C)
    res = {}

    def run(t):
        res[t] = [ctx.area_batch(C[t::4]) for _ in range(5)]

    th = [threading.Thread(target=run, args=(t,)) for t in range(4)]
    for t in th:
        t.start()
    for t in th:
        t.join()
    for t in range(4):
        for r in res[t]:
            assert np.array_equal(r, want[t::4])


@pytest.mark.parametrize("threads", [2, 16])
def test_concurrent_closure_calls(ctx, pkg, orc, threads):
    """mac_area_f64 (the single-candidate closure) from many host threads at once, as
    DirectSearch's threaded poll calls it (src/TDM_STATIC_opt.jl:129): concurrent calls are combined
    into one batched closure launch (maxcover.hip ClReq), and every call still returns its own
    candidate's area, equal to the C oracle's, for mixed disk counts and repeated candidates."""
    wl = pkg.workloads
    rng = wl.SplitMix64(2100 + threads)
    x, y, w = wl.grid_points(220)
    ctx.set_points(x, y, w)
    polls = []
    for N in (12, 12, 7):   # two threads' worth of N = 12 and one of N = 7: batches by size
        x0 = wl.uniform_disks(N, 220, rng)
        polls.append(wl.poll_candidates(x0, rng)[:24])
    rec = recs(x, y, w)
    pl = orc.PointerList(rec)
    want = [pl.area_batch(C) for C in polls]
    errs = []

    def run(t):
        C, A = polls[t % 3], want[t % 3]
        for rep in range(6):
            for k in range(t % 5, C.shape[0], 5):
                got = ctx.area(np.ascontiguousarray(C[k]))
                if got != A[k]:
                    errs.append((t, k, got, A[k]))

    th = [threading.Thread(target=run, args=(t,)) for t in range(threads)]
    for h in th:
        h.start()
    for h in th:
        h.join()
    assert not errs, errs[:5]


def test_closure_bar_and_copy_paths_agree(pkg, orc):
    """The closure's two ways in (maxcover.hip closure_launch): candidates written by the host
    straight into fine-grained device memory through the BAR (the default on a large-BAR device)
    and pinned staging + a copy (MAXCOVER_CL_BAR=0, read at context creation). Same areas, equal to
    the C oracle's, for several disk counts and weighted entries, from one thread and from eight at
    once (combined batches)."""
    import os
    import threading
    wl = pkg.workloads
    rng = wl.SplitMix64(4242)
    x, y, w = wl.grid_points(180)
    w = w * (1.0 + (np.arange(w.size) % 7) / 8.0)   # weighted: the fp64 credit path
    rec = recs(x, y, w)
    pl = orc.PointerList(rec)
    polls = [wl.poll_candidates(wl.uniform_disks(N, 180, rng), rng)[:16] for N in (5, 17, 40)]
    want = [pl.area_batch(C) for C in polls]
    got = {}
    for bar in ("1", "0"):
        old = os.environ.get("MAXCOVER_CL_BAR")
        os.environ["MAXCOVER_CL_BAR"] = bar
        try:
            c = pkg.Context(0)
        finally:
            if old is None:
                del os.environ["MAXCOVER_CL_BAR"]
            else:
                os.environ["MAXCOVER_CL_BAR"] = old
        try:
            c.set_points(x, y, w)
            single = [np.array([c.area(np.ascontiguousarray(C[k])) for k in range(C.shape[0])])
                      for C in polls]
            res = {}

            def run(t):
                C = polls[t % 3]
                res[t] = [c.area(np.ascontiguousarray(C[k])) for k in range(t % 2, C.shape[0], 2)]

            th = [threading.Thread(target=run, args=(t,)) for t in range(8)]
            for h in th:
                h.start()
            for h in th:
                h.join()
            got[bar] = (single, res)
        finally:
            c.close()
    for bar, (single, res) in got.items():
        for j, C in enumerate(polls):
            assert np.array_equal(single[j], want[j]), (bar, j)
        for t, vals in res.items():
            assert np.array_equal(np.array(vals), want[t % 3][t % 2::2]), (bar, t)


# ---------------------------------------------------------------------------- device API

def test_device_pointer_api(ctx, pkg, orc):
    import torch
    wl = pkg.workloads
    rng = wl.SplitMix64(31)
    x, y, w = wl.grid_points(150)
    dev = torch.device("cuda", ctx.device)
    tx, ty, tw = (torch.from_numpy(a).to(dev) for a in (x, y, w))
    ctx.set_points_device(tx, ty, tw)
    x0 = wl.uniform_disks(10, 150, rng)
    C = wl.poll_candidates(x0, rng)
    rmax = np.full(10, 36.0)
    tC = torch.from_numpy(C).to(dev)
    tA = torch.empty(C.shape[0], dtype=torch.float64, device=dev)
    s = torch.cuda.current_stream(dev)
    ctx.area_batch_dev(tC, C.shape[1], C.shape[0], tA, stream=s.cuda_stream)
    tR = torch.from_numpy(rmax).to(dev)
    tB = torch.empty(2, dtype=torch.float64, device=dev)
    tO = torch.empty(C.shape[0], dtype=torch.float64, device=dev)
    ctx.poll_best_dev(tC, C.shape[1], C.shape[0], tR, tB, idx_base=100, d_obj=tO,
                      stream=s.cuda_stream)
    torch.cuda.synchronize(dev)
    rec = recs(x, y, w)
    want = orc.PointerList(rec).area_batch(C)
    assert np.array_equal(tA.cpu().numpy(), want)
    wobj = np.array([orc.ref_objective(c, rec, rmax) for c in C])
    assert np.array_equal(tO.cpu().numpy(), wobj)
    b = tB.cpu()
    assert b[0].item() == wobj.min() and b.view(torch.int64)[1].item() == 100 + int(np.argmin(wobj))
    # the host side of a poll step: mirrored result of the latest poll, then the copy fallback
    # (another buffer), then a new poll on other candidates through the mirror again
    assert ctx.best_fetch(tB, stream=s.cuda_stream) == (wobj.min(), 100 + int(np.argmin(wobj)))
    tB2 = tB.clone()
    torch.cuda.synchronize(dev)
    assert ctx.best_fetch(tB2, stream=s.cuda_stream) == (wobj.min(), 100 + int(np.argmin(wobj)))
    C2 = C[::-1].copy()
    ctx.poll_best_dev(torch.from_numpy(C2).to(dev), C.shape[1], C.shape[0], tR, tB,
                      stream=s.cuda_stream)
    w2 = wobj[::-1]
    assert ctx.best_fetch(tB, stream=s.cuda_stream) == (w2.min(), int(np.argmin(w2)))
    # the bound poll step (bench.py's loop): same result, repeatable, alternating sets
    tC2 = torch.from_numpy(C2).to(dev)
    st1 = ctx.poll_step(tC, C.shape[1], C.shape[0], tR, tB, idx_base=100, stream=s.cuda_stream)
    st2 = ctx.poll_step(tC2, C.shape[1], C.shape[0], tR, tB, stream=s.cuda_stream)
    for _ in range(3):
        assert st1() == (wobj.min(), 100 + int(np.argmin(wobj)))
        assert st2() == (w2.min(), int(np.argmin(w2)))


def test_null_stream_orders_after_default_stream_producer(ctx, pkg, orc):
    """A caller that writes d_cands with torch ops on the default stream — queued behind a long
    default-stream job, so the candidates land late — and then polls with stream=None and fetches
    with stream=None, with no synchronisation anywhere: every poll reads the candidates the
    default stream wrote (NULL / None = HIP's null stream, ordered with torch's default stream;
    include/maxcover.h). Checked against the oracle's objectives."""
    import torch
    wl = pkg.workloads
    rng = wl.SplitMix64(93)
    x, y, w = wl.grid_points(160)
    ctx.set_points(x, y, w)
    dev = torch.device("cuda", ctx.device)
    torch.cuda.synchronize(dev)
    assert torch.cuda.current_stream(dev).cuda_stream == 0
    rec = recs(x, y, w)
    N = 12
    rmax = np.full(N, 35.0)
    tR = torch.from_numpy(rmax).to(dev)
    tB = torch.empty(2, dtype=torch.float64, device=dev)
    big = torch.randn(4096, 4096, device=dev)
    for t in range(4):
        C = wl.poll_candidates(wl.uniform_disks(N, 160, rng), rng)
        wobj = np.array([orc.ref_objective(c, rec, rmax) for c in C])
        src = torch.from_numpy(C).pin_memory()
        tC = torch.zeros(C.shape, dtype=torch.float64, device=dev)
        for _ in range(3):
            big = big @ big.T / 4096.0                # keeps the default stream busy
        tC.copy_(src, non_blocking=True)               # lands after the matmuls
        tC.add_(big[0, 0] * 0.0)                       # a dependent kernel on the default stream
        ctx.poll_best_dev(tC, 3 * N, C.shape[0], tR, tB)
        got = ctx.best_fetch(tB)
        k = int(np.argmin(wobj))
        assert got == (wobj[k], k), (t, got, (wobj[k], k))
        del tC                                         # (freed after the poll: stream order)


def test_concurrent_device_polls(ctx, pkg, orc):
    """Two host threads, each with its own stream and d_best, issue mac_poll_best_dev_f64 +
    mac_best_fetch on one context (DirectSearch SetMaxEvals, src/TDM_STATIC_opt.jl:129): every
    fetched result equals the oracle's argmin of the poll that thread issued (each d_best has its
    own mapped result slot, include/maxcover.h mac_best_fetch)."""
    import torch
    wl = pkg.workloads
    rng = wl.SplitMix64(77)
    x, y, w = wl.grid_points(160)
    ctx.set_points(x, y, w)
    dev = torch.device("cuda", ctx.device)
    rec = recs(x, y, w)
    rmax = np.full(12, 35.0)
    tR = torch.from_numpy(rmax).to(dev)
    polls = []
    for _ in range(4):
        C = wl.poll_candidates(wl.uniform_disks(12, 160, rng), rng)
        wobj = np.array([orc.ref_objective(c, rec, rmax) for c in C])
        polls.append((torch.from_numpy(C).to(dev), wobj))
    errs = []

    def run(t):
        try:
            s = torch.cuda.Stream(dev)
            tB = torch.empty(2, dtype=torch.float64, device=dev)
            for it in range(12):
                tC, wobj = polls[(t + it) % len(polls)]
                ctx.poll_best_dev(tC, tC.shape[1], tC.shape[0], tR, tB, idx_base=1000 * t,
                                  stream=s.cuda_stream)
                got = ctx.best_fetch(tB, stream=s.cuda_stream)
                k = int(np.argmin(wobj))
                if got != (wobj[k], 1000 * t + k):
                    errs.append((t, it, got, (wobj[k], 1000 * t + k)))
        except Exception as e:  # surfaced below
            errs.append((t, repr(e)))

    th = [threading.Thread(target=run, args=(t,)) for t in range(2)]
    for t in th:
        t.start()
    for t in th:
        t.join()
    assert not errs, errs[:4]


def test_best_fetch_then_other_stream(ctx, pkg, orc):
    """mac_best_fetch's contract: once it returns, d_best holds the result for device work, and
    work ordered after `stream` (an event) reads it from another stream."""
    import torch
    wl = pkg.workloads
    rng = wl.SplitMix64(78)
    x, y, w = wl.grid_points(120)
    ctx.set_points(x, y, w)
    dev = torch.device("cuda", ctx.device)
    C = wl.poll_candidates(wl.uniform_disks(8, 120, rng), rng)
    rmax = np.full(8, 35.0)
    wobj = np.array([orc.ref_objective(c, recs(x, y, w), rmax) for c in C])
    k = int(np.argmin(wobj))
    s1, s2 = torch.cuda.Stream(dev), torch.cuda.Stream(dev)
    tC = torch.from_numpy(C).to(dev)
    tR = torch.from_numpy(rmax).to(dev)
    tB = torch.empty(2, dtype=torch.float64, device=dev)
    for _ in range(3):
        ctx.poll_best_dev(tC, C.shape[1], C.shape[0], tR, tB, stream=s1.cuda_stream)
        assert ctx.best_fetch(tB, stream=s1.cuda_stream) == (wobj[k], k)
        ev = torch.cuda.Event()
        ev.record(s1)
        s2.wait_event(ev)
        with torch.cuda.stream(s2):
            copy = tB.clone()
        s2.synchronize()
        assert copy[0].item() == wobj[k] and copy.view(torch.int64)[1].item() == k
        tB.fill_(0.0)   # (on the current stream: ordered before the next poll by the sync)
        torch.cuda.synchronize(dev)


# ---------------------------------------------------------------------------- full size

def test_config2_full_size(ctx, pkg, orc):
    """32 UAVs x 1,048,576 cells fp64: both kernels == the C oracle == integer lattice count."""
    x, y, w, C, rmax = pkg.workloads.make_config(2)
    ctx.set_points(x, y, w)
    want = orc.PointerList(recs(x, y, w)).area_batch(C)
    assert want[0] == 25.0 * orc.lattice_count_fast(C[0].astype(np.int64), 1024)
    for a, got in both(ctx, lambda: ctx.area_batch(C)).items():
        assert np.array_equal(got, want), a
    kept = ctx.remove_covered(C[0])
    assert np.array_equal(kept, orc.ref_remove_covered(C[0], recs(x, y, w)))


def test_config3_full_poll(ctx, pkg, orc):
    """128 UAVs x 4M cells, K=769: tiled == scan on every candidate; lattice KAT on a sample."""
    x, y, w, C, rmax = pkg.workloads.make_config(3)
    ctx.set_points(x, y, w)
    r = both(ctx, lambda: ctx.area_batch(C))
    assert np.array_equal(r["tiled"], r["scan"])
    for k in range(0, C.shape[0], 97):
        assert r["tiled"][k] == 25.0 * orc.lattice_count_fast(C[k].astype(np.int64), 2048), k
    pen = np.array([sum(abs(float(c[256 + i]) - float(rmax[i])) for i in range(128)) for c in C])
    wobj = -r["scan"] + pen * 1e5
    # cons3 around the incumbent with d_lim = 5 m: a mix of feasible and infeasible moves
    tan = float(np.tan(100 / 180 * np.pi / 2))
    dlim = np.full(128, 5.0)
    feas = np.array([orc.ref_cons3(C[0], c, dlim, tan) for c in C])
    assert 0 < feas.sum() < C.shape[0]
    wbar = np.where(feas, wobj, np.inf)
    for a, (bo, bi, objs) in both(ctx, lambda: ctx.poll_best(C, rmax, want_all=True)).items():
        assert np.array_equal(objs, wobj) and bi == int(np.argmin(wobj)), a
    for a, (bo, bi, objs) in both(ctx, lambda: ctx.poll_best(
            C, rmax, 1e5, prev=C[0], d_lim=dlim, tan_half_fov=tan, want_all=True)).items():
        assert np.array_equal(objs, wbar) and bi == int(np.argmin(wbar)) and bo == wbar[bi], a


def _full_poll_check(ctx, orc, C, rmax, G, algos, tag):
    """Every candidate of a full poll against the exact integer lattice count, through every
    listed walk; objectives (-25*count + 1e5*sequential violation) and the argmin bit-exact,
    without and with cons3 (d_lim = 10 m around the incumbent, src/FullSimulation.jl:740)."""
    cnt = orc.lattice_count_batch(C, G)
    want_area = 25.0 * cnt.astype(np.float64)
    want_obj = -want_area + orc.violation_batch(C, rmax) * 1e5
    tan = float(np.tan(100 / 180 * np.pi / 2))
    dlim = np.full(C.shape[1] // 3, 10.0)
    feas = orc.cons3_batch(C[0], C, dlim, tan)
    want_bar = np.where(feas, want_obj, np.inf)
    for a in algos:
        ctx.set_algo(a)
        got = ctx.area_batch(C)
        bad = np.flatnonzero(got != want_area)
        assert bad.size == 0, (tag, a, bad[:5], got[bad[:5]], want_area[bad[:5]])
        bo, bi, objs = ctx.poll_best(C, rmax, want_all=True)
        assert np.array_equal(objs, want_obj), (tag, a, np.flatnonzero(objs != want_obj)[:5])
        k = int(np.argmin(want_obj))
        assert bi == k and bo == want_obj[k], (tag, a, bi, k)
        bo, bi, objs = ctx.poll_best(C, rmax, 1e5, prev=C[0], d_lim=dlim, tan_half_fov=tan,
                                     want_all=True)
        assert np.array_equal(objs, want_bar), (tag, a)
        k = int(np.argmin(want_bar))
        assert bi == k and bo == want_bar[k], (tag, a, bi, k)
    ctx.set_algo("auto")
    return cnt


@pytest.mark.parametrize("algo", ["auto", "poll", "tiled"])
def test_config4_full_poll(ctx, pkg, orc, algo):
    """512 UAVs x 16.8M cells, K=3073 — the bench workload, through the walk the bench times
    (auto = the poll walk for K >= 64) and the others: all 3073 areas == 25 x the exact integer
    lattice count, objectives and argmin bit-exact (with and without cons3); the streaming scan
    agrees on a sample."""
    x, y, w, C, rmax = pkg.workloads.make_config(4)
    ctx.set_points(x, y, w)
    cnt = _full_poll_check(ctx, orc, C, rmax, 4096, [algo], "config4")
    if algo == "auto":
        ctx.set_algo("scan")
        got_scan = ctx.area_batch(C[::384])
        ctx.set_algo("auto")
        assert np.array_equal(got_scan, 25.0 * cnt[::384])


@pytest.mark.parametrize("disks", ["uniform", "clustered"])
def test_cons3_failures_not_evaluated(ctx, pkg, orc, disks):
    """A poll at mesh step 8 (ell = 3): about half of the LTMADS candidates move some UAV more
    than d_lim and fail cons3. With cons3 the prep leaves the failures out of the regions and the
    index maps them to one inert position (k_prep.h, k_index.h): the feasible candidates'
    objectives are still bit-exact (exact lattice counts) and the failures +inf, through every
    walk; without cons3 (and for area_batch) nothing is left out."""
    wl = pkg.workloads
    rng = wl.SplitMix64(3003 if disks == "uniform" else 3004)
    G, N = 512, 128
    x, y, w = wl.grid_points(G)
    ctx.set_points(x, y, w)
    x0 = (wl.uniform_disks if disks == "uniform" else wl.clustered_disks)(N, G, rng)
    C = wl.poll_candidates(x0, rng, ell=3)
    feas = orc.cons3_batch(C[0], C, np.full(N, 10.0), TAN50)
    assert 0 < int(feas.sum()) < C.shape[0], int(feas.sum())
    _full_poll_check(ctx, orc, C, np.full(N, 30.0 * TAN50), G, ["auto", "poll", "tiled"],
                     "ell3-" + disks)


@pytest.mark.parametrize("N", [600, 2100])
def test_many_uav_full_poll_auto(ctx, pkg, orc, N):
    """Polls past config 4's shape (src/TDM_STATIC_opt.jl:123: n = 3N, no cap). N = 600: K = 3601
    takes the wide disk index (6 candidates per thread, K <= 6145); N = 2100: K = 12601 takes the
    identity map and the poll walk (more disks than the per-candidate walk holds). AUTO through
    the device poll: sampled candidates == 25 x the exact lattice count; every objective ==
    -area + 1e5 x the sequential violation of the reported area; the argmin of those."""
    wl = pkg.workloads
    rng = wl.SplitMix64(600 + N)
    G = 1024
    x, y, w = wl.grid_points(G)
    ctx.set_points(x, y, w)
    x0 = wl.uniform_disks(N, G, rng)
    C = wl.poll_candidates(x0, rng)
    K = C.shape[0]
    assert K == 6 * N + 1
    rmax = np.full(N, 30.0 * TAN50)
    ctx.set_algo("auto")
    area = ctx.area_batch(C)
    pick = np.unique(np.concatenate([[0, K - 1], np.floor(rng.uniform(24) * K).astype(np.int64)]))
    cnt = orc.lattice_count_batch(C[pick], G)
    assert np.array_equal(area[pick], 25.0 * cnt.astype(np.float64)), (N, pick)
    bo, bi, objs = ctx.poll_best(C, rmax, want_all=True)
    want = -area + orc.violation_batch(C, rmax) * 1e5
    assert np.array_equal(objs, want)
    k = int(np.argmin(want))
    assert bi == k and bo == want[k]


def test_penalty_chain_sequential_blocks(ctx, pkg, orc):
    """The prep launch folds a candidate's penalty chain (src/TDM_STATIC_opt.jl:88-92) in UAV
    order across blocks of 512 UAVs (k_prep.h). N = 1100 (three blocks): integer terms, 2^-10
    fractions, one odd term in block 0, 1 or 2 only, huge terms, and non-finite R. Every
    objective == -area + 1e5 x the C oracle's sequential chain, bit for bit."""
    wl = pkg.workloads
    rng = wl.SplitMix64(1100)
    G = 256
    x, y, w = wl.grid_points(G)
    ctx.set_points(x, y, w)
    N = 1100
    base = wl.uniform_disks(N, G, rng)
    rmax = np.floor(rng.uniform(N) * 40.0) + 1.0
    rows = []
    for case in range(12):
        c = base.copy()
        R = np.floor(rng.uniform(N) * 40.0) + 1.0
        if case in (1, 2):
            R = R + np.floor(rng.uniform(N) * 1024.0) / 1024.0
        elif case in (3, 4, 5):
            blk = case - 3
            R[blk * 512 + 7] += 0.1
        elif case == 6:
            R[600] = 2.0 ** 40
        elif case == 7:
            R[1099] = 2.0 ** 43 / N + 1.0
        elif case == 8:
            R[10] = np.nan
        elif case == 9:
            R[520] = np.inf
        elif case == 10:
            R = R * 1.5 + 0.25 / 3.0
        c[2 * N:] = R
        rows.append(c)
    C = np.array(rows)
    area = ctx.area_batch(C)
    got = ctx.objective_batch(C, rmax)
    want = -area + orc.violation_batch(C, rmax) * 1e5
    assert np.array_equal(got, want, equal_nan=True), np.nonzero(got != want)


@pytest.mark.parametrize("algo", ["auto", "poll"])
def test_config4_clustered_full_poll(ctx, pkg, orc, algo):
    """SURVEY 8(d)'s "clustered" variant at full size: 512 R=36 disks within sqrt(N)*40 m of the
    centre of the 16.8M-cell grid, so most disks overlap lower-index ones and the shared-entry
    pass (ownership between overlapping disks) carries a large part of every candidate's area.
    Every candidate == exact lattice count; objectives, cons3 and argmin bit-exact."""
    x, y, w, C, rmax = pkg.workloads.make_config(4, disks="clustered")
    ctx.set_points(x, y, w)
    _full_poll_check(ctx, orc, C, rmax, 4096, [algo], "config4-clustered")


def _walk_of(ctx, C):
    """(areas, the walk the device chose for the batch)."""
    ctx.profile(True)
    ctx.profile_read(reset=True)
    area = ctx.area_batch(C)
    walk = ctx.profile_read(reset=True)[3]
    ctx.profile(False)
    return area, walk


@pytest.mark.parametrize("disks", ["clustered", "uniform"])
def test_walk_choice_poll_batches(ctx, pkg, orc, disks):
    """The device's walk choice (k_poll_shared.h walk_choice, costs in poll-walk test units) on
    MADS polls of K >= 64: crowded (every disk overlapping lower-index ones: the config-5 poll
    that once took 3.96 ms in the per-candidate walk) and scattered disks both take the poll walk
    under AUTO; the forced per-candidate walk, with its pairs from the poll-level neighbour
    lists, gives the same areas (slower, never different). Areas == the exact lattice counts."""
    wl = pkg.workloads
    rng = wl.SplitMix64(4242 if disks == "clustered" else 4243)
    G, N = 512, 96
    x, y, w = wl.grid_points(G)
    ctx.set_points(x, y, w)
    x0 = (wl.clustered_disks if disks == "clustered" else wl.uniform_disks)(N, G, rng)
    C = wl.poll_candidates(x0, rng)
    assert C.shape[0] == 6 * N + 1 >= 64
    want = 25.0 * orc.lattice_count_batch(C, G).astype(np.float64)
    with pkg.Context(0) as c2:   # (a fresh context: AUTO's routing history is the context's)
        c2.set_points(x, y, w)
        area, walk = _walk_of(c2, C)
        assert walk == "poll", walk
        assert np.array_equal(area, want)
        c2.set_algo("tiled")
        area_t, walk_t = _walk_of(c2, C[:64])
        # the whole crowded poll through the forced per-candidate walk: its pairs come from the
        # poll-level neighbour lists (k_walk.h), no unit rebuilds all N(N-1)/2 of them
        area_f, walk_f = _walk_of(c2, C)
    assert walk_t == walk_f == "tiled", (walk_t, walk_f)
    assert np.array_equal(area_t, want[:64])
    assert np.array_equal(area_f, want)


def test_walk_choice_scattered_batch(ctx, pkg, orc):
    """A batch that is not a poll (64 unrelated random layouts of 8 disks: no shared footprint
    across candidates) takes the per-candidate walk under AUTO; areas == exact lattice counts.
    The choice is made on the device once the neighbour lists exist; the host launches that
    walk's kernel when the lane's recent polls chose it (maxcover.hip enqueue_eval), so a lane
    that ran poll-walk polls runs this batch once through the poll walk (same areas), records
    the choice, and takes the per-candidate walk from the next call on (the five-launch chain on
    a fresh context; AUTO there takes the fused chain, which has no walk choice: same areas)."""
    wl = pkg.workloads
    rng = wl.SplitMix64(4244)
    G, N, K = 512, 8, 64
    x, y, w = wl.grid_points(G)
    ctx.set_points(x, y, w)
    C = np.stack([wl.uniform_disks(N, G, rng) for _ in range(K)])
    want = 25.0 * orc.lattice_count_batch(C, G).astype(np.float64)
    with pkg.Context(0) as c2:   # (a fresh context: AUTO's routing history is the context's)
        c2.set_points(x, y, w)
        fused = _walk_of(c2, C)   # AUTO on a fresh context: the fused chain (no walk choice)
        c2.set_chain("five")      # the five-launch chain's walk choice
        runs = [_walk_of(c2, C) for _ in range(2)]
    # (a lane with no report launches the per-candidate walk's kernel at once; one that ran
    # poll-walk polls records the choice on its first call) by the second call, that walk
    assert runs[-1][1] == "tiled", [r[1] for r in runs]
    for area, _ in [fused] + runs:
        assert np.array_equal(area, want)


@pytest.mark.parametrize("case", ["real_clustered", "big_radius", "mixed_weights", "pythagorean",
                                  "crowded", "lattice_mixed", "key_mix", "key_escape"])
def test_poll_walk_stress(ctx, pkg, orc, case):
    """The poll walk's rare paths: fp64 band decisions on real-valued coordinates, ownership
    between overlapping disks, regions larger than one LDS chunk and more than 64 tile rows.
    "pythagorean": integer points at distance exactly r from integer centres (3-4-5, 5-12-13,
    7-24-25 ...), where a = r^2 sits next to the threshold T(r) < r^2: every such entry is in
    the fp32 filter's band and must be decided in fp64 (not covered: sqrt(r^2) < r is false).
    "crowded": 100 disks over one small square, so disks past the 64th have more lower-index
    neighbours than the list keeps (per-candidate shared path) and the rest take the coverage-
    word path; "lattice_mixed": lattice polls (few distinct positions) with unequal weights
    (the word path's bit-by-bit credit); "key_mix": a lattice poll whose odd UAVs carry offsets
    no fp32 key reproduces (and one UAV with -0.0 against candidate 0's +0.0), so those disks take
    the index's identity map while the others are deduplicated (k_index.h "Keys"); "key_escape":
    a lattice poll where some candidates of some UAVs move by half-integers or by more than the
    packed key holds (|dx| > 1023, |dr| > 511): those values take the fp32 escape rows while the
    rest of the same disk packs (k_prep.h "Packed keys"), and the disk is still deduplicated."""
    wl = pkg.workloads
    rng = wl.SplitMix64(4242 + len(case))
    if case == "pythagorean":
        g = np.arange(200, dtype=np.float64)
        x = np.repeat(g, 200)
        y = np.tile(g, 200)
        w = np.full(x.size, 25.0)
        N = 20
        radii = np.array([5.0, 10.0, 13.0, 25.0, 15.0, 17.0])
        x0 = np.concatenate([np.floor(rng.uniform(N) * 120) + 40, np.floor(rng.uniform(N) * 120) + 40,
                             radii[np.floor(rng.uniform(N) * radii.size).astype(int)]])
        ctx.set_points(x, y, w)
        C = np.concatenate([x0[None, :], wl.poll_candidates(x0, rng, ell=1)], axis=0)
        C[:, 2 * N:] = np.maximum(C[:, 2 * N:], 1.0)
        want = orc.PointerList(recs(x, y, w)).area_batch(C)
        r = both(ctx, lambda: ctx.area_batch(C))
        for a, got in r.items():
            assert np.array_equal(got, want), (a, np.flatnonzero(got != want)[:5])
        return
    if case == "key_mix":
        M = 40000
        x = np.floor(rng.uniform(M) * 400.0)
        y = np.floor(rng.uniform(M) * 400.0)
        w = np.full(M, 25.0)
        N = 24
        x0 = np.concatenate([np.floor(200 + rng.uniform(N) * 160 - 80),
                             np.floor(200 + rng.uniform(N) * 160 - 80),
                             np.floor(rng.uniform(N) * 20 + 15)])
        x0[0] = 0.0
        ctx.set_points(x, y, w)
        C = np.concatenate([x0[None, :], wl.poll_candidates(x0, rng, ell=2)], axis=0)
        K = C.shape[0]
        for v in list(range(1, N, 2)) + [N + 3, 2 * N + 5]:
            pick = np.flatnonzero(rng.uniform(K) < 0.3)
            pick = pick[pick > 0]
            C[pick, v] += 1e-9 * (1.0 + rng.uniform(pick.size))     # not an fp32 offset
        zero = np.flatnonzero(C[:, 0] == 0.0)
        C[zero[1::2], 0] = -0.0
        assert zero.size > 2 and K >= 64
        want = orc.PointerList(recs(x, y, w)).area_batch(C)
        r = both(ctx, lambda: ctx.area_batch(C))
        for a, got in r.items():
            assert np.array_equal(got, want), (a, np.flatnonzero(got != want)[:5])
        rmax = np.full(N, 30.0)
        bo, bi, objs = ctx.poll_best(C, rmax, want_all=True)
        want_obj = np.array([orc.ref_objective(c, recs(x, y, w), rmax) for c in C])
        assert np.array_equal(objs, want_obj)
        return
    if case == "key_escape":
        M = 40000
        x = np.floor(rng.uniform(M) * 400.0)
        y = np.floor(rng.uniform(M) * 400.0)
        w = np.full(M, 25.0)
        N = 24
        x0 = np.concatenate([np.floor(200 + rng.uniform(N) * 160 - 80),
                             np.floor(200 + rng.uniform(N) * 160 - 80),
                             np.floor(rng.uniform(N) * 20 + 15)])
        ctx.set_points(x, y, w)
        C = np.concatenate([x0[None, :], wl.poll_candidates(x0, rng, ell=2)], axis=0)
        K = C.shape[0]
        # escapes (half-integers, |d| past the packed range) and the packed range's edges
        # (|dx|, |dy| = 1023 and |dr| = 511 pack; 1024 and 512 escape): sign extension checked
        for v, d in [(1, 0.5), (2, 1500.0), (N + 4, -0.25), (N + 5, -2048.0), (2 * N + 6, 600.0),
                     (2 * N + 7, 0.5), (3, 1023.0), (4, -1023.0), (5, 1024.0), (N + 6, -1024.0),
                     (2 * N + 8, 511.0), (2 * N + 9, 512.0), (2 * N + 10, -511.0)]:
            pick = np.flatnonzero(rng.uniform(K) < 0.2)
            pick = pick[pick > 0]
            C[pick, v] += d
        assert K >= 64
        want = orc.PointerList(recs(x, y, w)).area_batch(C)
        r = both(ctx, lambda: ctx.area_batch(C))
        for a, got in r.items():
            assert np.array_equal(got, want), (a, np.flatnonzero(got != want)[:5])
        rmax = np.full(N, 30.0)
        bo, bi, objs = ctx.poll_best(C, rmax, want_all=True)
        want_obj = np.array([orc.ref_objective(c, recs(x, y, w), rmax) for c in C])
        assert np.array_equal(objs, want_obj)
        return
    if case in ("crowded", "lattice_mixed"):
        M = 40000
        x = np.floor(rng.uniform(M) * 400.0)
        y = np.floor(rng.uniform(M) * 400.0)
        w = np.full(M, 25.0) if case == "crowded" else np.floor(rng.uniform(M) * 7) + 1
        N = 100 if case == "crowded" else 30
        span = 60 if case == "crowded" else 160
        x0 = np.concatenate([np.floor(200 + rng.uniform(N) * span - span / 2),
                             np.floor(200 + rng.uniform(N) * span - span / 2),
                             np.floor(rng.uniform(N) * 20 + 15)])
        ctx.set_points(x, y, w)
        C = np.concatenate([x0[None, :], wl.poll_candidates(x0, rng, ell=2)], axis=0)
        want = orc.PointerList(recs(x, y, w)).area_batch(C)
        r = both(ctx, lambda: ctx.area_batch(C))
        for a, got in r.items():
            assert np.array_equal(got, want), (a, np.flatnonzero(got != want)[:5])
        return
    if case == "big_radius":
        x, y, w = wl.grid_points(240)
        N = 6
        x0 = np.concatenate([rng.uniform(N) * 1200, rng.uniform(N) * 1200,
                             rng.uniform(N) * 300 + 350])
    else:
        M = 60000
        x = rng.uniform(M) * 800.0
        y = rng.uniform(M) * 800.0
        w = np.full(M, 25.0) if case == "real_clustered" else rng.uniform(M) * 3 + 1
        N = 40
        x0 = np.concatenate([400 + rng.uniform(N) * 120 - 60, 400 + rng.uniform(N) * 120 - 60,
                             rng.uniform(N) * 30 + 10])
    ctx.set_points(x, y, w)
    C = np.concatenate([x0[None, :], wl.poll_candidates(x0, rng, ell=1)], axis=0)
    C[1:, :] += (rng.uniform(C[1:].size) * 0.02 - 0.01).reshape(C[1:].shape)  # non-lattice
    want = orc.PointerList(recs(x, y, w)).area_batch(C)
    r = both(ctx, lambda: ctx.area_batch(C))
    for a, got in r.items():
        if case == "mixed_weights":
            np.testing.assert_allclose(got, want, rtol=1e-12, atol=0, err_msg=a)
        else:
            assert np.array_equal(got, want), (a, np.flatnonzero(got != want)[:5])
    assert np.array_equal(r["poll"], r["tiled"]) or case == "mixed_weights"


@pytest.mark.parametrize("case", ["crowded", "real_clustered", "mixed_weights", "pythagorean",
                                  "lattice_mixed"])
def test_shared_entry_passes(ctx, pkg, orc, case):
    """Both shared-entry passes of the poll walk, forced (MAC_OPT_SHARED): the poll kernel's fp64
    jobs and the bit-word kernel (k_bits.h: per-position coverage words, band entries in fp64,
    weighted credit bit by bit), each against the C oracle. "crowded": 100 disks over one square
    (neighbour lists past 64 go to the fp64 jobs even when the bit-words are forced);
    "real_clustered": non-lattice coordinates (band decisions); "mixed_weights": real weights
    (rtol 1e-12, the summation order differs from the list order); "pythagorean": entries exactly
    at distance r (every one in the band, not covered); "lattice_mixed": integer weights (exact)."""
    wl = pkg.workloads
    rng = wl.SplitMix64(9090 + len(case))
    if case == "pythagorean":
        g = np.arange(160, dtype=np.float64)
        x, y = np.repeat(g, 160), np.tile(g, 160)
        w = np.full(x.size, 25.0)
        N = 24
        radii = np.array([5.0, 10.0, 13.0, 25.0, 15.0, 17.0])
        x0 = np.concatenate([np.floor(rng.uniform(N) * 50) + 55, np.floor(rng.uniform(N) * 50) + 55,
                             radii[np.floor(rng.uniform(N) * radii.size).astype(int)]])
        ell = 1
    else:
        M = 40000
        x = np.floor(rng.uniform(M) * 400.0) if case != "real_clustered" else rng.uniform(M) * 400.0
        y = np.floor(rng.uniform(M) * 400.0) if case != "real_clustered" else rng.uniform(M) * 400.0
        w = (np.full(M, 25.0) if case in ("crowded", "real_clustered") else
             rng.uniform(M) * 3 + 1 if case == "mixed_weights" else np.floor(rng.uniform(M) * 7) + 1)
        N = 100 if case == "crowded" else 40
        span = 60 if case == "crowded" else 120
        x0 = np.concatenate([np.floor(200 + rng.uniform(N) * span - span / 2),
                             np.floor(200 + rng.uniform(N) * span - span / 2),
                             np.floor(rng.uniform(N) * 20 + 15)])
        ell = 2
    ctx.set_points(x, y, w)
    C = np.concatenate([x0[None, :], wl.poll_candidates(x0, rng, ell=ell)], axis=0)
    if case == "pythagorean":
        C[:, 2 * N:] = np.maximum(C[:, 2 * N:], 1.0)
    if case in ("real_clustered", "mixed_weights"):
        C[1:, :] += (rng.uniform(C[1:].size) * 0.02 - 0.01).reshape(C[1:].shape)
    want = orc.PointerList(recs(x, y, w)).area_batch(C)
    rmax = np.full(N, 30.0)
    want_obj = -want + orc.violation_batch(C, rmax) * 1e5 if case != "mixed_weights" else None
    ctx.set_algo("poll")
    try:
        for mode in ("fp64", "bits"):
            ctx.set_shared(mode)
            got = ctx.area_batch(C)
            if case == "mixed_weights":
                np.testing.assert_allclose(got, want, rtol=1e-12, atol=0, err_msg=mode)
            else:
                assert np.array_equal(got, want), (mode, np.flatnonzero(got != want)[:5])
                bo, bi, objs = ctx.poll_best(C, rmax, want_all=True)
                assert np.array_equal(objs, want_obj), mode
                k = int(np.argmin(want_obj))
                assert bi == k and bo == want_obj[k], mode
    finally:
        ctx.set_shared("auto")
        ctx.set_algo("auto")


@pytest.mark.parametrize("mode", ["fp64", "bits"])
def test_config4_clustered_shared_passes(ctx, pkg, orc, mode):
    """The clustered config-4 poll at full size through each forced shared-entry pass: every
    candidate == the exact lattice count, objectives, cons3 and argmin bit-exact."""
    x, y, w, C, rmax = pkg.workloads.make_config(4, disks="clustered")
    ctx.set_points(x, y, w)
    ctx.set_shared(mode)
    try:
        _full_poll_check(ctx, orc, C, rmax, 4096, ["poll"], "config4-clustered-" + mode)
    finally:
        ctx.set_shared("auto")


# ---------------------------------------------------------------------------- native MADS driver

@pytest.mark.parametrize("with_cons3", [False, True])
def test_native_mads_matches_python_driver(ctx, pkg, with_cons3):
    """mac_mads_run (candidates generated on the device from the splitmix64 stream) == the
    Python restatement TDM_STATIC_opt.mads evaluating explicit candidate matrices: same iterates,
    objective, iteration and evaluation counts, step by step."""
    wl = pkg.workloads
    TS = pkg.TDM_STATIC_opt
    TC = pkg.TDM_Constraints
    x, y, w = wl.grid_points(160)
    rng = wl.SplitMix64(77)
    N = 6
    x0 = np.concatenate([np.round(300 + rng.uniform(N) * 200), np.round(300 + rng.uniform(N) * 200),
                         np.full(N, 30.0)])
    r_max = np.full(N, 30.0 * math.tan(100 / 180 * math.pi / 2))
    rec = np.stack([x, y, w, w, np.zeros_like(x)], axis=1)
    obj = TS.createObjective(rec, N, r_max, ctx)
    cons = [TC.cons1]
    kw = {}
    if with_cons3:
        c3 = TC.create_cons3(x0, 100 / 180 * math.pi, np.full(N, 10.0))
        cons.append(c3)
        kw = dict(prev=c3.prev, d_lim=c3.d_lim, tan_half_fov=c3.tan_half_fov)
    res = TS.mads(x0, obj, cons, N_iter=40, ell0=2, ell_max=5, seed=4321)
    xn, st = ctx.mads_run(x0, r_max, 1e5, n_iter=40, ell0=2, ell_max=5, seed=4321, **kw)
    want_x = res.x if res.x is not None else res.i
    assert np.array_equal(xn, want_x)
    assert st["f"] == res.x_cost
    assert st["iterations"] == res.status.iteration
    assert st["evaluations"] == res.status.function_evaluations
    assert (st["status"] == 0) == (res.status.optimization_status == "MeshPrecisionLimit")
    # the evaluations the reference makes (candidates passing cons3), and the polls cons3
    # rejects whole with no launch (only ones where no candidate passes)
    assert st["feasible_evaluations"] == res.status.cons3_passed
    assert st["successes"] == res.status.successes
    assert st["rejected_polls"] <= res.status.cons3_empty_polls
    if not with_cons3:
        assert st["rejected_polls"] == 0


@pytest.mark.parametrize("algo", ["auto", "poll"])
def test_native_mads_matches_oracle_loop(ctx, pkg, orc, algo):
    """mac_mads_run against the reference's own per-trial-point loop on the C oracle: the Python
    driver TDM_STATIC_opt.mads with an objective that is a plain callable (no batch, no poll),
    so every feasible candidate goes through orc.ref_objective (src/TDM_STATIC_opt.jl:82-100)
    one at a time, cons1 and cons3 checked per candidate (src/TDM_Constraints.jl). N = 12 UAVs:
    K = 72 candidates per poll, past the poll walk's threshold, disks overlapping (shared
    entries). Same iterate, objective and iteration count; libmaxcover is not on the reference
    side at all."""
    wl = pkg.workloads
    TS = pkg.TDM_STATIC_opt
    TC = pkg.TDM_Constraints
    x, y, w = wl.grid_points(160)
    rec = np.stack([x, y, w, w, np.zeros_like(x)], axis=1)
    rng = wl.SplitMix64(2024)
    N = 12
    x0 = np.concatenate([np.round(320 + rng.uniform(N) * 160), np.round(320 + rng.uniform(N) * 160),
                         np.full(N, 36.0)])
    r_max = np.full(N, 30.0 * TAN50)
    c3 = TC.create_cons3(x0, 100 / 180 * math.pi, np.full(N, 10.0))

    def oracle_objective(v):
        return orc.ref_objective(v, rec, r_max, 1e5)

    res = TS.mads(x0, oracle_objective, [TC.cons1, c3], N_iter=30, ell0=2, ell_max=5, seed=99)
    ctx.set_points_records(rec)
    ctx.set_algo(algo)
    try:
        xn, st = ctx.mads_run(x0, r_max, 1e5, prev=c3.prev, d_lim=c3.d_lim,
                              tan_half_fov=c3.tan_half_fov, n_iter=30, ell0=2, ell_max=5, seed=99)
    finally:
        ctx.set_algo("auto")
    want_x = res.x if res.x is not None else res.i
    assert res.x_cost < oracle_objective(x0)   # the loop moved (~1,100 feasible evaluations)
    assert np.array_equal(xn, want_x)
    assert st["f"] == res.x_cost
    assert st["iterations"] == res.status.iteration


@pytest.mark.parametrize("world", [2, 3])
def test_native_mads_sharded_steppers(ctx, pkg, world):
    """The multi-GPU MADS loop's native side in one process: `world` steppers (mac_mads_begin with
    candidate shards [floor(rK/P), floor((r+1)K/P)) of every poll), each poll's local bests
    combined by dist.reduce_best (what the 16-B all-gather computes on P GPUs) and applied to
    every stepper: every stepper ends on mac_mads_run's iterate, objective, iteration and
    evaluation counts, with cons3."""
    from importlib import import_module
    d = import_module(pkg.__name__ + ".dist")
    wl = pkg.workloads
    x, y, w = wl.grid_points(200)
    ctx.set_points(x, y, w)
    rng = wl.SplitMix64(303)
    N = 9
    x0 = np.concatenate([np.round(250 + rng.uniform(N) * 400), np.round(250 + rng.uniform(N) * 400),
                         np.full(N, 30.0)])
    r_max = np.full(N, 30.0 * TAN50)
    kw = dict(prev=x0, d_lim=np.full(N, 10.0), tan_half_fov=TAN50, n_iter=30, ell0=2, ell_max=5,
              seed=777)
    want_x, want = ctx.mads_run(x0, r_max, 1e5, **kw)
    K = 2 * x0.size
    steppers = [ctx.mads_stepper(x0, r_max, 1e5, shard=d.shard_range(K, r, world), **kw)
                for r in range(world)]
    polls = 0
    while True:
        res = [s_.poll() for s_ in steppers]
        assert len({r[0] for r in res}) == 1
        if res[0][0]:
            break
        polls += 1
        bo, bi = d.reduce_best([r[1] for r in res], [r[2] for r in res])
        for s_ in steppers:
            s_.update(bo, bi)
    assert polls == want["iterations"] > 5
    polls_or_rounds = polls
    for s_ in steppers:
        xs, st = s_.result()
        s_.close()
        assert np.array_equal(xs, want_x)
        assert st["f"] == want["f"] and st["iterations"] == want["iterations"]
        assert st["evaluations"] == want["evaluations"]
        # every poll's result came through the mapped slot (round 5's check-word mismatch made each
        # wait run into its 50-ms limit and fall back to a copy): no fallback, and no long waits
        assert st["slot_fallbacks"] == 0
        assert st["wait_s"] < 0.005 * max(polls_or_rounds, 1) + 0.05


@pytest.mark.parametrize("world", [2, 4])
def test_native_mads_speculative_steppers(ctx, pkg, world):
    """The speculative multi-GPU loop's native side in one process (mac_mads_poll_ahead /
    mac_mads_advance): stepper j polls the whole poll that follows j failures, and every stepper
    applies the P results in order up to the first success (what dist.mads_loop_speculative does
    after its all-gather). Every stepper ends on mac_mads_run's iterate, objective, iteration and
    evaluation counts, with cons3, in fewer rounds than iterations."""
    wl = pkg.workloads
    x, y, w = wl.grid_points(200)
    ctx.set_points(x, y, w)
    rng = wl.SplitMix64(919)
    N = 9
    x0 = np.concatenate([np.round(250 + rng.uniform(N) * 400), np.round(250 + rng.uniform(N) * 400),
                         np.full(N, 30.0)])
    r_max = np.full(N, 30.0 * TAN50)
    kw = dict(prev=x0, d_lim=np.full(N, 10.0), tan_half_fov=TAN50, n_iter=40, ell0=2, ell_max=6,
              seed=4711)
    want_x, want = ctx.mads_run(x0, r_max, 1e5, **kw)
    steppers = [ctx.mads_stepper(x0, r_max, 1e5, **kw) for _ in range(world)]
    rounds = 0
    useful = 0
    while True:
        res = [s_.poll_ahead(j) for j, s_ in enumerate(steppers)]
        rounds += 1
        finished = False
        for j in range(world):
            done, bo, bi, fe = res[j]
            if done:
                finished = True
                break
            useful += fe
            moved = [s_.advance(bo, bi) for s_ in steppers]
            assert len(set(moved)) == 1
            if moved[0]:
                break
        if finished:
            break
    assert rounds < want["iterations"]
    assert useful == want["feasible_evaluations"]   # the applied polls' evaluations = the loop's
    polls_or_rounds = rounds
    for s_ in steppers:
        xs, st = s_.result()
        s_.close()
        assert np.array_equal(xs, want_x)
        assert st["f"] == want["f"] and st["iterations"] == want["iterations"]
        assert st["evaluations"] == want["evaluations"]
        # every poll's result came through the mapped slot (round 5's check-word mismatch made each
        # wait run into its 50-ms limit and fall back to a copy): no fallback, and no long waits
        assert st["slot_fallbacks"] == 0
        assert st["wait_s"] < 0.005 * max(polls_or_rounds, 1) + 0.05


def test_mads_best_buffer_device_exchange(ctx, pkg):
    """dist.DeviceGather's device path (mac_mads_best_buffer): every poll of a sharded stepper
    also writes its 16-B shard best into the bound device buffer, and once poll() has returned
    the buffer holds exactly that poll's (objective, index) — read here on ANOTHER torch stream
    with no event (what the RCCL all-gather does) — including an empty shard's {+inf, -1}
    record. The steppers then follow mac_mads_run's iterates."""
    import torch
    from importlib import import_module
    d = import_module(pkg.__name__ + ".dist")
    wl = pkg.workloads
    x, y, w = wl.grid_points(160)
    ctx.set_points(x, y, w)
    rng = wl.SplitMix64(4242)
    N = 9
    x0 = np.concatenate([np.round(200 + rng.uniform(N) * 350), np.round(200 + rng.uniform(N) * 350),
                         np.full(N, 30.0)])
    r_max = np.full(N, 30.0 * TAN50)
    kw = dict(prev=x0, d_lim=np.full(N, 10.0), tan_half_fov=TAN50, n_iter=20, ell0=2, ell_max=5,
              seed=31337)
    want_x, want = ctx.mads_run(x0, r_max, 1e5, **kw)
    K = 2 * x0.size
    shards = [(0, 20), (20, 20), (20, K)]   # the middle one is empty
    dev = torch.device("cuda", ctx.device)
    side = torch.cuda.Stream(dev)
    steppers, bufs = [], []
    for sh in shards:
        s_ = ctx.mads_stepper(x0, r_max, 1e5, shard=sh, **kw)
        b = torch.full((2,), 7.0, dtype=torch.float64, device=dev)   # not the record
        torch.cuda.current_stream(dev).synchronize()
        s_.best_buffer(b)
        steppers.append(s_)
        bufs.append(b)
    host = torch.empty((len(shards), 2), dtype=torch.float64, pin_memory=True)
    polls = 0
    while True:
        res = [s_.poll() for s_ in steppers]
        if res[0][0]:
            break
        polls += 1
        with torch.cuda.stream(side):   # no event: ordered only by poll()'s return
            for q, b in enumerate(bufs):
                host[q].copy_(b, non_blocking=True)
        side.synchronize()
        for q, (done, bo, bi) in enumerate(res):
            got_o = float(host[q, 0])
            got_i = int(host[q].view(torch.int64)[1])
            if shards[q][0] == shards[q][1]:
                assert (got_o, got_i) == (math.inf, -1), (polls, q)
            else:
                assert got_i == bi and (got_o == bo or (math.isinf(got_o) and math.isinf(bo))), \
                    (polls, q, got_o, got_i, bo, bi)
        bo, bi = d.reduce_best([r[1] for r in res], [r[2] for r in res])
        for s_ in steppers:
            s_.update(bo, bi)
    assert polls == want["iterations"] > 3
    for s_ in steppers:
        xs, st = s_.result()
        s_.best_buffer(None)
        s_.close()
        assert np.array_equal(xs, want_x) and st["f"] == want["f"]


@pytest.mark.parametrize("N,n_iter,ell0,ell_max,cons3,stall", [
    (40, 60, 2, 5, True, False),     # iteration limit, cons3
    (40, 200, 2, 4, False, True),    # mesh precision limit after 3 polls: later polls already enqueued
    (40, 1, 2, 5, True, False),      # fewer polls than the window
    (40, 2, 2, 5, False, False),
    (300, 25, 3, 6, True, False),    # K = 1800
])
def test_native_mads_pipelined_matches_stepper(ctx, pkg, N, n_iter, ell0, ell_max, cons3, stall):
    """mac_mads_run's pipelined loop (each poll's update applied on the device by its finalize,
    polls enqueued ahead of their outcomes: maxcover.hip mads_run_pipelined) == the stepper driven
    one poll at a time from Python (mac_mads_begin / _poll / _update, host update): same iterate
    bit for bit, objective, iteration and evaluation counts and status. `stall`: two entries
    under UAV 0 with every radius at r_max, so no poll can improve (a move keeps the union, a
    radius change adds penalty) and the loop stops at the mesh precision limit after ell0 + 1
    polls while later polls are already enqueued."""
    wl = pkg.workloads
    rng = wl.SplitMix64(9000 + N + n_iter)
    r_max = np.full(N, 30.0 * TAN50)
    x0 = np.concatenate([np.round(200 + rng.uniform(N) * 500), np.round(200 + rng.uniform(N) * 500),
                         np.full(N, 30.0)])
    if stall:
        x0[2 * N:] = r_max
        ctx.set_points(np.array([x0[0], x0[0] + 1.0]), np.array([x0[N], x0[N]]), np.ones(2))
    else:
        x, y, w = wl.grid_points(220)
        ctx.set_points(x, y, w)
    kw = dict(n_iter=n_iter, ell0=ell0, ell_max=ell_max, seed=31337 + N)
    if cons3:
        kw.update(prev=x0, d_lim=np.full(N, 12.0), tan_half_fov=TAN50)
    want_x, want = ctx.mads_run(x0, r_max, 1e5, **kw)
    st_ = ctx.mads_stepper(x0, r_max, 1e5, **kw)
    try:
        while True:
            done, bo, bi = st_.poll()
            if done:
                break
            st_.update(bo, bi)
        xs, got = st_.result()
    finally:
        st_.close()
    assert np.array_equal(want_x, xs)
    for key in ("f", "iterations", "evaluations", "status", "feasible", "feasible_evaluations",
                "rejected_polls", "successes"):
        assert want[key] == got[key], key   # (rejections: device-side vs host-side, alike)
    if cons3 and not stall and n_iter >= 40:   # (ell reaches 5: 2^5 - 12 > 12 on every axis)
        assert want["rejected_polls"] > 0 and want["feasible_evaluations"] > 0
    if stall:
        assert want["status"] == 0 and want["iterations"] == ell0 + 1
        assert np.array_equal(want_x, x0)


def test_armed_polls_match_plain_polls(pkg):
    """mac_poll_arm_dev_f64 / mac_poll_fire: a loop of dependent polls armed one ahead (behind the
    context's doorbell, released after the previous result is read, alternating d_best buffers)
    returns every poll's (objective, index) exactly as mac_poll_best_dev_f64; a context destroyed
    with an armed poll never fired releases it (no hang)."""
    import torch
    wl = pkg.workloads
    x, y, w = wl.grid_points(192)
    rng = wl.SplitMix64(808)
    N = 16
    x0 = wl.clustered_disks(N, 192, rng)
    polls = [wl.poll_candidates(x0, rng) for _ in range(3)]
    K = polls[0].shape[0]
    r_max = np.full(N, 30.0 * TAN50)
    dev = torch.device("cuda", 0)
    d_polls = [torch.from_numpy(np.ascontiguousarray(p)).to(dev) for p in polls]
    d_prev = [torch.from_numpy(np.ascontiguousarray(p[0])).to(dev) for p in polls]
    d_rmax = torch.from_numpy(r_max).to(dev)
    d_dlim = torch.full((N,), 10.0, dtype=torch.float64, device=dev)
    bests = [torch.empty(2, dtype=torch.float64, device=dev) for _ in range(2)]
    stream = torch.cuda.Stream(dev)
    with pkg.Context(0) as ctx:
        ctx.set_points(x, y, w)
        want = []
        for j in range(7):
            ctx.poll_best_dev(d_polls[j % 3], 3 * N, K, d_rmax, bests[0], d_prev=d_prev[j % 3],
                              d_dlim=d_dlim, tan_half_fov=TAN50, stream=stream.cuda_stream)
            want.append(ctx.best_fetch(bests[0], stream=stream.cuda_stream))
        torch.cuda.synchronize()
        arm, fire, fetch = ctx.armed_steps(
            [dict(d_cands=d_polls[j % 3], three_n=3 * N, K=K, d_rmax=d_rmax, d_best=bests[j % 2],
                  d_prev=d_prev[j % 3], d_dlim=d_dlim, tan_half_fov=TAN50) for j in range(6)],
            stream=stream.cuda_stream)
        got = []
        arm(0)
        for j in range(7):
            fire(j % 6)
            if j + 1 < 7:
                arm((j + 1) % 6)
            got.append(fetch(j % 6))
        assert got == want
        assert len({o for o, _ in want}) > 1   # (different polls, different bests)
        with pytest.raises(pkg.MaxCoverError):
            ctx.poll_fire(10 ** 6)              # never armed
        with pytest.raises(pkg.MaxCoverError):  # HIP's null stream refused (nothing enqueued)
            ctx.poll_arm(d_polls[0], 3 * N, K, d_rmax, bests[1], stream=0)
    with pkg.Context(0) as ctx2:                # destroyed with an armed poll never fired
        ctx2.set_points(x, y, w)
        ctx2.poll_arm(d_polls[0], 3 * N, K, d_rmax, bests[1], stream=stream.cuda_stream)
    torch.cuda.synchronize()


def test_armed_poll_grows_lane_buffers(pkg):
    """An armed poll larger than anything its lane has run (more candidates and more UAVs: every
    scratch buffer grows inside the arming call). Freeing the old buffers there would wait for the
    device, which waits for the unfired ticket: the buffers are released at the next device
    synchronisation instead (include/maxcover.h). The results equal plain polls'. An argument error
    is reported before anything is enqueued and takes no ticket, and a plain poll on another
    stream runs and is fetched while an armed poll is pending."""
    import torch
    wl = pkg.workloads
    x, y, w = wl.grid_points(192)
    rng = wl.SplitMix64(809)
    dev = torch.device("cuda", 0)
    shapes = (4, 24, 40)                                   # N, growing
    polls = [wl.poll_candidates(wl.uniform_disks(n, 192, rng), rng) for n in shapes]
    with pkg.Context(0) as ref:
        ref.set_points(x, y, w)
        want = [ref.poll_best(p, np.full(p.shape[1] // 3, 36.0)) for p in polls]
    d_polls = [torch.from_numpy(np.ascontiguousarray(p)).to(dev) for p in polls]
    d_rmax = [torch.full((p.shape[1] // 3,), 36.0, dtype=torch.float64, device=dev) for p in polls]
    bests = [torch.empty(2, dtype=torch.float64, device=dev) for _ in polls]
    s1, s2 = torch.cuda.Stream(dev), torch.cuda.Stream(dev)
    torch.cuda.synchronize(dev)
    with pkg.Context(0) as ctx:
        ctx.set_points(x, y, w)
        got = []
        for j, p in enumerate(polls):
            t = ctx.poll_arm(d_polls[j], p.shape[1], p.shape[0], d_rmax[j], bests[j],
                             stream=s1.cuda_stream)
            with pytest.raises(pkg.MaxCoverError):     # checked before anything is enqueued
                ctx.poll_arm(d_polls[j], p.shape[1], p.shape[0], d_rmax[j], None,
                             stream=s1.cuda_stream)
            if j == 1:   # a plain poll on another stream while ticket t is pending
                ctx.poll_best_dev(d_polls[0], polls[0].shape[1], polls[0].shape[0], d_rmax[0],
                                  bests[0], stream=s2.cuda_stream)
                assert ctx.best_fetch(bests[0], stream=s2.cuda_stream) == want[0]
            ctx.poll_fire(t)
            got.append(ctx.best_fetch(bests[j], stream=s1.cuda_stream))
        assert got == want
        ctx.set_points(x, y, w)          # (a device synchronisation: deferred frees released)
        ctx.poll_best_dev(d_polls[2], polls[2].shape[1], polls[2].shape[0], d_rmax[2], bests[2],
                          stream=s1.cuda_stream)
        assert ctx.best_fetch(bests[2], stream=s1.cuda_stream) == want[2]
    torch.cuda.synchronize(dev)


@pytest.mark.parametrize("cons3", [False, True])
def test_config4_basis_form_poll(ctx, pkg, orc, cons3):
    """mac_poll_basis_f64 at config 4 (512 UAVs x 16.8M cells, n = 1536, 2n = 3072 candidates):
    the incumbent, the LTMADS basis as L's packed lower triangle plus its row / column permutations
    and delta (src/TDM_STATIC_opt.jl:22-44's b / i / maximal_basis) expanded on the device. Every
    objective equals -25 x the exact lattice count + 1e5 x the oracle's sequential violation (or
    +inf where the oracle's cons3 fails), bit for bit, and equals mac_poll_best_f64 on the 3N x 2n
    matrix the same arithmetic builds; the argmin is the lowest minimiser."""
    wl = pkg.workloads
    rng = wl.SplitMix64(wl.SEED + 61)
    x, y, w = wl.grid_points(4096)
    ctx.set_points(x, y, w)
    N = 512
    x0 = wl.uniform_disks(N, 4096, rng)
    n = 3 * N
    # (cons3: mesh step 8 = ell 3, where some candidates move a UAV more than d_lim = 10 m; at the
    # bench's ell = 2 every candidate passes)
    Lm, rp, cp = wl.ltmads_basis_parts(n, 3 if cons3 else 2, rng)
    B = Lm[rp][:, cp].astype(np.float64)
    delta = 1.0
    C = np.ascontiguousarray(np.concatenate([x0[None, :] + delta * B.T, x0[None, :] - delta * B.T]))
    rmax = np.full(N, 30.0 * TAN50)
    kw = dict(prev=x0, d_lim=np.full(N, 10.0), tan_half_fov=TAN50) if cons3 else {}
    bo, bi, objs = ctx.poll_basis(x0, Lm, rp, cp, delta, rmax, 1e5, want_all=True, **kw)
    mo, mi, mobjs = ctx.poll_best(C, rmax, 1e5, want_all=True, **kw)
    assert np.array_equal(objs, mobjs) and (bo, bi) == (mo, mi)
    want = -25.0 * orc.lattice_count_batch(C, 4096).astype(np.float64) + orc.violation_batch(C, rmax) * 1e5
    if cons3:
        feas = orc.cons3_batch(x0, C, np.full(N, 10.0), TAN50)
        assert 0 < int(feas.sum()) < C.shape[0]
        want = np.where(feas, want, np.inf)
    assert np.array_equal(objs, want), np.flatnonzero(objs != want)[:5]
    k = int(np.argmin(want))
    assert bi == k and bo == want[k]


def test_basis_form_scaled_and_rejected(ctx, pkg, orc):
    """The basis form off the unit mesh: delta = 0.75 and 2.5 (B's entries delta * L as doubles,
    matrix built with the same products), a small N through the generic walks; and argument
    errors (a permutation entry outside [0, n), a packed triangle of the wrong size) refused
    before anything runs."""
    wl = pkg.workloads
    rng = wl.SplitMix64(77)
    x, y, w = wl.grid_points(256)
    ctx.set_points(x, y, w)
    N = 12
    x0 = wl.uniform_disks(N, 256, rng)
    n = 3 * N
    rmax = np.full(N, 30.0 * TAN50)
    for delta in (0.75, 2.5):
        Lm, rp, cp = wl.ltmads_basis_parts(n, 3, rng)
        Bd = delta * Lm[rp][:, cp].astype(np.float64)
        C = np.ascontiguousarray(np.concatenate([x0[None, :] + Bd.T, x0[None, :] - Bd.T]))
        for algo in ("auto", "poll", "tiled"):
            ctx.set_algo(algo)
            got = ctx.poll_basis(x0, Lm, rp, cp, delta, rmax, want_all=True)
            want = ctx.poll_best(C, rmax, want_all=True)
            assert got[:2] == want[:2] and np.array_equal(got[2], want[2]), (delta, algo)
        ctx.set_algo("auto")
        rec = np.stack([x, y, w, w, np.zeros_like(x)], axis=1)
        viol = orc.violation_batch(C, rmax) * 1e5
        for k in np.unique(np.floor(rng.uniform(6) * C.shape[0]).astype(np.int64)):
            assert got[2][k] == -orc.ref_area(C[k], rec) + viol[k], (delta, k)
    bad = rp.copy()
    bad[3] = n
    with pytest.raises(pkg.MaxCoverError):
        ctx.poll_basis(x0, Lm, bad, cp, 1.0, rmax)
    with pytest.raises(ValueError):
        ctx.poll_basis(x0, Lm[np.tril_indices(n)][:-1], rp, cp, 1.0, rmax)
