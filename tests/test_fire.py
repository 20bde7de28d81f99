"""Fire stream (config 5): the CA fire generator of src/DynamicArea.jl
on the GPU vs its C restatement, appending points to a context (update_POI), and the
FirePoints table converter."""
import math
import os

import numpy as np
import pytest



def _refire(orc, nx, ny, ign, seed, **kw):
    return orc.RefFire(nx, ny, ignition=ign, seed=seed, **kw)


# ---------------------------------------------------------------------------- CPU: the oracle

def test_ref_fire_semantics(orc):
    """Properties of the restated rules (:52-72): border cells never change; FIRE persists;
    every pushed point sits on a cell that turned TREE -> FIRE this step, once per igniting
    neighbour; points come in i-outer / j-inner cell order."""
    nx, ny = 40, 30
    f = _refire(orc, nx, ny, (18, 22, 14, 16), 7)
    g0 = f.grid.reshape(nx, ny).copy()
    total = 0
    for _ in range(12):
        before = f.grid.reshape(nx, ny).copy()
        pts = f.step()
        after = f.grid.reshape(nx, ny)
        assert np.array_equal(after[0], before[0]) and np.array_equal(after[-1], before[-1])
        assert np.array_equal(after[:, 0], before[:, 0]) and np.array_equal(after[:, -1], before[:, -1])
        assert np.all(after[before == 2] == 2)
        newly = (before == 1) & (after == 2)
        i = np.rint((pts[:, 0] + 2.5) / 5).astype(int)
        j = np.rint((pts[:, 1] + 2.5) / 5).astype(int)
        assert np.all(newly[i - 1, j - 1])
        cells = sorted(set(zip(i.tolist(), j.tolist())))
        assert len(cells) == int(newly.sum())
        order = (i - 1) * ny + (j - 1)
        assert np.all(np.diff(order) >= 0)
        for (ci, cj) in cells:                       # at most one point per FIRE neighbour
            k = int(np.sum((i == ci) & (j == cj)))
            block = before[ci - 2:ci + 1, cj - 2:cj + 1]
            assert 1 <= k <= int(np.sum(block == 2))
        assert np.all(pts[:, 2] == 25.0) and np.all(pts[:, 3] == 25.0) and np.all(pts[:, 4] == 0)
        total += pts.shape[0]
    assert total > 0 and not np.array_equal(g0, f.grid.reshape(nx, ny))


def test_ref_fire_wind_thresholds(orc):
    """:63 with the reference's wind (4, 270 deg) and prob_spread 0.5: the nine thresholds
    2*cos(3pi/2 - atan(2-c, 2-r)) — up-wind slots always ignite (> 1), cross-wind ones at 0."""
    f = _refire(orc, 10, 10, (4, 5, 4, 5), 1)
    want = np.array([4 * math.cos(math.radians(270) - math.atan2(2 - c, 2 - r)) * 0.5
                     for c in (1, 2, 3) for r in (1, 2, 3)])
    assert np.array_equal(f.p9, want)


def test_firepoints_converter_roundtrip(pkg, firepoints, tmp_path):
    fp = pkg.firepoints
    rows = firepoints + [np.zeros((0, 5))] + firepoints[:2]     # an empty timestep in the middle
    p = fp.write_csv(rows, str(tmp_path / "fp.csv"), source="test")
    back = fp.read_csv(p)
    assert len(back) == len(rows)
    assert all(np.array_equal(a, b) for a, b in zip(rows, back))
    assert back[len(firepoints)].shape == (0, 5)


@pytest.mark.skipif(not os.path.exists("/root/reference/src/FirePoints.xlsx"),
                    reason="reference data not present (build container only)")
def test_firepoints_xlsx_reader_matches_fixture(pkg, firepoints):
    rows = pkg.firepoints.read_xlsx("/root/reference/src/FirePoints.xlsx")
    assert len(rows) == len(firepoints) == 68
    assert all(np.array_equal(a, b) for a, b in zip(rows, firepoints))


# ---------------------------------------------------------------------------- GPU

@pytest.mark.gpu
@pytest.mark.parametrize("shape,ign,seed", [((80, 60), (30, 40, 25, 28), 11),
                                            ((100, 100), (40, 60, 69, 71), 20250216),
                                            ((257, 131), (100, 140, 60, 70), 3)])
def test_fire_gpu_matches_oracle(pkg, orc, shape, ign, seed):
    nx, ny = shape
    kw = dict(forest_density=0.7, prob_spread=0.5, wind_speed=4.0, wind_direction=math.radians(270))
    ref = _refire(orc, nx, ny, ign, seed, **kw)
    gpu = pkg.Fire(nx, ny, 5.0, 5.0, kw["forest_density"], kw["prob_spread"], kw["wind_speed"],
                   kw["wind_direction"], ign, seed)
    assert np.array_equal(gpu.thresholds(), ref.p9)
    assert np.array_equal(gpu.grid().reshape(-1), ref.grid)
    for t in range(25):
        want = ref.step()
        n = gpu.step()
        assert n == want.shape[0], t
        assert np.array_equal(gpu.last_points(), want), t
        assert np.array_equal(gpu.grid().reshape(-1), ref.grid), t
    gpu.close()


@pytest.mark.gpu
def test_dynamic_area_defaults(pkg, orc):
    """The reference's parameters (100 x 100 cells, ignition [40,60] x [69,71], wind 270 deg):
    initial points (:37-42) and 20 steps, exported like export_data."""
    D = pkg.DynamicArea.DynamicArea()
    assert D.grid_size == (100, 100) and D.ignition == (40, 60, 69, 71)
    init = D.export_data[0]
    assert init.shape == (21 * 3, 5)
    assert np.array_equal(init[:3, :2], [[197.5, 342.5], [202.5, 342.5], [207.5, 342.5]])
    ref = _refire(orc, 100, 100, (40, 60, 69, 71), pkg.DynamicArea.SEED)
    rows = D.run(20)
    for t in range(1, 21):
        assert np.array_equal(rows[t], ref.step()), t
    D.close()


@pytest.mark.gpu
def test_append_points_and_stream(ctx, pkg, orc):
    """update_POI appends at the end of the list (list order = summation order); a fire
    streaming into the context gives the same list, areas and removal as the oracle."""
    rng = pkg.workloads.SplitMix64(55)
    a = np.stack([rng.uniform(3000) * 400, rng.uniform(3000) * 400], axis=1)
    b = np.stack([rng.uniform(1500) * 400, rng.uniform(1500) * 400], axis=1)
    wa = rng.uniform(3000) + 1.0
    wb = rng.uniform(1500) + 1.0
    ctx.set_points(a[:, 0], a[:, 1], wa)
    ctx.append_points(b[:, 0], b[:, 1], wb)
    x, y, w = ctx.get_points()
    assert np.array_equal(x, np.concatenate([a[:, 0], b[:, 0]]))
    assert np.array_equal(w, np.concatenate([wa, wb]))
    rec = np.stack([x, y, w, w, np.zeros_like(x)], axis=1)
    C = np.concatenate([np.concatenate([rng.uniform(6) * 400, rng.uniform(6) * 400,
                                        rng.uniform(6) * 40 + 10])[None, :] for _ in range(5)])
    want = orc.PointerList(rec).area_batch(C)
    np.testing.assert_allclose(ctx.area_batch(C), want, rtol=1e-12, atol=0)

    # a fire streaming into a context: initial points, then each step appended on the device
    fire = pkg.Fire(90, 90, 5.0, 5.0, 0.7, 0.5, 4.0, math.radians(270), (35, 50, 40, 45), 99)
    init = fire.initial_points()
    ctx.set_points_records(init)
    lst = [init]
    for _ in range(15):
        fire.step(append_to=ctx)
        lst.append(fire.last_points())
    full = np.concatenate(lst)
    x, y, w = ctx.get_points()
    assert np.array_equal(np.stack([x, y], axis=1), full[:, :2])
    circles = np.array([200.0, 240.0, 180.0, 210.0, 230.0, 260.0, 36.0, 36.0, 30.0])
    assert ctx.area(circles) == orc.ref_area(circles, full)
    kept = ctx.remove_covered(circles)
    assert np.array_equal(kept, orc.ref_remove_covered(circles, full))
    fire.close()


@pytest.mark.gpu
def test_full_simulation_dynamic_matches_replay(ctx, pkg, orc):
    """Config 5 in miniature (src/FullSimulation.jl:42-100 with the fire stream): per MPC step
    the device list equals the oracle's replay (fire points appended, then rmvCoveredPOI by the
    previous circles), and the native MADS output equals the Python driver's on that list, with
    the oracle's objective."""
    FS = pkg.FullSimulation
    TS = pkg.TDM_STATIC_opt
    TC = pkg.TDM_Constraints
    tan50 = math.tan(100 / 180 * math.pi / 2)
    x0 = orc.ref_allocate_even_circles(15.0, 5, 10 * tan50, 250.0, 250.0)   # :803
    x0 = np.round(x0)
    D = pkg.DynamicArea.DynamicArea(x_start1=200, x_start2=300, y_start1=200, y_start2=260)
    sim = FS.Simulation(ctx, x0, fire=D, N_iter=25, seed=99)
    ref = _refire(orc, 100, 100, D.ignition, pkg.DynamicArea.SEED)
    lst = D.initial_points()
    ctx2 = pkg.Context(0)
    x_prev = x0.copy()
    for t in range(1, 5):
        rec = sim.step()
        lst = np.concatenate([lst, ref.step()])
        kept = orc.ref_remove_covered(x_prev, lst)
        lst = lst[kept]
        x, y, w = ctx.get_points()
        assert np.array_equal(np.stack([x, y, w], axis=1), lst[:, [0, 1, 3]]), t
        # the Python driver on the replayed list, same input / seed / constraint
        obj = TS.createObjective(lst, 5, sim.r_max, ctx2)
        c3 = TC.create_cons3(x_prev, 100 / 180 * math.pi, np.full(5, 10.0))
        res = TS.mads(rec["input"], obj, [TC.cons1, c3], N_iter=25, ell0=2, ell_max=6,
                      seed=99 + t)
        want = res.x if res.x is not None else res.i
        assert np.array_equal(sim.outputs[-1], want), t
        assert rec["f"] == res.x_cost, t
        if np.isfinite(rec["f"]):
            assert rec["f"] == orc.ref_objective(want, lst, sim.r_max), t
        x_prev = sim.outputs[-1]
    ctx2.close()
    D.close()


@pytest.mark.gpu
def test_config5_full_size_mpc_step(ctx, pkg, orc):
    """Config 5 at full size (512 UAVs over the 512^2-cell ignition block of a 4096^2 CA fire):
    one MPC step (fire step + append, rmvCoveredPOI, native MADS), then a complete 2n + 1 poll
    around its output through AUTO (the device index, the poll walk and the shared-entry jobs:
    the clustered disks overlap heavily) against the C oracle on the device's final list, on
    64 sampled candidates and the poll's argmin (every sampled oracle objective >= the device's
    best, the device's best = the oracle's objective of its index); the MADS objective of the
    bench's 100-iteration run against the oracle too."""
    wl = pkg.workloads
    cfg = wl.CONFIGS[5]
    rng = wl.SplitMix64(5555)
    fire_kw, x0 = wl.config5_setup(rng, cfg["G"], cfg["N"], cfg["ignition"])
    D = pkg.DynamicArea.DynamicArea(**fire_kw, seed=5555, device=0)
    sim = pkg.FullSimulation.Simulation(ctx, x0, fire=D, N_iter=100, seed=5555)
    rec = sim.step()
    x, y, w = ctx.get_points()
    assert x.size == rec["points"] > 100000
    lst = np.stack([x, y, w, w, np.zeros_like(x)], axis=1)
    N = cfg["N"]
    xo = sim.outputs[-1]
    # many overlapping disk pairs: the shared-entry jobs carry part of every candidate's area
    cx, cy = xo[:N], xo[N:2 * N]
    d2 = (cx[:, None] - cx[None, :]) ** 2 + (cy[:, None] - cy[None, :]) ** 2
    assert int(np.sum(np.triu(d2 < (2 * 36.0) ** 2, 1))) > 200
    if np.isfinite(rec["f"]):
        assert rec["f"] == orc.ref_objective(xo, lst, sim.r_max)
    C = wl.poll_candidates(xo, rng)
    ctx.set_algo("auto")
    bo, bi, objs = ctx.poll_best(C, sim.r_max, 1e5, want_all=True)
    pick = np.unique(np.concatenate([[0, bi], np.floor(rng.uniform(64) * C.shape[0]).astype(np.int64)]))
    assert pick.size >= 60
    pl = orc.PointerList(lst)
    area = pl.area_batch(C[pick], 16)
    viol = orc.violation_batch(C[pick], sim.r_max)
    want = -area + viol * 1e5
    assert np.array_equal(objs[pick], want), pick
    # the device's argmin against the oracle, not against the device's own objectives
    assert want[np.searchsorted(pick, bi)] == bo
    assert np.all(want >= bo), (pick[want < bo], bo)
    assert bi == int(np.argmin(objs)) and bo == objs[bi]
    D.close()


def _c5_poll293(pkg, ell_at=None):
    """The config-5 poll behind the bit-word kernel's 1.1-ms launch (tests/golden/c5_poll293.npz,
    tests/golden/make_c5_poll_fixture.py): (x, y, w, candidates K x 3N, prev, r_max, ell); with
    ell_at, the same stream position's poll at mesh index ell_at."""
    import importlib.util
    import os
    root = os.path.dirname(os.path.abspath(__file__))
    spec = importlib.util.spec_from_file_location(
        "make_c5_poll_fixture", os.path.join(root, "golden", "make_c5_poll_fixture.py"))
    mk = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mk)
    d = np.load(os.path.join(root, "golden", "c5_poll293.npz"))
    seed, it, ell = (int(v) for v in d["meta"][:3])
    ell = ell if ell_at is None else ell_at
    cells = d["cells"].astype(np.float64)
    x, y = cells[:, 0] * 5.0 - 2.5, cells[:, 1] * 5.0 - 2.5
    w = np.full(x.size, 25.0)
    X = mk.candidates(pkg.workloads, d["xinc"], seed, it, ell)
    return x, y, w, X, d["prev"], d["rmax"], ell


def test_c5_poll293_fixture_regenerates(pkg):
    """CPU: the fixture's stream position reproduces a complete LTMADS poll (2n candidates on the
    granular mesh around the incumbent, steps bounded by 2^ell)."""
    x, y, w, X, prev, rmax, ell = _c5_poll293(pkg)
    n = X.shape[1]
    assert X.shape == (2 * n, n) and n == 3 * 512 and x.size == 192317
    xc = (X[0] + X[n]) / 2                      # the incumbent
    D = X[:n] - xc[None, :]
    assert np.all(D == np.round(D)) and np.abs(D).max() == 2 ** ell
    assert np.array_equal(X[n:], xc[None, :] - D)


@pytest.mark.gpu
@pytest.mark.parametrize("shared", ["auto", "bits", "fp64"])
def test_c5_poll293_against_oracle(ctx, pkg, orc, shared):
    """The slowest config-5 poll of rounds 3-4 (ell = 5: ~1,460 distinct positions per UAV, 132K
    shared entries): every shared-entry pass (auto = what the MADS loop runs, bits = the union
    pass forced, fp64 = the poll kernel's jobs) gives the same K objectives, 64 sampled
    candidates and the argmin equal the C oracle, and no sampled oracle objective is below the
    device's best."""
    x, y, w, X, prev, rmax, ell = _c5_poll293(pkg)
    N = X.shape[1] // 3
    tan50 = math.tan(100 / 180 * math.pi / 2)
    ctx.set_points(x, y, w)
    ctx.set_algo("auto")
    ctx.set_shared(shared)
    dl = np.full(N, 10.0)
    try:
        # without cons3 (every objective finite), twice: the second poll takes the lane's hint
        res = [ctx.poll_best(X, rmax, 1e5, want_all=True) for _ in range(2)]
        # with cons3 against the MPC step's start, as the loop ran it
        bo3, bi3, objs3 = ctx.poll_best(X, rmax, 1e5, prev=prev, d_lim=dl, tan_half_fov=tan50,
                                        want_all=True)
    finally:
        ctx.set_shared("auto")
    assert np.array_equal(res[0][2], res[1][2]) and res[0][:2] == res[1][:2]
    bo, bi, objs = res[1]
    rng = pkg.workloads.SplitMix64(293)
    pick = np.unique(np.concatenate([[0, bi], np.floor(rng.uniform(64) * X.shape[0]).astype(np.int64)]))
    lst = np.stack([x, y, w, w, np.zeros_like(x)], axis=1)
    area = orc.PointerList(lst).area_batch(X[pick], 16)
    viol = orc.violation_batch(X[pick], rmax)
    want = -area + viol * 1e5
    assert np.array_equal(objs[pick], want), pick[objs[pick] != want]
    assert want[np.searchsorted(pick, bi)] == bo
    assert bi == int(np.argmin(objs)) and bo == objs[bi]
    assert np.all(want >= bo)
    # cons3: the extreme barrier on top of the same objectives (the loop's poll: all infeasible
    # at ell = 5, every step is 32 m against d_lim = 10 m)
    ok3 = orc.cons3_batch(prev, X, dl, tan50)
    assert np.array_equal(objs3, np.where(ok3, objs, np.inf))
    assert bi3 == (int(np.argmin(objs3)) if np.isfinite(objs3).any() else -1)


@pytest.mark.gpu
@pytest.mark.parametrize("ell", [5, 4, 3])
def test_c5_poll293_takes_the_poll_walk(ctx, pkg, ell):
    """AUTO's walk choice on the crowded config-5 poll (k_poll_shared.h walk_choice): the poll walk
    at every mesh step. The per-candidate walk tests each visited entry against the disk's whole
    neighbour list; priced once per candidate (round 3) it was chosen at ell = 5 and took 7.1 ms
    against 0.69 ms (tools/c5_walks.py). Twice: the second call runs on the lane's hint."""
    x, y, w, X, prev, rmax, _ = _c5_poll293(pkg, ell_at=ell)
    ctx.set_points(x, y, w)
    ctx.set_algo("auto")
    walks = []
    cons3 = dict(prev=prev, d_lim=np.full(X.shape[1] // 3, 10.0),
                 tan_half_fov=math.tan(100 / 180 * math.pi / 2))
    for kw in ({}, {}, cons3, cons3):   # without and with cons3 (failures left out), as the loop
        ctx.profile(True)
        ctx.profile_read(reset=True)
        ctx.poll_best(X, rmax, 1e5, **kw)
        walks.append(ctx.profile_read(reset=True)[3])
        ctx.profile(False)
    assert walks == ["poll"] * 4, walks
