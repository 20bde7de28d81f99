"""CPU: the oracle itself, pinned against the reference's data and integer known answers."""
import math
import os

import numpy as np
import pytest


def test_c_and_numpy_restatements_agree(orc, pkg):
    wl = pkg.workloads
    rng = wl.SplitMix64(11)
    for _ in range(20):
        M = int(rng.integers(0, 3000, 1)[0])
        x = rng.uniform(M) * 200 - 20
        y = rng.uniform(M) * 200 - 20
        w = rng.uniform(M) * 3
        N = int(rng.integers(1, 12, 1)[0])
        c = np.concatenate([rng.uniform(N) * 200, rng.uniform(N) * 200, rng.uniform(N) * 40])
        rec = np.stack([x, y, w, w, np.zeros(M)], axis=1) if M else np.zeros((0, 5))
        assert orc.ref_area(c, rec) == orc.np_area(c, x, y, w)


def test_lattice_kat_matches_oracle(orc, pkg):
    wl = pkg.workloads
    rng = wl.SplitMix64(12)
    x, y, w = wl.grid_points(50)
    rec = np.stack([x, y, w, w, np.zeros_like(x)], axis=1)
    for N in (1, 2, 7, 25):
        c = wl.uniform_disks(N, 50, rng)
        c[2 * N:] = rng.integers(1, 60, N)
        assert orc.ref_area(c, rec) == 25.0 * orc.lattice_count_np(c.astype(np.int64), 50)
    c = np.array([10.0, 20.0, 7.0])
    assert orc.lattice_count(c, 12) == orc.lattice_count_np(c, 12)


def test_golden_vectors_reproduce(orc, pkg, golden, firepoints):
    """The committed vectors are what the C oracle computes now (guards oracle drift)."""
    ACC = pkg.AreaCoverageCalculation
    poi = ACC.createPOI(5.0, 5.0, 100.0, 100.0)
    for c, a, o in zip(golden["A_cands"], golden["A_area"], golden["A_obj"]):
        assert orc.ref_area(c, poi) == a
        assert orc.ref_objective(c, poi, golden["A_rmax"]) == o
    fp10 = np.concatenate(firepoints[:10])
    for c, a in zip(golden["B_cands"], golden["B_area10"]):
        assert orc.ref_area(c, fp10) == a
    for k, c in enumerate(golden["D_cands"]):
        N = int(golden["D_N"][k])
        cc = c[: 3 * N]
        x, y, w = pkg.workloads.grid_points(64)
        rec = np.stack([x, y, w, w, np.zeros_like(x)], axis=1)
        assert orc.ref_area(cc, rec) == 25.0 * golden["D_count"][k]


def test_firepoints_fixture_shape(firepoints):
    """Pins the converted reference data to SURVEY.md's measurements (68 rows, 6,276 entries,
    3,061 unique (x,y), all weights 25, rows 1-10 = 455 entries)."""
    assert len(firepoints) == 68
    allp = np.concatenate(firepoints)
    assert allp.shape == (6276, 5)
    assert len({(a, b) for a, b in allp[:, :2]}) == 3061
    assert np.all(allp[:, 3] == 25.0) and np.all(allp[:, 2] == 25.0)
    assert sum(len(r) for r in firepoints[:10]) == 455
    # half-integer offsets: multiples of 5 minus 2.5
    assert np.all(np.mod(allp[:, :2] + 2.5, 5.0) == 0)


def test_reference_start_covers_nothing_of_rows_1_10(orc, pkg, firepoints):
    """the reference start point covers none of FirePoints rows 1..10."""
    BF = pkg.Base_Functions
    x0 = BF.allocate_even_circles(15.0, 5, 10 * math.tan(100 / 180 * math.pi / 2), 250.0, 250.0)
    assert orc.ref_area(x0, np.concatenate(firepoints[:10])) == 0.0


def test_inexact_error(orc):
    with pytest.raises(orc.InexactError):
        orc.ref_area(np.zeros(4), np.zeros((3, 5)))


def test_threshold_exact(pkg, orc):
    """The library's exact threshold (host build) equals the rational-arithmetic one."""
    rs = [1.0, 2.0, 36.0, 35.75261336008773, 5e-324, 1e-310, 2.0 ** -1022, 1e308,
          1.7976931348623157e308, math.inf, 0.0, -1.0, math.nan]
    rng = np.random.default_rng(3)
    rs += list(rng.uniform(0, 100, 500)) + list(np.exp(rng.uniform(-740, 709, 500)))
    rs += [2.0 ** e for e in range(-1074, 1024, 7)]
    for r in rs:
        assert pkg.cover_threshold(r) == orc.exact_threshold(r) or (
            math.isnan(r) and pkg.cover_threshold(r) == -1.0), r
    for r in rs[:600]:
        T = pkg.cover_threshold(r)
        if not (T >= 0):
            continue
        for a in (T, math.nextafter(T, math.inf), math.nextafter(T, 0.0), r * r):
            if 0 <= a < math.inf:
                assert (math.sqrt(a) < r) == (a <= T)


def test_remove_covered_oracle_order(orc, pkg, golden):
    poi = pkg.AreaCoverageCalculation.createPOI(5.0, 5.0, 100.0, 100.0)
    kept = orc.ref_remove_covered(golden["A_rmv_cand"], poi)
    assert np.array_equal(kept, golden["A_rmv_kept"])
    assert np.all(np.diff(kept) > 0)


def test_cons3_oracle_matches_host_mirror(orc, pkg, golden):
    TC = pkg.TDM_Constraints
    prev = golden["A_prev"]
    cons3 = TC.create_cons3(prev, 100 / 180 * math.pi, golden["A_dlim"])
    for c, f in zip(golden["A_cands"], golden["A_cons3"]):
        assert cons3(c) == bool(f) == orc.ref_cons3(prev, c, golden["A_dlim"], golden["A_tan"][0])


def test_reference_mads_outputs_on_mesh_and_cons3_feasible(orc, pkg, quadrotor_steps):
    """The reference's only recorded outputs on this path (UAV 1's MADS targets of its static
    N = 5 run, Quadrotor_Targets.xlsx, with the UAV states of Quadrotor_States*.xlsx; converted
    by tests/golden/make_quadrotor_fixture.py): every target lies on the granular mesh the
    build's LTMADS driver uses (integer x, y and R = z tan(FOV/2); granularity 1.0,
    src/TDM_STATIC_opt.jl:131-137), and passes cons3 (src/TDM_Constraints.jl:54-75, d_lim = 10 m,
    src/FullSimulation.jl:740) against where its step started, through the C oracle and the host
    mirror alike — the restated extreme barrier rejects none of the reference's own accepted
    points; a point 10.5 m from the start fails it (the check has teeth). The other UAVs'
    targets were never written (src/FullSimulation.jl:370-374), so objectives cannot be replayed."""
    steps, tan = quadrotor_steps
    assert len(steps) == 40
    fov = 100 / 180 * math.pi
    for prev, tgt in steps:
        assert tgt[0] == round(tgt[0]) and tgt[1] == round(tgt[1])
        assert abs(tgt[2] - round(tgt[2])) < 1e-9
        cand = np.array([tgt[0], tgt[1], float(round(tgt[2]))])
        assert orc.ref_cons3(prev, cand, np.array([10.0]), tan)
        assert pkg.TDM_Constraints.create_cons3(prev, fov, np.array([10.0]))(cand)
        far = np.array([prev[0] + 10.5, prev[1], prev[2]])   # 10.5 m from the start
        assert not orc.ref_cons3(prev, far, np.array([10.0]), tan)


def test_reference_second_recording_targets_on_mesh():
    """The longer recording under src/ (src/Quadrotor_Targets.xlsx, 120 MPC steps of UAV 1's
    MADS targets; converted by tests/golden/make_quadrotor_fixture.py). Its state files come
    from other runs (40/120/120/60 rows), so the start of each step is unknown and only the mesh
    is pinned: integer x, y and R = z tan(FOV/2) integral (granularity 1.0,
    src/TDM_STATIC_opt.jl:131-137) — the lattice the build's poll candidates are generated on."""
    D = np.loadtxt(os.path.join(os.path.dirname(__file__), "golden", "quadrotor_run_src.csv"),
                   delimiter=",", comments="#")
    assert D.shape == (120, 3)
    tan = math.tan(100 / 180 * math.pi / 2)
    assert np.array_equal(D[:, :2], np.round(D[:, :2]))
    R = D[:, 2] * tan
    assert np.abs(R - np.round(R)).max() < 1e-9
    assert (np.round(R) >= 1).all()
