"""CPU: host-side logic of the package (generators, mirrors that need no GPU)."""
import math

import numpy as np
import pytest


def test_splitmix64_known_values(pkg):
    # splitmix64 from seed 0: first outputs (published reference values)
    r = pkg.workloads.SplitMix64(0)
    v = r.next_u64(3)
    assert [int(a) for a in v] == [0xE220A8397B1DCDAF, 0x6E789E6AA1B965F4, 0x06C45D188009454F]


def test_ltmads_basis_structure(pkg):
    wl = pkg.workloads
    rng = wl.SplitMix64(5)
    for n, ell in ((6, 0), (15, 2), (48, 3)):
        B = wl.ltmads_basis(n, ell, rng)
        assert B.shape == (n, n)
        assert np.all(np.abs(B) <= 2 ** ell)
        # exactly one +-2^ell per row and per column (the permuted diagonal) and full rank
        # |det| = (2^ell)^n: a permuted triangular matrix with +-2^ell on the diagonal
        sign, logdet = np.linalg.slogdet(B.astype(float))
        assert sign != 0 and abs(logdet - n * ell * math.log(2)) < 1e-6
        assert np.all(np.sum(np.abs(B) == 2 ** ell, axis=0) >= 1)


def test_poll_candidates_shape(pkg):
    wl = pkg.workloads
    rng = wl.SplitMix64(6)
    x0 = wl.uniform_disks(5, 100, rng)
    C = wl.poll_candidates(x0, rng)
    assert C.shape == (31, 15)
    assert np.array_equal(C[0], x0)
    assert np.array_equal(C[1:16] - x0, -(C[16:] - x0))


def test_configs(pkg):
    for cfg, (G, N, K) in {2: (1024, 32, 1), 3: (2048, 128, 769), 4: (4096, 512, 3073)}.items():
        c = pkg.workloads.CONFIGS[cfg]
        assert (c["G"], c["N"], c["K"]) == (G, N, K)
        if cfg == 4:
            assert 6 * N + 1 == K


def test_createPOI_matches_oracle(pkg, orc):
    for args in ((5.0, 5.0, 100.0, 100.0), (1.0, 2.0, 3.0, 7.0), (2.5, 5.0, 10.5, 4.0)):
        assert np.array_equal(pkg.AreaCoverageCalculation.createPOI(*args), orc.ref_create_poi(*args))


def test_make_circles_roundtrip(pkg):
    ACC = pkg.AreaCoverageCalculation
    x = np.arange(12, dtype=float)
    assert np.array_equal(ACC.make_MADS(ACC.make_circles(x)), x)
    with pytest.raises(pkg.InexactError):
        ACC.make_circles(np.zeros(7))
    with pytest.raises(pkg.InexactError):
        ACC.calculateArea(np.zeros(5), np.zeros((1, 5)))


def test_allocate_even_circles_matches_oracle(pkg, orc):
    t = 10 * math.tan(100 / 180 * math.pi / 2)
    a = pkg.Base_Functions.allocate_even_circles(15.0, 5, t, 250.0, 250.0)
    assert np.array_equal(a, orc.ref_allocate_even_circles(15.0, 5, t, 250.0, 250.0))


def test_cells_initialise_dynamic(pkg, firepoints):
    CF = pkg.CellFunctions
    c = CF.initialise_POI(CF.Cells(), "dynamic", firepoints)
    assert c.points_of_interest.shape == (455, 5)
    CF.update_POI(c, 1, firepoints)
    assert c.points_of_interest.shape == (455, 5)
    CF.update_POI(c, 2, firepoints)   # appends row 12 (row 11 is never read)
    assert c.points_of_interest.shape[0] == 455 + len(firepoints[11])
    s = CF.initialise_POI(CF.Cells(), "static")
    assert s.points_of_interest.shape == (10000, 5)


def test_shard_range_and_reduce(pkg):
    from importlib import import_module
    d = import_module(pkg.__name__ + ".dist")
    for K in (0, 1, 7, 3073):
        for P in (1, 2, 3, 8):
            cuts = [d.shard_range(K, r, P) for r in range(P)]
            assert cuts[0][0] == 0 and cuts[-1][1] == K
            assert all(cuts[i][1] == cuts[i + 1][0] for i in range(P - 1))
    o, i = d.reduce_best(np.array([3.0, 1.0, 1.0, np.inf]), np.array([5, 9, 4, -1]))
    assert (o, i) == (1.0, 4)
    assert d.reduce_best(np.array([np.inf]), np.array([-1])) == (np.inf, -1)
    assert d.reduce_best(np.array([np.nan, 2.0]), np.array([0, 1])) == (2.0, 1)
