"""GPU parity of the fp32 entry points (*_f32, include/maxcover.h; SURVEY 8(b), config 3 "fp32").

The reference has one Float64 path (calculateArea(circles::Vector{Float64}, ...),
src/AreaCoverageCalculation.jl:63). An fp32 caller's values reach it as Float64(::Float32), which
is exact; the *_f32 entry points widen the same way on the device, so their results must equal the
fp64 evaluation (the oracle, and the *_f64 calls) of the widened inputs bit for bit.
"""
import math

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

TAN50 = math.tan(100 / 180 * math.pi / 2)


def recs(x, y, w):
    return np.stack([x, y, w, w, np.zeros_like(x)], axis=1)


def test_f32_config3_full_poll(ctx, pkg, orc):
    """Config 3 as fp32 (128 UAVs x 4.2M cells, K = 769): points (i - 1/2) * 5 and integer disks
    are exact in fp32, so every area equals 25 x the exact lattice count and the fp64 call's
    result; objectives, cons3 and the argmin equal the fp64 poll's bit for bit (auto and the
    poll walk)."""
    x, y, w, C, rmax = pkg.workloads.make_config(3)
    assert np.array_equal(x.astype(np.float32).astype(np.float64), x)
    ctx.set_points_f32(x.astype(np.float32), y.astype(np.float32), w.astype(np.float32))
    assert ctx.num_points == x.size
    C32 = C.astype(np.float32)
    assert np.array_equal(C32.astype(np.float64), C)
    cnt = orc.lattice_count_batch(C, 2048)
    dlim = np.full(128, 5.0)
    for algo in ("auto", "poll", "tiled"):
        ctx.set_algo(algo)
        got = ctx.area_batch_f32(C32)
        assert np.array_equal(got, 25.0 * cnt.astype(np.float64)), algo
        b64 = ctx.poll_best(C, rmax, 1e5, prev=C[0], d_lim=dlim, tan_half_fov=TAN50, want_all=True)
        b32 = ctx.poll_best_f32(C32, rmax, 1e5, prev=C32[0], d_lim=dlim, tan_half_fov=TAN50,
                                want_all=True)
        assert b32[0] == b64[0] and b32[1] == b64[1], algo
        assert np.array_equal(b32[2], b64[2]), algo
    ctx.set_algo("auto")
    assert ctx.area_f32(C32[5]) == 25.0 * cnt[5]


def test_f32_real_values_vs_oracle(ctx, pkg, orc):
    """Real-valued fp32 coordinates (not on any lattice): the oracle on the widened doubles."""
    wl = pkg.workloads
    rng = wl.SplitMix64(3232)
    M = 50000
    x = (rng.uniform(M) * 600.0).astype(np.float32)
    y = (rng.uniform(M) * 600.0).astype(np.float32)
    w = np.full(M, 25.0, dtype=np.float32)
    ctx.set_points_f32(x, y, w)
    N = 24
    x0 = np.concatenate([300 + rng.uniform(N) * 200 - 100, 300 + rng.uniform(N) * 200 - 100,
                         rng.uniform(N) * 25 + 10])
    C = np.concatenate([x0[None, :], wl.poll_candidates(x0, rng, ell=1)], axis=0)
    C[1:] += (rng.uniform(C[1:].size) * 0.3).reshape(C[1:].shape)
    C32 = C.astype(np.float32)
    Cw = C32.astype(np.float64)
    rec = recs(x.astype(np.float64), y.astype(np.float64), w.astype(np.float64))
    want = orc.PointerList(rec).area_batch(Cw)
    for algo in ("auto", "poll", "tiled", "scan"):
        ctx.set_algo(algo)
        got = ctx.area_batch_f32(C32)
        assert np.array_equal(got, want), (algo, np.flatnonzero(got != want)[:5])
    ctx.set_algo("auto")
    rmax = np.full(N, 30.0 * TAN50)
    want_obj = np.array([orc.ref_objective(c, rec, rmax) for c in Cw])
    bo, bi, objs = ctx.poll_best_f32(C32, rmax, want_all=True)
    assert np.array_equal(objs, want_obj)
    k = int(np.argmin(want_obj))
    assert bi == k and bo == want_obj[k]


def test_f32_device_poll(ctx, pkg, orc):
    """mac_poll_best_dev_f32 (fp32 device matrix, widened on the stream) == the fp64 device poll."""
    torch = pytest.importorskip("torch")
    x, y, w, C, rmax = pkg.workloads.make_config(3)
    ctx.set_points(x, y, w)
    dev = torch.device("cuda", 0)
    K, n3 = C.shape
    d32 = torch.from_numpy(np.ascontiguousarray(C.astype(np.float32))).to(dev)
    d64 = torch.from_numpy(np.ascontiguousarray(C)).to(dev)
    d_rmax = torch.from_numpy(rmax).to(dev)
    d_prev32 = d32[0].contiguous()
    d_prev64 = d64[0].contiguous()
    d_dlim = torch.full((n3 // 3,), 5.0, dtype=torch.float64, device=dev)
    o32 = torch.empty(K, dtype=torch.float64, device=dev)
    o64 = torch.empty(K, dtype=torch.float64, device=dev)
    b32 = torch.empty(2, dtype=torch.float64, device=dev)
    b64 = torch.empty(2, dtype=torch.float64, device=dev)
    ctx.poll_best_dev_f32(d32, n3, K, d_rmax, b32, d_prev=d_prev32, d_dlim=d_dlim,
                          tan_half_fov=TAN50, d_obj=o32)
    r32 = ctx.best_fetch(b32)
    ctx.poll_best_dev(d64, n3, K, d_rmax, b64, d_prev=d_prev64, d_dlim=d_dlim,
                      tan_half_fov=TAN50, d_obj=o64)
    r64 = ctx.best_fetch(b64)
    torch.cuda.synchronize()
    assert r32 == r64
    assert torch.equal(o32, o64)


def test_f32_storage_option_refused(ctx, pkg):
    """The list is kept in fp64: MAC_STORE_F32 is refused, not faked."""
    with pytest.raises(pkg.MaxCoverError):
        ctx.set_option(pkg._lib.MAC_OPT_STORAGE, pkg._lib.MAC_STORE_F32)
    ctx.set_option(pkg._lib.MAC_OPT_STORAGE, pkg._lib.MAC_STORE_F64)
