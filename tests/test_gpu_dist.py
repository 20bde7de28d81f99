"""GPU: the RCCL side of the multi-GPU exchanges (dist.py) on the one GPU a box has — a world of
one rank with the nccl (= RCCL) backend, so the device collectives, events and pinned reads of
the strong step (PollGather), of the sharded MADS loop (DeviceGather bound to a stepper) and of
the point broadcast run as they do on the 8-GPU node (the gloo tests in test_dist.py cover two
ranks on the CPU). Reference: src/TDM_STATIC_opt.jl:129 (the poll the ranks split)."""
import math
import os
import socket
from importlib import import_module

import numpy as np
import pytest

pytestmark = pytest.mark.gpu
TAN50 = math.tan(100 / 180 * math.pi / 2)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.fixture(scope="module")
def nccl1(ctx):
    import torch
    import torch.distributed as dist

    os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{_free_port()}", rank=0,
                            world_size=1, device_id=dev)
    assert dist.get_backend() == "nccl"
    yield dev
    dist.destroy_process_group()


@pytest.mark.parametrize("reduce", ["host", "device"])
def test_poll_gather_over_rccl(nccl1, ctx, pkg, reduce):
    """PollGather (bench.py's multi-GPU step): each device poll's d_best goes through the RCCL
    all-gather and either the pinned record + host argmin or the device argmin
    (mac_best_reduce_dev) + mapped slot; the result equals the poll's own (objective, index) from
    mac_poll_best_f64, poll after poll, with no allocation in between."""
    import torch

    d = import_module(pkg.__name__ + ".dist")
    wl = pkg.workloads
    x, y, w = wl.grid_points(256)
    ctx.set_points(x, y, w)
    rng = wl.SplitMix64(71)
    N = 16
    rmax = np.full(N, 30.0 * TAN50)
    d_rmax = torch.from_numpy(rmax).to(nccl1)
    d_best = torch.empty(2, dtype=torch.float64, device=nccl1)
    gather = d.PollGather(nccl1, ctx=ctx if reduce == "device" else None)
    out_ptr = gather.out.data_ptr()
    # the polls and the gather on one stream of the caller's (as bench.py's ranks do); the
    # default-stream variant is the next test
    s = torch.cuda.Stream(nccl1)
    with torch.cuda.stream(s):
        for t in range(5):
            C = wl.poll_candidates(wl.uniform_disks(N, 256, rng), rng)
            want = ctx.poll_best(C, rmax)
            d_c = torch.from_numpy(np.ascontiguousarray(C)).to(nccl1)
            ctx.poll_best_dev(d_c, 3 * N, C.shape[0], d_rmax, d_best, stream=s.cuda_stream)
            got = gather(d_best)
            assert got == (want[0], want[1]), (t, got, want)
    assert gather.calls == 5 and gather.out.data_ptr() == out_ptr


@pytest.mark.parametrize("reduce", ["host", "device"])
def test_poll_gather_over_rccl_default_stream(nccl1, ctx, pkg, reduce):
    """The same exchange with no stream of the caller's: the candidates are copied, the poll
    enqueued (stream=None) and the all-gather issued on torch's default stream, with no
    synchronisation in between. stream=None is torch's current stream, which here is HIP's null
    stream — the C ABI's NULL (include/maxcover.h) — so the poll is ordered after the copy of its
    candidates and before the all-gather that reads its d_best. (Round 4 mapped NULL to a private
    stream of the context: this exact sequence returned another poll's argmin at poll 4.)"""
    import torch

    d = import_module(pkg.__name__ + ".dist")
    wl = pkg.workloads
    x, y, w = wl.grid_points(256)
    ctx.set_points(x, y, w)
    rng = wl.SplitMix64(71)
    N = 16
    rmax = np.full(N, 30.0 * TAN50)
    d_rmax = torch.from_numpy(rmax).to(nccl1)
    d_best = torch.empty(2, dtype=torch.float64, device=nccl1)
    gather = d.PollGather(nccl1, ctx=ctx if reduce == "device" else None)
    assert torch.cuda.current_stream(nccl1).cuda_stream == 0
    for t in range(6):
        C = wl.poll_candidates(wl.uniform_disks(N, 256, rng), rng)
        want = ctx.poll_best(C, rmax)
        d_c = torch.from_numpy(np.ascontiguousarray(C)).to(nccl1)
        ctx.poll_best_dev(d_c, 3 * N, C.shape[0], d_rmax, d_best)          # stream=None
        got = gather(d_best)
        assert got == (want[0], want[1]), (t, got, want)
        # the raw C NULL (an int 0 handle) is the same stream
        ctx.poll_best_dev(d_c, 3 * N, C.shape[0], d_rmax, d_best, stream=0)
        assert gather(d_best) == (want[0], want[1]), t


def test_sharded_mads_loop_over_rccl(nccl1, ctx, pkg):
    """dist.mads_loop with the RCCL DeviceGather bound to the stepper's device best buffer (the
    config-5 multi-GPU loop's exchange): the same iterate, objective and counts as mac_mads_run."""
    d = import_module(pkg.__name__ + ".dist")
    wl = pkg.workloads
    x, y, w = wl.grid_points(200)
    ctx.set_points(x, y, w)
    rng = wl.SplitMix64(404)
    N = 9
    x0 = np.concatenate([np.round(250 + rng.uniform(N) * 400), np.round(250 + rng.uniform(N) * 400),
                         np.full(N, 30.0)])
    r_max = np.full(N, 30.0 * TAN50)
    kw = dict(prev=x0, d_lim=np.full(N, 10.0), tan_half_fov=TAN50, n_iter=25, ell0=2, ell_max=5,
              seed=909)
    want_x, want = ctx.mads_run(x0, r_max, 1e5, **kw)
    # (make_gather is the identity for a world of one: the RCCL gather is bound explicitly)
    gather = d.DeviceGather(nccl1)
    st = ctx.mads_stepper(x0, r_max, 1e5, shard=(0, 2 * x0.size), **kw)
    xs, stats = d.mads_loop(st, gather)
    st.close()
    assert np.array_equal(xs, want_x)
    assert stats["f"] == want["f"] and stats["iterations"] == want["iterations"]
    assert gather.calls == want["iterations"]
    assert stats["slot_fallbacks"] == 0   # every poll's best read through the mapped slot


def test_broadcast_points_over_rccl(nccl1, pkg):
    """broadcast_points over RCCL from rank 0's host arrays to device tensors, bit for bit."""
    d = import_module(pkg.__name__ + ".dist")
    rng = np.random.default_rng(5)
    x, y, w = rng.normal(size=1000), rng.normal(size=1000), rng.uniform(size=1000)
    gx, gy, gw = d.broadcast_points(x, y, w, src=0, device=nccl1)
    assert gx.device.type == "cuda"
    for a, b in ((gx, x), (gy, y), (gw, w)):
        assert np.array_equal(a.cpu().numpy(), b)


def test_best_reduce_dev_matches_reduce_best(ctx, pkg):
    """mac_best_reduce_dev (the device side of the multi-GPU exchange) against dist.reduce_best on
    record sets with ties (lowest index wins), empty shards (index -1), +inf / NaN objectives
    (never selected), -inf, no record at all and more records than one wave (130)."""
    import torch

    d = import_module(pkg.__name__ + ".dist")
    dev = torch.device("cuda", 0)
    cases = [
        [(3.0, 7), (1.0, 9), (1.0, 4), (2.0, 1)],
        [(np.inf, -1), (np.inf, -1)],
        [(np.inf, 3), (np.nan, 2), (5.0, -1)],
        [(-np.inf, 8), (-1e300, 2), (-np.inf, 5)],
        [],
        [(float(v), int(i)) for v, i in zip(np.random.default_rng(3).integers(0, 4, 130),
                                            np.random.default_rng(4).permutation(130))],
    ]
    res = torch.empty(2, dtype=torch.float64, device=dev)
    for recs in cases:
        rec = torch.zeros((max(len(recs), 1), 2), dtype=torch.float64)
        for j, (o, i) in enumerate(recs):
            rec[j, 0] = o
            rec.view(torch.int64)[j, 1] = i
        drec = rec.to(dev)
        ctx.best_reduce_dev(drec, len(recs), res, stream=0)
        got = ctx.best_fetch(res, stream=0)
        want = d.reduce_best([o for o, _ in recs], [i for _, i in recs])
        assert got[1] == want[1] and (got[0] == want[0] or (want[1] < 0 and got[0] == np.inf)), \
            (recs[:6], got, want)


def test_rccl_exchange_in_library(nccl1, ctx, pkg):
    """dist.RcclExchange (bench.py's default multi-GPU step over RCCL): libmaxcover's own RCCL
    communicator (id from rank 0, broadcast once), then per poll one C call — the all-gather of the
    16-B d_best on the poll's stream, the device argmin and the mapped-slot read. Poll after poll
    its (objective, index) equals mac_poll_best_f64's, on a caller's stream and on torch's default
    (null) stream, with and without cons3."""
    import torch

    d = import_module(pkg.__name__ + ".dist")
    wl = pkg.workloads
    x, y, w = wl.grid_points(256)
    with pkg.Context(0) as c2:   # (a context of its own: the communicator lives with it)
        c2.set_points(x, y, w)
        ex = d.RcclExchange(c2, nccl1)
        rng = wl.SplitMix64(73)
        N = 16
        rmax = np.full(N, 30.0 * TAN50)
        d_rmax = torch.from_numpy(rmax).to(nccl1)
        d_best = torch.empty(2, dtype=torch.float64, device=nccl1)
        s = torch.cuda.Stream(nccl1)
        for t in range(6):
            C = wl.poll_candidates(wl.uniform_disks(N, 256, rng), rng, ell=3)
            kw = dict(prev=C[0], d_lim=np.full(N, 10.0), tan_half_fov=TAN50) if t % 2 else {}
            want = c2.poll_best(C, rmax, 1e5, **kw)
            d_c = torch.from_numpy(np.ascontiguousarray(C)).to(nccl1)
            dkw = dict(d_prev=torch.from_numpy(C[0].copy()).to(nccl1),
                       d_dlim=torch.full((N,), 10.0, dtype=torch.float64, device=nccl1),
                       tan_half_fov=TAN50) if t % 2 else {}
            if t < 3:
                with torch.cuda.stream(s):
                    c2.poll_best_dev(d_c, 3 * N, C.shape[0], d_rmax, d_best, stream=s.cuda_stream, **dkw)
                    got = ex(d_best)
            else:
                torch.cuda.synchronize()
                c2.poll_best_dev(d_c, 3 * N, C.shape[0], d_rmax, d_best, **dkw)   # torch's default stream
                got = ex(d_best)
            assert got == (want[0], want[1]), (t, got, want)
        assert ex.calls == 6
        torch.cuda.synchronize()


@pytest.mark.parametrize("mode", ["shard", "speculate"])
def test_mads_loops_over_the_library_exchange(nccl1, pkg, mode):
    """The config-5 multi-GPU loops over libmaxcover's own RCCL communicator: the sharded loop with
    dist.RcclShardGather (the stepper's device best buffer all-gathered and reduced on the device,
    mac_poll_exchange) and the speculative loop with dist.RcclSpecGather (every rank's 32-B record,
    mac_exchange_records). Same iterate, objective and iteration count as mac_mads_run."""
    d = import_module(pkg.__name__ + ".dist")
    wl = pkg.workloads
    x, y, w = wl.grid_points(200)
    rng = wl.SplitMix64(505)
    N = 9
    x0 = np.concatenate([np.round(250 + rng.uniform(N) * 400), np.round(250 + rng.uniform(N) * 400),
                         np.full(N, 30.0)])
    r_max = np.full(N, 30.0 * TAN50)
    kw = dict(prev=x0, d_lim=np.full(N, 10.0), tan_half_fov=TAN50, n_iter=30, ell0=2, ell_max=5,
              seed=919)
    with pkg.Context(0) as c2:
        c2.set_points(x, y, w)
        want_x, want = c2.mads_run(x0, r_max, 1e5, **kw)
        st = c2.mads_stepper(x0, r_max, 1e5, **kw)
        try:
            if mode == "shard":
                g = d.RcclShardGather(c2, nccl1)
                xs, stats = d.mads_loop(st, g)
                assert g.calls == want["iterations"] and stats["slot_fallbacks"] == 0
            else:
                g = d.RcclSpecGather(c2, nccl1)
                xs, stats = d.mads_loop_speculative(st, g)
                # (one rank: one iteration per round, and the round that finds the loop done)
                assert stats["rounds"] == want["iterations"] + 1
                assert stats["feasible_evaluations"] == want["feasible_evaluations"]
        finally:
            st.close()
    assert np.array_equal(xs, want_x)
    assert stats["f"] == want["f"] and stats["iterations"] == want["iterations"]
