"""CPU, world_size 2 over gloo: candidate sharding + the 16-byte all-gather argmin give the
single-process poll result (the per-shard evaluation is the oracle here; on the GPU box it is
libmaxcover's poll, see bench.py)."""
import os
import socket

import numpy as np
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q, mode="strong"):
    import sys
    import torch
    import torch.distributed as dist
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path.insert(0, root)
    import __graft_entry__ as ge
    pkg = ge.load_package()
    orc = ge.load_oracle()
    from importlib import import_module
    d = import_module(pkg.__name__ + ".dist")
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    wl = pkg.workloads
    rng = wl.SplitMix64(77)
    x, y, w = wl.grid_points(40)
    rec = np.stack([x, y, w, w, np.zeros_like(x)], axis=1)
    x0 = wl.clustered_disks(6, 40, rng)
    C = wl.poll_candidates(x0, rng)
    # make ties: duplicate the best candidate at a later index on the other shard
    C = np.concatenate([C, C[:3]], axis=0)
    rmax = np.full(6, 36.0)
    if mode == "weak":
        # bench.py --scaling weak: every rank polls a whole candidate set of its own (rank r's set
        # drawn from its own stream), global index = r * K + k; the step's poll is the union
        sets = [C] + [wl.poll_candidates(x0, wl.SplitMix64(1000 + r)) for r in range(1, world)]
        K = C.shape[0]
        sets[1:] = [np.concatenate([s_, s_[:3]], axis=0) for s_ in sets[1:]]   # same K
        mine = sets[rank]
        lo = rank * K
        objs = np.array([orc.ref_objective(c, rec, rmax) for c in mine])
        C = np.concatenate(sets, axis=0)
    else:
        lo, hi = d.shard_range(C.shape[0], rank, world)
        objs = np.array([orc.ref_objective(c, rec, rmax) for c in C[lo:hi]])
    k = int(np.argmin(objs)) if objs.size else -1
    best = d.pack_best(objs[k] if k >= 0 else np.inf, lo + k if k >= 0 else -1)
    got = d.gather_best(best)
    allobj = np.array([orc.ref_objective(c, rec, rmax) for c in C])
    want = (float(allobj.min()), int(np.argmin(allobj)))
    q.put((rank, got, want))
    dist.destroy_process_group()


import pytest


@pytest.mark.parametrize("mode", ["strong", "weak"])
def test_gloo_world2_poll_argmin(mode):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q, mode)) for r in range(2)]
    for p in procs:
        p.start()
    res = [q.get(timeout=300) for _ in procs]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for rank, got, want in res:
        assert got == want, (rank, got, want)


def _mads_worker(rank, world, port, q):
    """The sharded MADS loop (dist.mads_loop over a PollStepper shard, 16-B gloo all-gather per
    iteration) against the single-process mads() on the same problem: the oracle evaluates."""
    import sys
    import torch.distributed as dist
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path.insert(0, root)
    import __graft_entry__ as ge
    pkg = ge.load_package()
    orc = ge.load_oracle()
    from importlib import import_module
    d = import_module(pkg.__name__ + ".dist")
    TS, TC = pkg.TDM_STATIC_opt, pkg.TDM_Constraints
    if world > 1:
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        dist.init_process_group("gloo", rank=rank, world_size=world)
    wl = pkg.workloads
    rng = wl.SplitMix64(515)
    x, y, w = wl.grid_points(48)
    rec = np.stack([x, y, w, w, np.zeros_like(x)], axis=1)
    N = 5
    x0 = np.concatenate([np.round(60 + rng.uniform(N) * 120), np.round(60 + rng.uniform(N) * 120),
                         np.full(N, 20.0)])
    rmax = np.full(N, 22.0)
    c3 = TC.create_cons3(x0, 100 / 180 * np.pi, np.full(N, 6.0))

    def obj(v):
        return orc.ref_objective(v, rec, rmax)

    def poll_fn(X):
        f = np.array([obj(v) if c3(v) else np.inf for v in X])
        k = int(np.argmin(f))
        return (f[k], k) if np.isfinite(f[k]) else (np.inf, -1)

    f0 = obj(x0) if c3(x0) else np.inf
    n = x0.size
    lo, hi = d.shard_range(2 * n, rank, world)
    st = TS.PollStepper(x0, f0, poll_fn, N_iter=25, ell0=2, ell_max=4, seed=99, shard=(lo, hi))
    xs, info = d.mads_loop(st, d.make_gather("cpu"))
    ref = TS.mads(x0, obj, [c3], N_iter=25, ell0=2, ell_max=4, seed=99)
    want_x = ref.x if ref.x is not None else ref.i
    q.put((rank, xs.tolist(), info["f"], info["iterations"], want_x.tolist(), ref.x_cost,
           ref.status.iteration))
    if world > 1:
        dist.destroy_process_group()


def test_gloo_world2_sharded_mads_loop():
    """World size 2: each rank polls half of every LTMADS poll; after the all-gather both hold
    the single-process MADS iterate, objective and iteration count."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_mads_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = [q.get(timeout=300) for _ in procs]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for rank, xs, f, it, want_x, want_f, want_it in res:
        assert xs == want_x and f == want_f and it == want_it, rank
    assert res[0][1] == res[1][1]


def _spec_worker(rank, world, port, q):
    """dist.mads_loop_speculative over gloo: rank j evaluates the whole poll that follows j
    failures (TDM_STATIC_opt.PollStepper.poll_ahead on the C oracle), SpecGather exchanges the
    results, every rank advances through them up to the first success."""
    import sys
    import torch.distributed as dist
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path.insert(0, root)
    import __graft_entry__ as ge
    pkg = ge.load_package()
    orc = ge.load_oracle()
    from importlib import import_module
    d = import_module(pkg.__name__ + ".dist")
    TS, TC = pkg.TDM_STATIC_opt, pkg.TDM_Constraints
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    wl = pkg.workloads
    rng = wl.SplitMix64(616)
    x, y, w = wl.grid_points(48)
    rec = np.stack([x, y, w, w, np.zeros_like(x)], axis=1)
    N = 4
    x0 = np.concatenate([np.round(60 + rng.uniform(N) * 120), np.round(60 + rng.uniform(N) * 120),
                         np.full(N, 20.0)])
    rmax = np.full(N, 22.0)
    c3 = TC.create_cons3(x0, 100 / 180 * np.pi, np.full(N, 6.0))

    def obj(v):
        return orc.ref_objective(v, rec, rmax)

    def poll_fn(X):
        f = np.array([obj(v) if c3(v) else np.inf for v in X])
        k = int(np.argmin(f))
        return (f[k], k) if np.isfinite(f[k]) else (np.inf, -1)

    f0 = obj(x0) if c3(x0) else np.inf
    st = TS.PollStepper(x0, f0, poll_fn, N_iter=30, ell0=3, ell_max=5, seed=41)
    xs, info = d.mads_loop_speculative(st, d.SpecGather("cpu"))
    ref = TS.mads(x0, obj, [c3], N_iter=30, ell0=3, ell_max=5, seed=41)
    want_x = ref.x if ref.x is not None else ref.i
    q.put((rank, xs.tolist(), info["f"], info["iterations"], info["rounds"], want_x.tolist(),
           ref.x_cost, ref.status.iteration))
    dist.destroy_process_group()


def test_gloo_speculative_mads_loop():
    """World sizes 2 and 3: the speculative loop (failure branches polled ahead on ranks
    1..P-1) holds the sequential MADS iterate, objective and iteration count on every rank, in
    fewer exchanges than iterations once failures run together."""
    for world in (2, 3):
        ctx = mp.get_context("spawn")
        q = ctx.Queue()
        port = _free_port()
        procs = [ctx.Process(target=_spec_worker, args=(r, world, port, q)) for r in range(world)]
        for p in procs:
            p.start()
        res = [q.get(timeout=300) for _ in procs]
        for p in procs:
            p.join(timeout=60)
            assert p.exitcode == 0
        for rank, xs, f, it, rounds, want_x, want_f, want_it in res:
            assert xs == want_x and f == want_f and it == want_it, (world, rank)
            assert rounds < it, (world, rounds, it)


def _bcast_worker(rank, world, port, q):
    import sys
    import torch.distributed as dist
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path.insert(0, root)
    import __graft_entry__ as ge
    pkg = ge.load_package()
    from importlib import import_module
    d = import_module(pkg.__name__ + ".dist")
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    x, y, w = pkg.workloads.grid_points(30)
    args = (x, y, w) if rank == 0 else (None, None, None)
    bx, by, bw = d.broadcast_points(*args)
    e0 = d.broadcast_points(*(([], [], []) if rank == 0 else (None, None, None)))
    q.put((rank, np.array_equal(bx.numpy(), x) and np.array_equal(by.numpy(), y)
           and np.array_equal(bw.numpy(), w), int(e0[0].numel())))
    dist.destroy_process_group()


def test_gloo_world2_broadcast_points():
    """The point list of rank 0 arrives bit-identical on every rank in one broadcast; an empty
    batch broadcasts as empty."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_bcast_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = [q.get(timeout=300) for _ in procs]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for rank, same, n_empty in res:
        assert same and n_empty == 0, rank


def _pollgather_worker(rank, world, port, q):
    """dist.PollGather on gloo (the bench's strong-mode exchange, CPU records): every rank's
    16-B {objective, index} record in, the lexicographic minimum over ranks out, per call, with
    ties to the lowest index and empty shards ({+inf, -1}) ignored."""
    import sys
    import torch.distributed as dist
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path.insert(0, root)
    import __graft_entry__ as ge
    pkg = ge.load_package()
    from importlib import import_module
    d = import_module(pkg.__name__ + ".dist")
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    g = d.PollGather("cpu")
    cases = [((5.0, 10), (4.0, 700)), ((3.0, 12), (3.0, 9)), ((np.inf, -1), (7.5, 1500)),
             ((np.inf, -1), (np.inf, -1)), ((-2.0, 3), (-2.0, 2000))]
    out = [g(d.pack_best(*c[rank])) for c in cases]
    q.put((rank, out, g.calls))
    dist.destroy_process_group()


def test_gloo_world2_poll_gather():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_pollgather_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = [q.get(timeout=300) for _ in procs]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    want = [(4.0, 700), (3.0, 9), (7.5, 1500), (np.inf, -1), (-2.0, 3)]
    for rank, out, calls in res:
        assert out == want and calls == 5, rank
