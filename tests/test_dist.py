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
