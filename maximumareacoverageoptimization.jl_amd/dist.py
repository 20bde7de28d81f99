"""Multi-GPU poll: candidate sharding + one 16-byte-per-rank all-gather of the local best.

One process per GPU (torch.distributed; backend "nccl" is RCCL on ROCm, over xGMI). Every rank
holds a full replica of the point list (403 MB at 16M fp64 entries, against 288 GB of HBM) and
evaluates the contiguous candidate slice [floor(rK/P), floor((r+1)K/P)). Its libmaxcover poll
writes {best objective (f64), best global index (i64 bits)} into a 16-byte device buffer; one
all_gather of those 16 B per rank (latency-bound, tens of microseconds) is the only data-path
collective, after which every rank takes the lexicographic minimum (objective, index): the
lowest index wins ties, the order in which a sequential poll keeps its first best.

The same exchange drives the multi-GPU MADS loop (config 5, `mads_loop`): every rank steps the
same LTMADS sequence over its shard of each poll and applies the same global best, so all ranks
hold the single-GPU loop's iterates. The point list needs no transfer either: the fire stream is
a deterministic counter-based CA, so every rank regenerates it on its own GPU (DynamicArea).
"""
from __future__ import annotations

import numpy as np


def shard_range(K: int, rank: int, world: int) -> tuple[int, int]:
    """Contiguous slice of the K candidates owned by `rank` (balanced to within one)."""
    if world <= 0 or not (0 <= rank < world):
        raise ValueError("bad rank/world")
    return (rank * K) // world, ((rank + 1) * K) // world


def reduce_best(objs: np.ndarray, idxs: np.ndarray) -> tuple[float, int]:
    """Lexicographic min over per-rank (objective, index); index -1 = rank had no candidate."""
    best_o, best_i = np.inf, -1
    for o, i in zip(np.asarray(objs, dtype=np.float64), np.asarray(idxs, dtype=np.int64)):
        if i < 0 or not (o < np.inf or o == -np.inf) or o != o:
            continue
        if best_i < 0 or o < best_o or (o == best_o and i < best_i):
            best_o, best_i = float(o), int(i)
    return best_o, best_i


_GATHER_OUT = {}


def gather_best(best16, group=None):
    """all_gather of the 16-byte {obj f64, idx i64} record; returns (obj, idx) lexicographic min.

    ``best16``: torch tensor of 2 float64 (the poll's d_best; the index is stored as raw int64
    bits). Works on any backend: RCCL for device tensors, gloo for CPU tensors. One collective
    into a preallocated (world x 2) buffer per (device, group), one 16*world-byte copy to the
    host: the per-poll cost is the collective's latency, not allocations."""
    import torch
    import torch.distributed as dist

    world = dist.get_world_size(group)
    key = (best16.device, id(group), world)
    out = _GATHER_OUT.get(key)
    if out is None:
        out = _GATHER_OUT[key] = torch.empty((world, 2), dtype=torch.float64, device=best16.device)
    if hasattr(dist, "all_gather_into_tensor"):
        dist.all_gather_into_tensor(out, best16.reshape(1, 2), group=group)
    else:   # pragma: no cover - older torch
        dist.all_gather(list(out.unbind(0)), best16, group=group)
    h = out.cpu()
    objs = h[:, 0].numpy().copy()
    idxs = h.view(torch.int64)[:, 1].numpy().copy()
    return reduce_best(objs, idxs)


def pack_best(obj: float, idx: int, device="cpu"):
    """Host-side constructor of the 16-byte record (for tests and CPU ranks)."""
    import torch

    t = torch.empty(2, dtype=torch.float64, device=device)
    t[0] = float(obj)
    t.view(torch.int64)[1] = int(idx)
    return t


def make_gather(device="cpu", group=None):
    """(obj, idx) -> the lexicographic minimum over all ranks' (obj, idx): one 16-byte all_gather
    per call (RCCL for a device tensor, gloo for a CPU one). Identity for a single process."""
    import torch.distributed as dist

    if not (dist.is_available() and dist.is_initialized()) or dist.get_world_size(group) == 1:
        return lambda obj, idx: (obj, idx)

    def gather(obj, idx):
        return gather_best(pack_best(obj, idx, device), group)

    return gather


def mads_loop(stepper, gather=None):
    """The sharded MADS loop's host side (mac_mads_poll / mac_mads_update, include/maxcover.h):
    per iteration the stepper polls its shard, ``gather`` combines the ranks' local bests and
    every rank applies the same global best. Returns stepper.result()."""
    while True:
        done, obj, idx = stepper.poll()
        if done:
            break
        if gather is not None:
            obj, idx = gather(obj, idx)
        stepper.update(obj, idx)
    return stepper.result()
