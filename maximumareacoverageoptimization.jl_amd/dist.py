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
hold the single-GPU loop's iterates. The config-5 point list needs no transfer: the fire stream
is a deterministic counter-based CA, so every rank regenerates it on its own GPU (DynamicArea).
A list no rank can regenerate (the FirePoints table, an external feed) goes out from one rank by
one broadcast of the packed list (`broadcast_points`) instead of a host upload per rank.
"""
from __future__ import annotations

import numpy as np

from ._lib import check_one_runtime


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


class PollGather:
    """The multi-GPU poll's exchange without per-poll allocations or pageable copies: the poll's
    16-B d_best (device) goes into ONE all-gather into a persistent (world x 2) buffer, ordered
    after the poll on torch's current stream (the caller's poll stream).

    With ``ctx`` (a libmaxcover Context on this rank's GPU) the world records are reduced ON THE
    DEVICE: mac_best_reduce_dev (one wave, ordered after the collective on the same stream) writes
    the lexicographic minimum to a persistent 16-B buffer and its mapped host slot, and
    mac_best_fetch reads that slot as soon as it lands — no device-to-host copy, event or stream
    synchronisation, no host argmin. Without ``ctx``: one pinned host read of the world x 16 B
    and the minimum on the host. On gloo (CPU rehearsal) d_best is first copied into a persistent
    pinned CPU record. ``seconds`` / ``calls``: host time spent here per poll."""

    def __init__(self, device, group=None, ctx=None):
        import torch
        import torch.distributed as dist

        self.group = group
        self.world = dist.get_world_size(group)
        self.device = torch.device(device)
        self.on_device = self.device.type == "cuda"
        if self.on_device:
            check_one_runtime()
        pin = torch.cuda.is_available()
        self.out = torch.empty((self.world, 2), dtype=torch.float64, device=self.device)
        self.host = (torch.empty((self.world, 2), dtype=torch.float64, pin_memory=pin)
                     if self.on_device else self.out)
        self.rec = None if self.on_device else torch.empty(2, dtype=torch.float64, pin_memory=pin)
        self.done = torch.cuda.Event() if self.on_device else None
        self.ctx = ctx if self.on_device else None
        self.res = (torch.empty(2, dtype=torch.float64, device=self.device)
                    if self.ctx is not None else None)
        self._reduce = {}   # stream handle -> bound reduce + fetch (Context.reduce_step)
        self.seconds = 0.0
        self.calls = 0

    def __call__(self, best16):
        import time
        import torch
        import torch.distributed as dist

        t0 = time.perf_counter()
        if self.ctx is not None:
            dist.all_gather_into_tensor(self.out, best16.reshape(1, 2), group=self.group)
            # (the collective's completion is ordered before torch's current stream's next work)
            sh = int(torch.cuda.current_stream(self.device).cuda_stream)
            step = self._reduce.get(sh)
            if step is None:
                step = self._reduce[sh] = self.ctx.reduce_step(self.out, self.world, self.res,
                                                                stream=sh)
            r = step()
            self.seconds += time.perf_counter() - t0
            self.calls += 1
            return r
        if self.on_device:
            dist.all_gather_into_tensor(self.out, best16.reshape(1, 2), group=self.group)
            self.host.copy_(self.out, non_blocking=True)
            self.done.record()
            self.done.synchronize()
        else:
            self.rec.copy_(best16)   # (synchronous: d_best to the CPU record)
            dist.all_gather_into_tensor(self.out, self.rec.reshape(1, 2), group=self.group)
        h = self.host
        r = reduce_best(h[:, 0].numpy(), h.view(torch.int64)[:, 1].numpy())
        self.seconds += time.perf_counter() - t0
        self.calls += 1
        return r


def rccl_path():
    """The librccl this process's torch uses (so libmaxcover binds the same RCCL), or None."""
    import os
    import torch

    p = os.path.join(os.path.dirname(os.path.abspath(torch.__file__)), "lib", "librccl.so")
    return p if os.path.exists(p) else None


class RcclExchange:
    """The multi-GPU poll's exchange inside libmaxcover (mac_poll_exchange): its own RCCL
    communicator over the group's ranks (the id made by rank 0 and broadcast once), then per poll
    ONE C call that enqueues the all-gather of the rank's 16-B d_best on the poll's stream (RCCL over
    xGMI, no cross-stream event as torch's collectives need), the one-wave device argmin into a
    persistent 16-B buffer and its mapped host slot, and reads the slot. ``seconds`` / ``calls``:
    host time spent here per poll. Needs a GPU backend (the ranks' devices)."""

    def __init__(self, ctx, device, group=None):
        import time
        import torch
        import torch.distributed as dist

        t0 = time.perf_counter()
        self.ctx = ctx
        self.group = group
        self.device = torch.device(device)
        self.rank, self.world = _lib_comm(ctx, device, group)
        self.res = torch.empty(2, dtype=torch.float64, device=self.device)
        self._steps = {}
        self.init_s = time.perf_counter() - t0
        self.seconds = 0.0
        self.calls = 0

    def step_for(self, best16, stream=None):
        """The bound exchange of best16 on ``stream`` (a raw handle; None: torch's current stream):
        a zero-argument callable returning the node's (objective, index)."""
        import torch

        sh = int(torch.cuda.current_stream(self.device).cuda_stream) if stream is None else int(stream)
        key = (int(best16.data_ptr()), sh)
        st = self._steps.get(key)
        if st is None:
            st = self._steps[key] = self.ctx.exchange_step(best16, self.res, stream=sh)
        return st

    def __call__(self, best16):
        import time

        t0 = time.perf_counter()
        r = self.step_for(best16)()
        self.seconds += time.perf_counter() - t0
        self.calls += 1
        return r


def _lib_comm(ctx, device, group=None):
    """libmaxcover's own communicator on ctx (mac_comm_init over the group's ranks, the id made
    by rank 0 and broadcast once); returns (rank, world)."""
    import torch
    import torch.distributed as dist

    check_one_runtime()
    rank, world = dist.get_rank(group), dist.get_world_size(group)
    path = rccl_path()
    uid = torch.zeros(128, dtype=torch.uint8, device=torch.device(device))
    if rank == 0:
        uid.copy_(torch.tensor(list(ctx.comm_unique_id(path)), dtype=torch.uint8))
    dist.broadcast(uid, 0, group=group)
    ctx.comm_init(bytes(uid.cpu().tolist()), rank, world, path)
    return rank, world


class RcclShardGather:
    """The sharded MADS loop's per-iteration exchange inside libmaxcover: the stepper's polls write
    their shard best into a persistent 16-B device buffer (mac_mads_best_buffer, bound by
    ``mads_loop``), and one C call (mac_poll_exchange) all-gathers every rank's buffer over the
    context's RCCL communicator, reduces it on the device and reads the result from its mapped
    slot. ``seconds`` / ``calls`` as DeviceGather's."""

    def __init__(self, ctx, device, group=None):
        import torch

        self.device = torch.device(device)
        self.rank, self.world = _lib_comm(ctx, device, group)
        self.ctx = ctx
        self.best = torch.zeros(2, dtype=torch.float64, device=self.device)
        self.res = torch.empty(2, dtype=torch.float64, device=self.device)
        self._step = None
        self.seconds = 0.0
        self.calls = 0

    def bind(self, stepper) -> None:
        import torch
        torch.cuda.current_stream(self.device).synchronize()   # (the zero-fill lands first)
        stepper.best_buffer(self.best)
        self._step = self.ctx.exchange_step(self.best, self.res, stream=0)

    def __call__(self, obj, idx):
        import time

        t0 = time.perf_counter()
        r = self._step()
        self.seconds += time.perf_counter() - t0
        self.calls += 1
        return r


class RcclSpecGather:
    """SpecGather's exchange inside libmaxcover (mac_exchange_records): every rank's {done,
    objective, index, feasible} 32-B record through the context's RCCL communicator in one C call
    (upload, all-gather, download, one synchronisation on a private stream)."""

    def __init__(self, ctx, device, group=None):
        import torch

        self.rank, self.world = _lib_comm(ctx, device, group)
        self.ctx = ctx
        self.rec = np.zeros(4, dtype=np.float64)
        self.out = np.zeros((self.world, 4), dtype=np.float64)
        self.stream = torch.cuda.Stream(torch.device(device))

    def __call__(self, done, obj, idx, feasible=0):
        self.rec[0] = 1.0 if done else 0.0
        self.rec[1] = float(obj)
        self.rec.view(np.int64)[2] = int(idx)
        self.rec.view(np.int64)[3] = int(feasible)
        self.ctx.exchange_records(self.rec, self.out, stream=self.stream.cuda_stream)
        hi = self.out.view(np.int64)
        return [(bool(self.out[j, 0] != 0.0), float(self.out[j, 1]), int(hi[j, 2]), int(hi[j, 3]))
                for j in range(self.world)]


class DeviceGather:
    """The per-iteration exchange of the sharded MADS loop without per-iteration allocations:
    on a GPU backend (RCCL) the stepper's polls write their 16-B shard best straight into a
    persistent device buffer (mac_mads_best_buffer, bound by ``mads_loop``) that the all-gather
    reads, and one pinned host read of the world x 16 B result follows; on gloo (CPU rehearsal)
    the host (obj, idx) goes into a persistent CPU record. ``seconds`` / ``calls``: time spent
    here (the loop's host overhead beside the stepper's own, mac_mads_stats)."""

    def __init__(self, device="cpu", group=None):
        import torch
        import torch.distributed as dist

        self.group = group
        self.world = dist.get_world_size(group)
        self.device = torch.device(device)
        self.on_device = self.device.type == "cuda"
        if self.on_device:
            check_one_runtime()
        self.best = torch.zeros(2, dtype=torch.float64, device=self.device)
        self.out = torch.empty((self.world, 2), dtype=torch.float64, device=self.device)
        self.host = (torch.empty((self.world, 2), dtype=torch.float64, pin_memory=True)
                     if self.on_device else self.out)
        self.seconds = 0.0
        self.calls = 0

    def bind(self, stepper) -> None:
        if self.on_device:
            import torch
            # the zero-fill of self.best (torch's current stream) lands before the stepper's
            # own writes to it (an empty shard's {+inf, -1} record is written at bind)
            torch.cuda.current_stream(self.device).synchronize()
            stepper.best_buffer(self.best)

    def __call__(self, obj, idx):
        import time
        import torch
        import torch.distributed as dist

        t0 = time.perf_counter()
        if not self.on_device:
            self.best[0] = float(obj)
            self.best.view(torch.int64)[1] = int(idx)
        dist.all_gather_into_tensor(self.out, self.best.reshape(1, 2), group=self.group)
        if self.on_device:
            self.host.copy_(self.out)   # (synchronous: the one host read per iteration)
        h = self.host
        r = reduce_best(h[:, 0].numpy(), h.view(torch.int64)[:, 1].numpy())
        self.seconds += time.perf_counter() - t0
        self.calls += 1
        return r


def broadcast_points(x=None, y=None, w=None, src: int = 0, device="cpu", group=None):
    """The point list (or a batch of appended points, src/CellFunctions.jl:59-79) from rank
    `src`'s host arrays to every rank's `device`: rank `src` uploads once, then ONE broadcast of
    the packed 3 x M float64 tensor (RCCL over xGMI for GPU tensors, gloo for CPU) instead of a
    host upload per rank — for lists a rank cannot regenerate (the FirePoints table, an external
    feed; config 5's CA fire is regenerated per rank instead). Returns (x, y, w) tensors on
    `device` on every rank; feed them to Context.set_points_device / append_points_device."""
    import torch
    import torch.distributed as dist

    dev = torch.device(device)
    if dev.type == "cuda":
        check_one_runtime()
    rank = dist.get_rank(group)
    n = torch.zeros(1, dtype=torch.int64, device=dev)
    if rank == src:
        n[0] = int(np.asarray(x).size)
    dist.broadcast(n, src, group=group)
    M = int(n.item())
    if rank == src:
        buf = torch.from_numpy(np.stack([np.asarray(x, dtype=np.float64).ravel(),
                                         np.asarray(y, dtype=np.float64).ravel(),
                                         np.asarray(w, dtype=np.float64).ravel()])).to(dev)
    else:
        buf = torch.empty((3, M), dtype=torch.float64, device=dev)
    if M:
        dist.broadcast(buf, src, group=group)
    return buf[0].contiguous(), buf[1].contiguous(), buf[2].contiguous()


def pack_best(obj: float, idx: int, device="cpu"):
    """Host-side constructor of the 16-byte record (for tests and CPU ranks)."""
    import torch

    t = torch.empty(2, dtype=torch.float64, device=device)
    t[0] = float(obj)
    t.view(torch.int64)[1] = int(idx)
    return t


def make_gather(device="cpu", group=None):
    """(obj, idx) -> the lexicographic minimum over all ranks' (obj, idx): one 16-byte all_gather
    per call into persistent buffers (DeviceGather: straight from the stepper's device buffer
    for a GPU device, a CPU record for gloo). Identity for a single process."""
    import torch.distributed as dist

    if not (dist.is_available() and dist.is_initialized()) or dist.get_world_size(group) == 1:
        return lambda obj, idx: (obj, idx)
    return DeviceGather(device, group)


class SpecGather:
    """The speculative loop's exchange: every rank's (done, best objective, best index, feasible
    candidates of its poll) in rank order — one all-gather of a 32-B record per rank (RCCL on a GPU
    device, gloo on CPU) and one host read."""

    def __init__(self, device="cpu", group=None):
        import torch
        import torch.distributed as dist

        self.group = group
        self.world = dist.get_world_size(group)
        self.rank = dist.get_rank(group)
        self.device = torch.device(device)
        self.on_device = self.device.type == "cuda"
        if self.on_device:
            check_one_runtime()
        pin = self.on_device
        self.stage = torch.zeros(4, dtype=torch.float64, pin_memory=pin)
        self.rec = torch.zeros(4, dtype=torch.float64, device=self.device)
        self.out = torch.empty((self.world, 4), dtype=torch.float64, device=self.device)
        self.host = (torch.empty((self.world, 4), dtype=torch.float64, pin_memory=True)
                     if self.on_device else self.out)

    def __call__(self, done, obj, idx, feasible=0):
        import torch
        import torch.distributed as dist

        self.stage[0] = 1.0 if done else 0.0
        self.stage[1] = float(obj)
        self.stage.view(torch.int64)[2] = int(idx)
        self.stage.view(torch.int64)[3] = int(feasible)
        self.rec.copy_(self.stage)
        dist.all_gather_into_tensor(self.out, self.rec.reshape(1, 4), group=self.group)
        if self.on_device:
            self.host.copy_(self.out)
        h = self.host
        hi = h.view(torch.int64)
        return [(bool(h[j, 0].item() != 0.0), float(h[j, 1].item()), int(hi[j, 2].item()),
                 int(hi[j, 3].item())) for j in range(self.world)]


def mads_loop_speculative(stepper, gather=None):
    """The multi-GPU MADS loop by speculation over failure branches (mac_mads_poll_ahead /
    mac_mads_advance, include/maxcover.h): rank j evaluates the whole poll that follows j
    consecutive failures of the current iteration (rank 0: the real poll), one exchange gathers
    all P results, and every rank applies them in order up to the first success — a run of
    failures advances up to P iterations per round, a success one. The iterates are the
    sequential loop's (src/TDM_STATIC_opt.jl:162). ``gather``: a SpecGather (None: one rank).
    Returns stepper.result() with ``rounds`` (exchanges) added to the statistics."""
    rank = gather.rank if gather is not None else 0
    world = gather.world if gather is not None else 1
    rounds = 0
    useful = 0   # the applied polls' feasible candidates (the sequential loop's evaluations)
    while True:
        mine = stepper.poll_ahead(rank)
        recs = gather(*mine) if gather is not None else [mine]
        rounds += 1
        finished = False
        for j in range(world):
            done, obj, idx, feas = recs[j]
            if done:
                finished = True
                break
            useful += feas
            if stepper.advance(obj, idx):
                break
        if finished:
            break
    x, st = stepper.result()
    st = dict(st)
    st["rounds"] = rounds
    # the stepper's own counter holds every poll this rank ran ahead, applied or not; the loop's
    # evaluations are the applied polls' (gathered from whichever rank ran them)
    st["speculative_feasible_evaluations"] = st.get("feasible_evaluations", useful)
    st["feasible_evaluations"] = useful
    st["useful_feasible_evaluations"] = useful
    return x, st


def mads_loop(stepper, gather=None):
    """The sharded MADS loop's host side (mac_mads_poll / mac_mads_update, include/maxcover.h):
    per iteration the stepper polls its shard, ``gather`` combines the ranks' local bests and
    every rank applies the same global best. Returns stepper.result()."""
    if gather is not None and hasattr(gather, "bind"):
        gather.bind(stepper)
    while True:
        done, obj, idx = stepper.poll()
        if done:
            break
        if gather is not None:
            obj, idx = gather(obj, idx)
        stepper.update(obj, idx)
    return stepper.result()
