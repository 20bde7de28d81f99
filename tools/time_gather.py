"""Time the multi-GPU exchanges over RCCL on one GPU (world 1): dist.PollGather (the strong-split
poll's 16-B all-gather + pinned host read) and dist.DeviceGather (the sharded MADS loop's), each
after a real device poll on torch's current stream, plus the bare collective. World 1 measures
the fixed per-call cost (launch, RCCL's proxy path, the pinned read, event synchronisation); the
xGMI hop of a real world-P ring adds ~P x 2-3 us.

    python tools/time_gather.py [--calls 2000]
"""
import argparse
import json
import os
import socket
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import __graft_entry__ as ge  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--calls", type=int, default=2000)
    args = ap.parse_args()
    import torch
    import torch.distributed as dist

    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK="0", WORLD_SIZE="1")
    torch.cuda.set_device(0)
    dist.init_process_group("nccl", rank=0, world_size=1)
    pkg = ge.load_package()
    pd = __import__(pkg.__name__ + ".dist", fromlist=["PollGather"])
    dev = torch.device("cuda", 0)
    out = {"world": 1, "backend": dist.get_backend(), "calls": args.calls}

    best = torch.tensor([1.0, 0.0], dtype=torch.float64, device=dev)
    # bare collective + event sync
    o = torch.empty((1, 2), dtype=torch.float64, device=dev)
    for _ in range(50):
        dist.all_gather_into_tensor(o, best.reshape(1, 2))
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.calls):
        dist.all_gather_into_tensor(o, best.reshape(1, 2))
        torch.cuda.current_stream().synchronize()
    out["all_gather_sync_us"] = (time.perf_counter() - t0) / args.calls * 1e6

    pg = pd.PollGather(dev)
    for _ in range(50):
        pg(best)
    pg.seconds, pg.calls = 0.0, 0
    t0 = time.perf_counter()
    for _ in range(args.calls):
        pg(best)
    out["poll_gather_us"] = (time.perf_counter() - t0) / args.calls * 1e6
    out["poll_gather_inner_us"] = pg.seconds / max(pg.calls, 1) * 1e6

    # a real poll then the exchange (the strong step's per-poll cost beyond the chain)
    x, y, w, C, rmax = pkg.workloads.make_config(4)
    ctx = pkg.Context(0)
    ctx.set_points(x, y, w)
    tC = torch.from_numpy(np.ascontiguousarray(C)).to(dev)
    tR = torch.from_numpy(rmax).to(dev)
    K, n3 = C.shape
    d_best = torch.empty(2, dtype=torch.float64, device=dev)
    st = torch.cuda.current_stream(dev).cuda_stream
    for _ in range(20):
        ctx.poll_best_dev(tC, n3, K, tR, d_best, 1e5, stream=st)
        pg(d_best)
    n = min(args.calls, 500)
    t0 = time.perf_counter()
    for _ in range(n):
        ctx.poll_best_dev(tC, n3, K, tR, d_best, 1e5, stream=st)
        pg(d_best)
    out["poll_plus_gather_us"] = (time.perf_counter() - t0) / n * 1e6
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(n):
        ctx.poll_best_dev(tC, n3, K, tR, d_best, 1e5, stream=st)
        torch.cuda.current_stream(dev).synchronize()
    out["poll_plus_sync_us"] = (time.perf_counter() - t0) / n * 1e6

    # the device-reduced exchange: all-gather, one-wave argmin, mapped-slot read (no copy/sync)
    pgd = pd.PollGather(dev, ctx=ctx)
    for _ in range(50):
        pgd(best)
    pgd.seconds, pgd.calls = 0.0, 0
    t0 = time.perf_counter()
    for _ in range(args.calls):
        pgd(best)
    out["poll_gather_device_reduce_us"] = (time.perf_counter() - t0) / args.calls * 1e6
    for _ in range(20):
        ctx.poll_best_dev(tC, n3, K, tR, d_best, 1e5, stream=st)
        pgd(d_best)
    t0 = time.perf_counter()
    for _ in range(n):
        ctx.poll_best_dev(tC, n3, K, tR, d_best, 1e5, stream=st)
        pgd(d_best)
    out["poll_plus_device_gather_us"] = (time.perf_counter() - t0) / n * 1e6
    # the poll alone through its own mapped slot (the 1-GPU step)
    step1 = ctx.poll_step(tC, n3, K, tR, d_best, 1e5, stream=st)
    for _ in range(20):
        step1()
    t0 = time.perf_counter()
    for _ in range(n):
        step1()
    out["poll_step_us"] = (time.perf_counter() - t0) / n * 1e6

    # libmaxcover's own communicator: all-gather on the poll's stream + device argmin + slot, one C call
    with pkg.Context(0) as cx:
        cx.set_points(x, y, w)
        rx = pd.RcclExchange(cx, dev)
        xs = rx.step_for(best, st)
        for _ in range(50):
            xs()
        t0 = time.perf_counter()
        for _ in range(args.calls):
            xs()
        out["rccl_exchange_us"] = (time.perf_counter() - t0) / args.calls * 1e6
        pstep = cx.poll_step(tC, n3, K, tR, d_best, 1e5, stream=st, fetch=False)
        xs2 = rx.step_for(d_best, st)
        for _ in range(20):
            pstep()
            xs2()
        t0 = time.perf_counter()
        for _ in range(n):
            pstep()
            xs2()
        out["poll_plus_rccl_exchange_us"] = (time.perf_counter() - t0) / n * 1e6
        out["rccl_exchange_init_s"] = rx.init_s

    dg = pd.DeviceGather(dev)
    for _ in range(50):
        dg(1.0, 0)
    t0 = time.perf_counter()
    for _ in range(args.calls):
        dg(1.0, 0)
    out["device_gather_us"] = (time.perf_counter() - t0) / args.calls * 1e6
    ctx.close()
    dist.destroy_process_group()
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
