"""Benchmark: MADS objective evaluations per second on MI355X (BASELINE.json metric).

One step = one complete MADS poll over a synthetic fire grid: K = 6N+1 candidates (incumbent +
2n LTMADS directions, n = 3N) evaluated by libmaxcover, objective + argmin on the device, and
— for N GPUs > 1 — the 16-byte-per-rank all-gather of the local best (RCCL over xGMI). Each
rank holds a full replica of the point list in HBM; inputs are resident before timing starts.

Multi-GPU (`--scaling`):
  weak (default)  every rank evaluates a complete K-candidate poll set of its own (independent
                  LTMADS bases around the same incumbent, rank 0's being the single-GPU poll), so
                  one step polls P*K candidates and the all-gather picks the best of all of
                  them: per-GPU work fixed as P grows;
  strong          the single K-candidate poll is split into P contiguous candidate shards.

Default workload: BASELINE config 4 (512 UAVs, 4096 x 4096 = 16.8M-cell grid, K = 3073, fp64),
the configuration the north-star targets are quoted on and the one the 1/2/4/8-GPU scaling
run uses. `--config 2|3` selects the other synthetic configs.

Prints ONE JSON line on rank 0 (contract in the task statement), with `roofline` for the
dominant kernel (coverage walk) measured with HIP events on its own stream over the timed
region, and `cpu_baseline` = the oracle's C restatement of the reference loop (rank 0, N=1).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--config 4] [--algo auto]
"""
from __future__ import annotations

import argparse
import json
import os
import platform
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

import __graft_entry__ as ge  # noqa: E402

METRIC = "MADS objective evals/sec (N UAVs × M fire cells), 1/2/4/8 MI355X"
HBM_PEAK_GBS = 8000.0      # MI355X_MICROARCH.md: 8.0 TB/s HBM3E (spec)


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def cpu_model() -> str:
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return platform.processor() or "unknown"


def cpu_baseline(x, y, w, cands, seconds_target: float, threads: int):
    """The oracle's C restatement of calculateArea (pointer-per-entry records, same loop and
    break, -O2 no FMA) on `threads` host threads, one candidate per thread, over a bounded
    sample of the same poll. Returns (evals/s, sample description, threads)."""
    orc = ge.load_oracle()
    rec = np.stack([x, y, w, w, np.zeros_like(x)], axis=1)
    pl = orc.PointerList(rec)
    del rec
    # calibrate on one candidate over a slice of the list, then size the sample
    t0 = time.perf_counter()
    sub = orc.PointerList(np.stack([x[:200000], y[:200000], w[:200000], w[:200000],
                                    np.zeros(200000)], axis=1))
    sub.area_batch(cands[:1], 1)
    per_eval = (time.perf_counter() - t0) * (x.size / 200000.0)
    sub.close()
    n = max(1, min(cands.shape[0], int(round(seconds_target / max(per_eval, 1e-9))) * threads))
    n = max(threads if n >= threads else n, 1)
    n = (n // threads) * threads if n >= threads else n
    t0 = time.perf_counter()
    pl.area_batch(cands[:n], threads)
    dt = time.perf_counter() - t0
    pl.close()
    desc = (f"{n} of the poll's {cands.shape[0]} candidates x all {x.size} entries, "
            f"{threads} OpenMP threads (one candidate per thread, as DirectSearch SetMaxEvals), "
            f"{dt:.1f} s, host CPU {cpu_model()}")
    return n / dt, desc


def bench_config5(args, pkg, dev_index):
    """Config 5: src/FullSimulation.jl's optimisation loop with the CA fire (src/DynamicArea.jl)
    streamed into the device list. One step = one MPC timestep: fire step + append/re-index,
    rmvCoveredPOI by the previous circles, and a native MADS run (mac_mads_run, N_iter
    iterations of a complete 2n-candidate poll). value = candidates evaluated / second over the
    timed MPC steps, everything inside the step included."""
    import torch
    wl = pkg.workloads
    cfg = wl.CONFIGS[5]
    rng = wl.SplitMix64(args.seed)
    fire_kw, x0 = wl.config5_setup(rng, cfg["G"], cfg["N"], cfg["ignition"])
    ctx = pkg.Context(dev_index)
    t_set = time.perf_counter()
    D = pkg.DynamicArea.DynamicArea(**fire_kw, seed=args.seed, device=dev_index)
    sim = pkg.FullSimulation.Simulation(ctx, x0, fire=D, N_iter=args.mads_iters, seed=args.seed)
    t_set = time.perf_counter() - t_set
    for _ in range(args.warmup):
        sim.step()
    torch.cuda.synchronize()
    ctx.profile(True)
    ctx.profile_read(reset=True)
    recs = []
    t0 = time.perf_counter()
    for _ in range(args.steps):
        recs.append(sim.step())
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    k_ms, k_launches, k_cands, k_walk = ctx.profile_read(reset=True)
    ctx.profile(False)
    evals = sum(r["evaluations"] for r in recs)
    M_avg = float(np.mean([r["points"] for r in recs]))
    b_eval = 24 * M_avg + 24 * cfg["N"] + 8
    avg_launch_ms = k_ms / max(k_launches, 1)
    cands_per_launch = k_cands / max(k_launches, 1)
    achieved = b_eval * cands_per_launch / (avg_launch_ms * 1e-3) / 1e9 if k_launches else None
    cpu = None
    if not args.no_cpu:
        x, y, w = ctx.get_points()
        polls = wl.poll_candidates(sim.x_prev, wl.SplitMix64(args.seed + 1))
        threads = int(os.environ.get("OMP_NUM_THREADS", "0")) or os.cpu_count() or 1
        threads = max(1, min(threads, 16))
        try:
            v, desc = cpu_baseline(x, y, w, polls, args.cpu_seconds, threads)
            cpu = {"value": v, "unit": "evals/s", "cores": threads, "kind": "port",
                   "sample": desc + " (the final config-5 point list)"}
        except Exception as e:  # report, never fake
            log("cpu baseline failed:", e)
    out = {
        "metric": METRIC, "value": evals / elapsed, "unit": "evals/s", "n_gpus": 1,
        "steps": args.steps, "warmup": args.warmup, "ms_per_step": elapsed / args.steps * 1e3,
        "higher_is_better": True, "scaling": "strong", "vs_baseline": None, "dtype": "f64",
        "data": "synthetic (seeded CA fire)",
        "config": {
            "workload": f"config 5: {cfg['name']}", "uavs": cfg["N"],
            "fire_grid": f"{cfg['G']}x{cfg['G']} cells @ 5 m, ignition {cfg['ignition']}^2 cells",
            "step": "one MPC timestep: fire CA step + append + rmvCoveredPOI + native MADS run",
            "mads_iterations_per_step": args.mads_iters,
            "candidates_per_poll": 6 * cfg["N"],
            "points_mean": M_avg,
            "evaluations": evals,
            "time_split_s": {k: float(np.sum([r[k] for r in recs]))
                             for k in ("fire_s", "remove_s", "mads_s")},
            "parallelism": "1 GPU",
        },
        "roofline": {
            "bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
            "frac": (achieved / HBM_PEAK_GBS) if achieved else None, "traffic": None,
            "kernel": f"coverage_{k_walk}_kernel", "bytes_per_eval": b_eval,
            "evals_per_launch": cands_per_launch, "avg_launch_ms": avg_launch_ms,
            "note": "SURVEY 8(d) algorithmic bytes at the mean list length; frac > 1 by design",
        },
        "cpu_baseline": cpu,
        "setup_s": t_set,
    }
    print(json.dumps(out), flush=True)
    D.close()
    ctx.close()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--config", type=int, default=4, choices=(2, 3, 4, 5),
                    help="4 (default): one MADS poll per step; 5: one end-to-end MPC step "
                         "(CA fire stream + rmvCoveredPOI + a MADS run) per step")
    ap.add_argument("--mads-iters", type=int, default=100, help="config 5: N_iter per MPC step")
    ap.add_argument("--algo", default="auto", choices=("auto", "tiled", "scan", "poll"))
    ap.add_argument("--polls", type=int, default=4, help="distinct poll sets cycled over steps")
    ap.add_argument("--tile-points", type=int, default=None,
                    help="points per spatial tile of the index (library default when omitted)")
    ap.add_argument("--cpu-seconds", type=float, default=15.0)
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--seed", type=int, default=20250216)
    ap.add_argument("--scaling", default="weak", choices=("weak", "strong"),
                    help="N>1: weak = one full poll set per GPU (P*K candidates per step); "
                         "strong = the single poll split over the GPUs")
    ap.add_argument("--dist-backend", default="nccl", choices=("nccl", "gloo"),
                    help="nccl (= RCCL on ROCm) for the real multi-GPU run; gloo only to rehearse "
                         "N>1 with several ranks sharing one GPU (MAXCOVER_BENCH_DEVICE)")
    args = ap.parse_args()

    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    distributed = world > 1
    # one process per GPU; MAXCOVER_BENCH_DEVICE pins every rank to one device (rehearsal only)
    dev_index = int(os.environ.get("MAXCOVER_BENCH_DEVICE", local))
    if distributed:
        torch.cuda.set_device(dev_index)
        if args.dist_backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", dev_index))
        else:
            dist.init_process_group("gloo")
    dev = torch.device("cuda", dev_index)
    torch.cuda.set_device(dev)
    coll_dev = dev if args.dist_backend == "nccl" else torch.device("cpu")

    pkg = ge.load_package()
    from importlib import import_module
    pdist = import_module(pkg.__name__ + ".dist")
    wl = pkg.workloads
    if args.config == 5:
        if world != 1:
            raise SystemExit("config 5 runs on one GPU (the native MADS loop is not sharded yet)")
        return bench_config5(args, pkg, dev_index)

    cfg = wl.CONFIGS[args.config]
    G, N = cfg["G"], cfg["N"]
    rng = wl.SplitMix64(args.seed)
    x, y, w = wl.grid_points(G)
    x0 = wl.uniform_disks(N, G, rng)
    if cfg["K"] == 1:
        polls = [x0[None, :].copy() for _ in range(args.polls)]
        for p in polls[1:]:
            p[0, : 2 * N] += rng.integers(-2, 2, 2 * N)
    else:
        # weak scaling: rank r > 0 draws its own poll sets (rank 0's are the single-GPU polls)
        prng = rng if (rank == 0 or args.scaling == "strong") else \
            wl.SplitMix64(args.seed ^ (0x9E3779B97F4A7C15 * rank & 0xFFFFFFFFFFFFFFFF))
        polls = [wl.poll_candidates(x0, prng) for _ in range(args.polls)]
    K = polls[0].shape[0]
    r_max = np.full(N, 30.0 * np.tan(100 / 180 * np.pi / 2))
    M = x.size
    if args.scaling == "weak":
        lo, hi = 0, K                      # a whole poll set per rank
        idx_base = rank * K                # global candidate index = rank * K + k
        K_step = K * world                 # candidates evaluated per step, all ranks
    else:
        lo, hi = pdist.shard_range(K, rank, world)
        idx_base = lo
        K_step = K
    Kl = hi - lo

    ctx = pkg.Context(dev_index, algo=args.algo, tile_points=args.tile_points)
    t_set = time.perf_counter()
    ctx.set_points(x, y, w)   # once per MPC step: upload + tile index (not part of an eval)
    t_set = time.perf_counter() - t_set
    d_polls = [torch.from_numpy(np.ascontiguousarray(p[lo:hi])).to(dev) for p in polls]
    d_rmax = torch.from_numpy(r_max).to(dev)
    d_best = torch.empty(2, dtype=torch.float64, device=dev)
    stream = torch.cuda.Stream(dev)
    s_handle = stream.cuda_stream

    # one bound poll per candidate set: the ctypes arguments are built once (Context.poll_step)
    steps = [ctx.poll_step(d, 3 * N, Kl, d_rmax, d_best, idx_base=idx_base, stream=s_handle)
             for d in d_polls]

    def step(i):
        """One MADS poll. It ends with the best (objective, index) on the host, because the
        next poll's candidates depend on it: polls never overlap."""
        if distributed:
            d = d_polls[i % len(d_polls)]
            ctx.poll_best_dev(d, 3 * N, Kl, d_rmax, d_best, idx_base=idx_base, stream=s_handle)
            with torch.cuda.stream(stream):
                return pdist.gather_best(d_best if coll_dev.type == "cuda" else d_best.cpu())
        return steps[i % len(steps)]()   # poll + the 16-B result from pinned host memory

    for i in range(args.warmup):
        step(i)
    torch.cuda.synchronize(dev)

    # correctness guard on the timed workload: scan kernel vs tiled on poll 0's first entries
    check = None
    if rank == 0:
        probe = polls[0][: min(8, K)]
        ctx.set_algo("scan")
        a_scan = ctx.area_batch(probe)
        ctx.set_algo(args.algo)
        a_main = ctx.area_batch(probe)
        check = bool(np.array_equal(a_scan, a_main))
        if not check:
            log("WARNING: scan/tiled disagree on the probe candidates", a_scan, a_main)

    ctx.profile(True)
    ctx.profile_read(reset=True)
    if distributed:
        dist.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    result = None
    for i in range(args.steps):
        result = step(args.warmup + i)
    if distributed:
        dist.barrier()
    torch.cuda.synchronize(dev)
    elapsed = time.perf_counter() - t0
    k_ms, k_launches, k_cands, k_walk = ctx.profile_read(reset=True)
    ctx.profile(False)
    if distributed:
        t = torch.tensor([elapsed], dtype=torch.float64, device=coll_dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    if result is None:
        b = d_best.cpu()
        result = (float(b[0]), int(b.view(torch.int64)[1]))

    total_evals = K_step * args.steps
    value = total_evals / elapsed
    ms_per_step = elapsed / args.steps * 1e3

    # roofline of the dominant kernel (this rank's launches; SURVEY §8(d) algorithmic bytes)
    s = 8  # fp64
    b_eval = 3 * M * s + 3 * N * s + 8
    avg_launch_ms = k_ms / max(k_launches, 1)
    cands_per_launch = k_cands / max(k_launches, 1)
    achieved = b_eval * cands_per_launch / (avg_launch_ms * 1e-3) / 1e9 if k_launches else None
    traffic = None
    pmc_path = os.path.join(ROOT, "profiles", f"pmc_traffic_config{args.config}.json")
    if world == 1 and args.algo == "auto" and os.path.exists(pmc_path):  # the profiled launch
        try:
            with open(pmc_path) as f:
                traffic = json.load(f).get("hbm_bytes_per_launch")
        except (OSError, ValueError):
            traffic = None

    out = None
    if rank == 0:
        cpu = None
        if not args.no_cpu and world == 1:
            threads = int(os.environ.get("OMP_NUM_THREADS", "0")) or os.cpu_count() or 1
            threads = max(1, min(threads, 16))
            try:
                v, desc = cpu_baseline(x, y, w, polls[0], args.cpu_seconds, threads)
                cpu = {"value": v, "unit": "evals/s", "cores": threads, "kind": "port",
                       "sample": desc}
            except Exception as e:  # report, never fake
                log("cpu baseline failed:", e)
        out = {
            "metric": METRIC,
            "value": value,
            "unit": "evals/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": ms_per_step,
            "higher_is_better": True,
            "scaling": args.scaling,
            "vs_baseline": None,
            "dtype": "f64",
            "data": "synthetic",
            "config": {
                "workload": f"config {args.config}: {cfg['name']}",
                "uavs": N, "cells": M, "grid": f"{G}x{G} @ 5 m", "candidates_per_poll": K,
                "candidates_per_step": K_step,
                "poll": "incumbent + 2n LTMADS directions (n=3N), l=2, delta=1",
                "disks": "integer centres uniform over the domain, R=36",
                "parallelism": (f"{world} GPU(s), one full poll set each, 16-B argmin all-gather"
                                if args.scaling == "weak" else
                                f"one poll's candidates sharded over {world} GPU(s), "
                                f"16-B argmin all-gather"),
                "algo": args.algo,
            },
            "roofline": {
                "bound": "hbm",
                "achieved": achieved,
                "peak": HBM_PEAK_GBS,
                "unit": "GB/s",
                "frac": (achieved / HBM_PEAK_GBS) if achieved else None,
                "traffic": traffic,
                "kernel": f"coverage_{k_walk}_kernel",
                "bytes_per_eval": b_eval,
                "evals_per_launch": cands_per_launch,
                "avg_launch_ms": avg_launch_ms,
                "traffic_frac": (traffic / (avg_launch_ms * 1e-3) / 1e9 / HBM_PEAK_GBS
                                 if traffic and avg_launch_ms else None),
                "timing": "in-kernel workgroup stamps (s_memrealtime) over the timed steps",
                "note": "achieved = SURVEY 8(d) algorithmic bytes (24 B x M entries + disks) per "
                        "eval x evals per launch / launch time; the walks read only the "
                        "entries near the disks, so frac > 1 is by design (see DESIGN.md). "
                        "traffic_frac = the kernel's measured HBM bytes per launch (PMC, "
                        "profiles/pmc_traffic_config4.json) / launch time / peak",
            },
            "cpu_baseline": cpu,
            "best": {"objective": result[0], "index": result[1]},
            "check_scan_vs_main": check,
            "setup_s": t_set,
        }
        print(json.dumps(out), flush=True)
    if distributed:
        dist.barrier()
        dist.destroy_process_group()
    ctx.close()


if __name__ == "__main__":
    main()
