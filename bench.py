"""Benchmark: MADS objective evaluations per second on MI355X (BASELINE.json metric).

One step = one complete MADS poll over a synthetic fire grid: K = 6N+1 candidates (incumbent +
2n LTMADS directions, n = 3N) evaluated by libmaxcover, objective + argmin on the device, and
— for N GPUs > 1 — the 16-byte-per-rank all-gather of the local best (RCCL over xGMI). Each
rank holds a full replica of the point list in HBM; inputs are resident before timing starts.

Multi-GPU (`--scaling`):
  strong (default) the single K-candidate poll is split into P contiguous candidate shards (the
                  north star's split); value = K candidates per step / the max-over-ranks time;
  weak            every rank evaluates a complete K-candidate poll set of its own (independent
                  LTMADS bases around the same incumbent, rank 0's being the single-GPU poll), so
                  one step polls P*K candidates and the all-gather picks the best of all of
                  them: per-GPU work fixed as P grows (a secondary, labelled line).
`--shard-of P` times rank 0's shard of a P-way split alone on one GPU (no collective): the
per-rank chain floor that bounds strong scaling.

Default workload: BASELINE config 4 (512 UAVs, 4096 x 4096 = 16.8M-cell grid, K = 3073, fp64),
the configuration the north-star targets are quoted on and the one the 1/2/4/8-GPU scaling
run uses. `--config 2|3` selects the other synthetic configs.

Prints ONE JSON line on rank 0 (contract in the task statement), with `roofline` for the poll
chain and its dominant kernel, timed by in-kernel workgroup stamps (s_memrealtime: first
workgroup start to last workgroup end of every launch, over the timed steps), and
`cpu_baseline` = the oracle's C restatement of the reference loop (rank 0, N=1).

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


def floor_bytes(x, y, w, cands, G):
    """Algorithmic bytes of one poll for an exact culling evaluation: the 3N x K
    candidate matrix read once (8 B per value), every entry inside the union over disks i of the
    poll-wide box of disk i's footprints [min(x-r), max(x+r)] x [min(y-r), max(y+r)] read once
    (16 B of coordinates, + 8 B of weight unless every weight is equal), and the 16-B result.
    Entries are counted on the G x G createPOI lattice (pitch 5, (i - 1/2) * 5)."""
    K, n3 = cands.shape
    N = n3 // 3
    cx, cy, r = cands[:, :N], cands[:, N:2 * N], cands[:, 2 * N:]
    good = r > 0
    lo_x = np.where(good, cx - r, np.inf).min(axis=0)
    hi_x = np.where(good, cx + r, -np.inf).max(axis=0)
    lo_y = np.where(good, cy - r, np.inf).min(axis=0)
    hi_y = np.where(good, cy + r, -np.inf).max(axis=0)
    mask = np.zeros((G, G), dtype=bool)
    for i in range(N):
        if not (lo_x[i] <= hi_x[i]):
            continue
        i0 = max(1, int(np.ceil(lo_x[i] / 5.0 + 0.5)))
        i1 = min(G, int(np.floor(hi_x[i] / 5.0 + 0.5)))
        j0 = max(1, int(np.ceil(lo_y[i] / 5.0 + 0.5)))
        j1 = min(G, int(np.floor(hi_y[i] / 5.0 + 0.5)))
        if i0 <= i1 and j0 <= j1:
            mask[i0 - 1:i1, j0 - 1:j1] = True
    E = int(mask.sum())
    per_entry = 16 if np.all(w == w[0]) else 24
    cand_b = 8 * n3 * K
    return {"bytes": cand_b + per_entry * E + 16, "candidate_bytes": cand_b, "entries": E,
            "bytes_per_entry": per_entry}


def floor_bytes_points(x, y, w, cands, cand_bytes):
    """floor_bytes for an arbitrary point list (the config-5 fire stream): every point inside
    some disk's poll-wide footprint box read once (16 B, + 8 B of weight unless all equal), the
    candidate inputs (`cand_bytes`: the generated poll's incumbent and permutations) and the
    16-B result."""
    K, n3 = cands.shape
    N = n3 // 3
    cx, cy, r = cands[:, :N], cands[:, N:2 * N], cands[:, 2 * N:]
    good = r > 0
    lo_x = np.where(good, cx - r, np.inf).min(axis=0)
    hi_x = np.where(good, cx + r, -np.inf).max(axis=0)
    lo_y = np.where(good, cy - r, np.inf).min(axis=0)
    hi_y = np.where(good, cy + r, -np.inf).max(axis=0)
    inside = np.zeros(x.size, dtype=bool)
    for i in range(N):
        if lo_x[i] <= hi_x[i]:
            inside |= (x >= lo_x[i]) & (x <= hi_x[i]) & (y >= lo_y[i]) & (y <= hi_y[i])
    E = int(inside.sum())
    per_entry = 16 if (w.size == 0 or np.all(w == w[0])) else 24
    return {"bytes": cand_bytes + per_entry * E + 16, "candidate_bytes": cand_bytes, "entries": E,
            "bytes_per_entry": per_entry}


def src_hash():
    """sha256 over the library sources (csrc/*.hip, csrc/*.h, include/maxcover.h): stamps the
    PMC traffic files so that a number measured on another build is never attached."""
    import hashlib
    h = hashlib.sha256()
    d = os.path.join(ROOT, "maximumareacoverageoptimization.jl_amd", "csrc")
    for name in sorted(os.listdir(d)):
        if name.endswith((".hip", ".h")):
            with open(os.path.join(d, name), "rb") as f:
                h.update(name.encode() + b"\0" + f.read())
    with open(os.path.join(ROOT, "include", "maxcover.h"), "rb") as f:
        h.update(f.read())
    return h.hexdigest()[:16]


def pmc_traffic(config, disks, world, algo):
    """(HBM bytes per poll chain, source note, {kernel: bytes per launch}) from
    profiles/pmc_traffic_config{config}.json when it was measured on these sources, this workload
    and the default walk; else (None, why, {})."""
    path = os.path.join(ROOT, "profiles", f"pmc_traffic_config{config}.json")
    if world != 1 or algo != "auto" or disks != "uniform":
        return None, "not profiled for this workload", {}
    try:
        with open(path) as f:
            d = json.load(f)
    except (OSError, ValueError):
        return None, "no PMC file", {}
    if d.get("src_sha") != src_hash():
        return None, f"PMC file is from another build (src_sha {d.get('src_sha')})", {}
    per = {}
    for name, v in d.get("kernels", {}).items():
        base = name.split("<")[0]
        if base.startswith("mac::"):
            per[base[5:]] = {"hbm_bytes": v.get("hbm_bytes_per_launch"),
                             "hbm_bytes_raw": v.get("hbm_bytes_per_launch_raw")}
    src = os.path.relpath(path, ROOT) + f" (src_sha {d['src_sha']})"
    if d.get("hbm_bytes_per_poll_raw") is not None:
        src += f"; uncorrected FETCH (lower bound): {d['hbm_bytes_per_poll_raw']:.4g} B per poll"
    return d.get("hbm_bytes_per_poll"), src, per


def kernel_table(kern, pmc_per=None):
    """{kernel: {"avg_us", "launches"[, "hbm_bytes"]}} of the poll chain's launches that ran
    (Context.profile_kernels: in-kernel stamps over the timed steps) and the dominant one (the
    longest average launch)."""
    out = {}
    for name, (ms, n) in kern.items():
        if n:
            out[name] = {"avg_us": ms / n * 1e3, "launches": n}
            if pmc_per and pmc_per.get(name) is not None:
                out[name].update({k: v for k, v in pmc_per[name].items() if v is not None})
    dom = max(out, key=lambda k: out[k]["avg_us"]) if out else None
    return out, dom


def usable_cpus():
    """(threads to use, description): the CPUs this process may run on — its affinity mask,
    capped by a cgroup CPU quota and by OMP_NUM_THREADS (the GPU pool sets it to the CPU share
    of one GPU: the box's os.cpu_count() is the whole machine, shared with other jobs)."""
    total = os.cpu_count() or 1
    try:
        aff = len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        aff = total
    quota = None
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            q, per = f.read().split()[:2]
            if q != "max":
                quota = max(1, int(int(q) // int(per)))
    except (OSError, ValueError):
        quota = None
    omp = int(os.environ.get("OMP_NUM_THREADS", "0") or 0) or None
    n = min(v for v in (aff, quota, omp) if v)
    info = {"host_logical_cpus": total, "affinity_cpus": aff, "cgroup_cpu_quota": quota,
            "omp_num_threads_env": omp}
    return max(1, n), info


def cpu_baseline(x, y, w, cands, seconds_target: float, threads: int):
    """The oracle's C restatement of calculateArea (pointer-per-entry records, same loop and
    break, -O2 no FMA) on `threads` host threads, one candidate per thread, over a bounded
    sample of the same poll. Returns (evals/s, sample description, threads)."""
    orc = ge.load_oracle()
    rec = np.stack([x, y, w, w, np.zeros_like(x)], axis=1)
    pl = orc.PointerList(rec)
    del rec
    # calibrate on one candidate over a slice of the list, then size the sample
    m = max(1, min(200000, x.size))
    sub = orc.PointerList(np.stack([x[:m], y[:m], w[:m], w[:m], np.zeros(m)], axis=1))
    t0 = time.perf_counter()
    sub.area_batch(cands[:1], 1)
    per_eval = (time.perf_counter() - t0) * (x.size / float(m))
    sub.close()
    K = cands.shape[0]
    n = max(1, min(K, int(round(seconds_target / max(per_eval, 1e-9))) * threads))
    n = max(n, min(threads, K))                          # at least one candidate per thread
    n = (n // threads) * threads if n >= threads else n  # whole rounds of the threads
    t0 = time.perf_counter()
    pl.area_batch(cands[:n], threads)
    dt = time.perf_counter() - t0
    pl.close()
    desc = (f"{n} of the poll's {cands.shape[0]} candidates x all {x.size} entries, "
            f"{threads} OpenMP threads (one candidate per thread, as DirectSearch SetMaxEvals), "
            f"{dt:.1f} s, host CPU {cpu_model()}")
    return n / dt, desc


def stamp_setup(ctx, stamp_timed):
    """Before the warmup (so that nothing stands between it and the timed region): the stamp slots
    allocated and zeroed (ctx.profile(True): a device synchronisation, 32 MB of slots, a memset),
    stamping then left on (--stamps timed; the warmup's stamps are reset before the timed steps) or
    off until the stamped pass after the timed region. Ranks sharing one GPU (the gloo rehearsals) ran the
    config-5 loop at 35.6 ms per MPC step with this set-up first done after the timed region, 22.6-24.4
    with it before (same box; cause not identified; single-GPU runs: profiles/r06_stamp_setup_ab.json).
    MAXCOVER_BENCH_NO_STAMP_SETUP=1 skips it (for that A/B)."""
    if stamp_timed or os.environ.get("MAXCOVER_BENCH_NO_STAMP_SETUP") != "1":
        ctx.profile(True)
        ctx.profile_read(reset=True)
        if not stamp_timed:
            ctx.profile(False)


def closure_threads(ctx, cands, sweep, seconds=0.25):
    """Aggregate mac_area_f64 calls/s with T native host threads calling at once (DirectSearch's
    SetMaxEvals threaded poll, src/TDM_STATIC_opt.jl:129: one objective call per trial point per
    thread), through csrc/closure_threads.cpp (Python threads would serialise on the GIL around
    every call). Thread t evaluates candidates t, t + T, ... of the poll; every result is checked
    against the single-threaded area of the same candidate."""
    import ctypes
    path = os.path.join(os.path.dirname(ctx._L._name), "libmaxcover_threads.so")
    if not os.path.exists(path):
        return {"error": "libmaxcover_threads.so not built"}
    H = ctypes.CDLL(path)
    H.mac_closure_threads.restype = ctypes.c_double
    H.mac_closure_threads.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64,
                                      ctypes.c_int64, ctypes.c_void_p, ctypes.c_int32, ctypes.c_double,
                                      ctypes.POINTER(ctypes.c_int64), ctypes.POINTER(ctypes.c_int64),
                                      ctypes.POINTER(ctypes.c_int64)]
    K = min(cands.shape[0], 64)
    C = np.ascontiguousarray(cands[:K])
    want = np.array([ctx.area(np.ascontiguousarray(C[k])) for k in range(K)])
    fn = ctypes.cast(ctx._L.mac_area_f64, ctypes.c_void_p).value
    out = {}
    for T in sweep:
        calls, bad, fail = ctypes.c_int64(), ctypes.c_int64(), ctypes.c_int64()
        dt = H.mac_closure_threads(fn, ctx._h, C.ctypes.data, K, C.shape[1], want.ctypes.data, int(T),
                                   float(seconds), ctypes.byref(calls), ctypes.byref(bad),
                                   ctypes.byref(fail))
        out[str(T)] = {"calls_per_s": calls.value / dt, "calls": calls.value,
                       "mismatches": bad.value, "failures": fail.value}
    base = out[str(sweep[0])]["calls_per_s"]
    for T in sweep:
        out[str(T)]["vs_1_thread"] = out[str(T)]["calls_per_s"] / base if base else None
    return out


def rank_launch_command(n: int, argv, port: int):
    """The command `bench.py --gpus N` runs when no launcher started it: torch.distributed.run
    with N local ranks (one process per GPU, RANK / LOCAL_RANK / WORLD_SIZE in their env) over
    127.0.0.1, each rank running this script with the same arguments."""
    return [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
            "--master-addr", "127.0.0.1", "--master-port", str(port),
            os.path.abspath(__file__), *argv]


def world_plan(gpus: int, env=None) -> str:
    """'run' (this process is a rank, or the only one) or 'launch' (start --gpus ranks first).
    Raises SystemExit (status 2) when a launcher's WORLD_SIZE disagrees with --gpus: a line for
    N GPUs must come from N ranks, never from a silently smaller run."""
    env = os.environ if env is None else env
    if gpus < 1:
        log("bench.py: --gpus must be >= 1")
        raise SystemExit(2)
    ws = env.get("WORLD_SIZE")
    if ws is None:
        return "launch" if gpus > 1 else "run"
    if int(ws) != gpus:
        log(f"bench.py: WORLD_SIZE={ws} from the launcher but --gpus {gpus}: "
            f"refusing to report a {ws}-rank run as {gpus} GPUs")
        raise SystemExit(2)
    return "run"


def launch_ranks(gpus: int, argv) -> int:
    """Start `gpus` ranks of this script (before this process touches any GPU) and return the
    launcher's exit status. Each rank uses its LOCAL_RANK's GPU, so the node must show that
    many devices, unless MAXCOVER_BENCH_DEVICE pins every rank to one device (rehearsals)."""
    import socket
    import subprocess
    import torch   # device_count does not initialise the GPU on this image

    if "MAXCOVER_BENCH_DEVICE" not in os.environ and torch.cuda.device_count() < gpus:
        log(f"bench.py: --gpus {gpus} but {torch.cuda.device_count()} GPU(s) visible")
        return 2
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    cmd = rank_launch_command(gpus, argv, port)
    log("bench.py: launching", " ".join(cmd))
    return subprocess.run(cmd).returncode


def bench_config5(args, pkg, dev_index, rank=0, world=1, coll_dev=None):
    """Config 5: src/FullSimulation.jl's optimisation loop with the CA fire (src/DynamicArea.jl)
    streamed into the device list. One step = one MPC timestep: fire step + append/re-index,
    rmvCoveredPOI by the previous circles, and a native MADS run (mac_mads_run, N_iter
    iterations of a complete 2n-candidate poll). value = candidates evaluated / second over the
    timed MPC steps, everything inside the step included. On P GPUs every rank regenerates the
    deterministic fire stream on its own GPU (no point transfer) and polls its shard of every
    LTMADS poll, one 16-B all-gather per MADS iteration (strong scaling: the same polls)."""
    import torch
    import torch.distributed as dist
    from importlib import import_module
    pdist = import_module(pkg.__name__ + ".dist")
    wl = pkg.workloads
    cfg = wl.CONFIGS[5]
    rng = wl.SplitMix64(args.seed)
    fire_kw, x0 = wl.config5_setup(rng, cfg["G"], cfg["N"], cfg["ignition"])
    ctx = pkg.Context(dev_index, algo=args.algo)
    ctx.set_chain(args.chain)
    t_set = time.perf_counter()
    D = pkg.DynamicArea.DynamicArea(**fire_kw, seed=args.seed, device=dev_index)
    shard = (rank, world) if world > 1 else None
    spec = world > 1 and args.mads_mode == "speculate"
    gather = None
    if world > 1 and coll_dev.type == "cuda" and args.exchange == "rccl":
        # libmaxcover's own communicator: the per-round exchange in one C call
        gather = (pdist.RcclSpecGather(ctx, coll_dev) if spec else pdist.RcclShardGather(ctx, coll_dev))
    elif world > 1:
        gather = pdist.SpecGather(coll_dev) if spec else pdist.make_gather(coll_dev)
    sim = pkg.FullSimulation.Simulation(ctx, x0, fire=D, N_iter=args.mads_iters, seed=args.seed,
                                        shard=shard, gather=gather, speculate=spec)
    t_set = time.perf_counter() - t_set
    # the in-kernel stamps: from the timed MPC steps (--stamps timed) or, by default, from as many
    # MPC steps run right after them (the loop's state moves on, so the same steps cannot be rerun);
    # the slots are set up before the warmup
    stamp_timed = args.stamps == "timed"
    stamp_setup(ctx, stamp_timed)
    for _ in range(args.warmup):
        sim.step()
    torch.cuda.synchronize()
    if stamp_timed:
        ctx.profile_read(reset=True)   # (the warmup steps' stamps out)
    recs = []
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        recs.append(sim.step())
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    if not stamp_timed:
        ctx.profile(True)
        ctx.profile_read(reset=True)
        for _ in range(args.steps):
            sim.step()
        torch.cuda.synchronize()
    split = ctx.profile_split()
    kern = ctx.profile_kernels()
    k_ms, k_launches, k_cands, k_walk = ctx.profile_read(reset=True)
    ctx.profile(False)
    if world > 1:
        tt = torch.tensor([elapsed], dtype=torch.float64, device=coll_dev)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        elapsed = float(tt.item())
        # every rank must hold the same iterates (lock-step check, 8 B per rank)
        h = torch.tensor([float(np.sum(sim.outputs[-1] * np.arange(1, sim.outputs[-1].size + 1)))],
                         dtype=torch.float64, device=coll_dev)
        hs = [torch.empty_like(h) for _ in range(world)]
        dist.all_gather(hs, h)
        lockstep = len({float(v.item()) for v in hs}) == 1
    else:
        lockstep = None
    # the evaluations the reference makes: poll candidates that pass cons3 (the extreme barrier
    # never calls the objective on the others), over every rank's shard
    feas = sum(r["feasible_evaluations"] for r in recs)
    if world > 1 and spec:
        # speculation: every rank applies the same polls; the useful evaluations are the applied
        # polls' (the sequential loop's), the discarded branches' are reported beside them
        work = torch.tensor([sum(r["speculative_feasible_evaluations"] for r in recs)],
                            dtype=torch.float64, device=coll_dev)
        dist.all_reduce(work)
        spec_work = int(work.item())
        feas = sum(r["useful_feasible_evaluations"] for r in recs)
    elif world > 1:
        ft = torch.tensor([feas], dtype=torch.float64, device=coll_dev)
        dist.all_reduce(ft)
        feas = int(ft.item())
        spec_work = None
    else:
        spec_work = None
    if rank != 0:
        D.close()
        ctx.close()
        return
    evals = sum(r["evaluations"] for r in recs)
    rejected = sum(r["rejected_polls"] for r in recs)
    iters = sum(r["iterations"] for r in recs)
    succ = sum(r["successes"] for r in recs)
    M_avg = float(np.mean([r["points"] for r in recs]))
    b_eval = 24 * M_avg + 24 * cfg["N"] + 8
    avg_launch_ms = k_ms / max(k_launches, 1)
    cands_per_launch = k_cands / max(k_launches, 1)
    # roofline as config 4's: the byte floor of one exact culling poll — here a
    # representative one, the LTMADS poll (l = 2) around the final incumbent on the final point
    # list; the generated poll reads only the incumbent and the permutations (no matrix) — over
    # the mean device chain per poll (in-kernel stamps)
    kernels, dominant = kernel_table(kern)
    x, y, w = ctx.get_points()
    polls = wl.poll_candidates(sim.x_prev, wl.SplitMix64(args.seed + 1))
    n = polls.shape[1]
    floor = floor_bytes_points(x, y, w, polls, 8 * n + 2 * 4 * n)
    chain_ms = (split[0] + split[1] + split[2]) / split[3] if split[3] else None
    achieved = floor["bytes"] / (chain_ms * 1e-3) / 1e9 if chain_ms else None
    cpu = None
    if not args.no_cpu and world == 1:
        threads, cinfo = usable_cpus()
        try:
            # the CPU sample evaluates what the reference would: the candidates passing cons3
            # (around the last MPC step's start, as the loop's polls are)
            orc = ge.load_oracle()
            prev = sim.records[-1]["input"]
            feas_mask = orc.cons3_batch(prev, polls, sim.d_lim, sim.tan)
            fpolls = polls[np.asarray(feas_mask, dtype=bool)]
            if fpolls.shape[0] == 0:
                raise RuntimeError("no candidate of the sample poll passes cons3")
            v, desc = cpu_baseline(x, y, w, fpolls, args.cpu_seconds, threads)
            cpu = {"value": v, "unit": "evals/s", "cores": threads, "kind": "port",
                   "sample": desc + f" (the final config-5 point list; the {fpolls.shape[0]} of "
                             f"{polls.shape[0]} candidates of an ell=2 poll that pass cons3)", **cinfo}
        except Exception as e:  # report, never fake
            log("cpu baseline failed:", e)
    out = {
        "metric": METRIC, "value": feas / elapsed, "unit": "evals/s", "n_gpus": world,
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
            "feasible_evaluations": feas,
            "candidates_polled": evals,
            "value_basis": "feasible_evaluations / elapsed: the poll candidates that pass cons3 "
                           "and are evaluated (the start points' evaluations not counted); "
                           "candidates_polled counts every generated candidate (1 + 2n per "
                           "iteration)",
            "mads_iterations": iters,
            "exchange_rounds": sum(r["rounds"] for r in recs),
            "speculative_feasible_evaluations_all_ranks": spec_work,
            "mads_successes": succ,
            "failure_fraction": (1.0 - succ / iters) if iters else None,
            "rejected_polls": rejected,
            "rejected_note": "iterations cons3 rejects whole (every variable's diagonal step "
                             "+-2^ell alone breaks d_lim): a failure with no launch (stepper) or "
                             "a poll whose launches return at once (pipelined loop)",
            "time_split_s": {k: float(np.sum([r[k] for r in recs]))
                             for k in ("fire_s", "remove_s", "mads_s")},
            "mads_host_split_s": {k: float(np.sum([r.get("mads_host_s", {}).get(k, 0.0) for r in recs]))
                                  for k in ("host_enqueue_s", "host_perm_s", "wait_s", "host_post_s")},
            "slot_fallbacks": int(sum(r.get("slot_fallbacks", 0) for r in recs)),
            "exchange": type(gather).__name__ if gather is not None else None,
            "parallelism": ("1 GPU" if world == 1 else
                            (f"{world} GPUs: speculation over failure branches (rank j polls the "
                             f"poll after j failures), one 24-B all-gather per round; fire stream "
                             f"regenerated per GPU") if spec else
                            f"{world} GPUs: every poll's 2n candidates sharded, 16-B all-gather "
                            f"per MADS iteration; fire stream regenerated per GPU"),
            "ranks_in_lockstep": lockstep,
        },
        "roofline": {
            "bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
            "frac": (achieved / HBM_PEAK_GBS) if achieved else None, "traffic": None,
            "kernel": (f"poll chains ({', '.join(k for k, v in kernels.items() if v.get('launches'))}); "
                       f"dominant kernel {dominant}"),
            "chain_ms": chain_ms, "polls": split[3],
            "split_ms_per_poll": ({"prep": split[0] / split[3], "walk": split[1] / split[3],
                                   "after_walk": split[2] / split[3]} if split[3] else None),
            "floor": floor, "evals_per_launch": cands_per_launch,
            "dominant_kernel": dominant,
            "avg_launch_ms": kernels[dominant]["avg_us"] * 1e-3 if dominant else avg_launch_ms,
            "kernels": kernels,
            "brute_force_equiv": {"bytes_per_eval": b_eval,
                                  "note": "SURVEY 8(d)'s full-scan bytes per evaluation at the mean "
                                          "list length: not a roofline of this algorithm"},
            "note": "achieved = floor.bytes (a representative poll: the final incumbent's) / the "
                    "mean device chain per poll (first workgroup start of its first launch to the "
                    "last workgroup end of finalize, in-kernel stamps)",
            "timing": ("in-kernel stamps over the timed MPC steps" if args.stamps == "timed" else
                       f"in-kernel stamps over {args.steps} MPC steps run right after the timed ones"),
        },
        "cpu_baseline": cpu,
        "setup_s": t_set,
    }
    if world != args.gpus:
        raise SystemExit(f"bench.py: {world} rank(s) but --gpus {args.gpus}")
    print(json.dumps(out), flush=True)
    D.close()
    ctx.close()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    # config 4's default timed region: 200 polls (~18 ms of device work, a steady state the
    # 20-poll region's 1.8 ms did not always reach), after 20 warmup polls
    ap.add_argument("--steps", type=int, default=None,
                    help="timed steps (default: 200 for configs 2-4, 3 for config 5)")
    ap.add_argument("--warmup", type=int, default=None,
                    help="warmup steps (default: 20 for configs 2-4, 1 for config 5)")
    ap.add_argument("--config", type=int, default=4, choices=(2, 3, 4, 5),
                    help="4 (default): one MADS poll per step; 5: one end-to-end MPC step "
                         "(CA fire stream + rmvCoveredPOI + a MADS run) per step")
    ap.add_argument("--mads-iters", type=int, default=100, help="config 5: N_iter per MPC step")
    ap.add_argument("--chain", choices=["auto", "five", "fused"], default="auto",
                    help="poll chain: the device's choice (auto), the five-launch chain or the "
                         "fused three-launch chain (MAC_OPT_CHAIN)")
    ap.add_argument("--mads-mode", choices=["shard", "speculate"], default="speculate",
                    help="config 5 on P GPUs: speculate (default) over failure branches (rank j "
                         "polls the poll after j failures: fewer dependent rounds), or shard "
                         "every poll's candidates (the per-poll chain does not shrink)")
    ap.add_argument("--algo", default="auto", choices=("auto", "tiled", "scan", "poll"))
    ap.add_argument("--polls", type=int, default=8,
                    help="distinct poll sets cycled over steps (8 x 37.8 MB at config 4: more than the "
                         "256-MB Infinity Cache holds, so every poll reads its matrix from HBM)")
    ap.add_argument("--tile-points", type=int, default=None,
                    help="points per spatial tile of the index (library default when omitted)")
    ap.add_argument("--cpu-seconds", type=float, default=15.0)
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--no-extras", action="store_true",
                    help="skip the parity guard and the closure timing (profiler passes: only "
                         "the warmup and timed polls launch kernels after set-up)")
    ap.add_argument("--seed", type=int, default=20250216)
    ap.add_argument("--scaling", default="weak", choices=("strong", "weak"),
                    help="N>1: weak (default) = one full poll set per GPU (P*K candidates per "
                         "step: a P-fold wider poll, one 16-B argmin all-gather); strong = the "
                         "single poll's candidates sharded over the GPUs (its latency-bound chain "
                         "barely shrinks per rank: DESIGN.md section 6)")
    ap.add_argument("--shard-of", type=int, default=1,
                    help="time rank 0's shard of a P-way strong split alone on one GPU (no "
                         "collective; value = shard candidates / time)")
    ap.add_argument("--disk-shard-of", type=int, default=1,
                    help="time rank 0's share of a P-way DISK split alone on one GPU: every "
                         "candidate's first ceil(N/P) UAVs (a lower bound of a disk-sharded rank: "
                         "no lower-index halo, no all-reduce of the K partial counts)")
    ap.add_argument("--disks", default="uniform", choices=("uniform", "clustered"),
                    help="UAV disks: uniform over the domain (default) or SURVEY 8(d)'s "
                         "clustered variant (sqrt(N)*40 m around the centre, overlapping)")
    ap.add_argument("--step-mode", default="plain", choices=("armed", "plain"),
                    help="one GPU: plain (default) = each poll enqueued after the previous result "
                         "(mac_poll_best_dev_f64); armed = each poll's chain enqueued behind the "
                         "context's doorbell while the previous poll runs and released once its "
                         "result is read (mac_poll_arm_dev_f64 / mac_poll_fire). Measured at "
                         "config 4: 0.0895 (plain) vs 0.0905 ms (armed): the stream's wait "
                         "releases the chain no sooner than a fresh launch starts it")
    ap.add_argument("--exchange", default="rccl", choices=("rccl", "torch"),
                    help="N>1 over RCCL: rccl (default) = libmaxcover's own communicator, the "
                         "all-gather on the poll's stream and the device argmin in one C call "
                         "(dist.RcclExchange); torch = torch.distributed's all-gather, then the "
                         "device argmin (dist.PollGather)")
    ap.add_argument("--stamps", default="separate", choices=("separate", "timed"),
                    help="config 2-4: in-kernel stamps (roofline.kernels, chain) from a second pass "
                         "over the same steps after the timed region (separate, default) or from "
                         "the timed steps themselves (timed)")
    ap.add_argument("--dist-backend", default="nccl", choices=("nccl", "gloo"),
                    help="nccl (= RCCL on ROCm) for the real multi-GPU run; gloo only to rehearse "
                         "N>1 with several ranks sharing one GPU (MAXCOVER_BENCH_DEVICE)")
    args = ap.parse_args()
    if args.steps is None:
        args.steps = 3 if args.config == 5 else 200
    if args.warmup is None:
        args.warmup = 1 if args.config == 5 else 20
    if world_plan(args.gpus) == "launch":
        sys.exit(launch_ranks(args.gpus, sys.argv[1:]))

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
        bench_config5(args, pkg, dev_index, rank, world, coll_dev)
        if distributed:
            dist.barrier()
            dist.destroy_process_group()
        return

    cfg = wl.CONFIGS[args.config]
    G, N = cfg["G"], cfg["N"]
    rng = wl.SplitMix64(args.seed)
    x, y, w = wl.grid_points(G)
    x0 = (wl.uniform_disks if args.disks == "uniform" else wl.clustered_disks)(N, G, rng)
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
    if args.disk_shard_of > 1 and not distributed:
        # rank 0's disks of a P-way disk split: UAVs [0, n) of every candidate
        n = -(-N // args.disk_shard_of)
        cols = np.concatenate([np.arange(n), N + np.arange(n), 2 * N + np.arange(n)])
        polls = [np.ascontiguousarray(p[:, cols]) for p in polls]
        N = n
    r_max = np.full(N, 30.0 * np.tan(100 / 180 * np.pi / 2))
    M = x.size
    if args.scaling == "weak":
        lo, hi = 0, K                      # a whole poll set per rank
        idx_base = rank * K                # global candidate index = rank * K + k
        K_step = K * world                 # candidates evaluated per step, all ranks
    elif args.shard_of > 1 and not distributed:
        lo, hi = pdist.shard_range(K, 0, args.shard_of)   # rank 0's shard, timed alone
        idx_base = lo
        K_step = hi - lo
    else:
        lo, hi = pdist.shard_range(K, rank, world)
        idx_base = lo
        K_step = K
    Kl = hi - lo

    ctx = pkg.Context(dev_index, algo=args.algo, tile_points=args.tile_points)
    ctx.set_chain(args.chain)
    # once per MPC step (src/FullSimulation.jl:50-61), outside the per-poll step: the host upload
    # of the list, then the device tile index over it (mac_set_points_dev_f64: sort, offsets)
    t_set = time.perf_counter()
    t_up = time.perf_counter()
    dx_, dy_, dw_ = (torch.from_numpy(a).to(dev) for a in (x, y, w))
    torch.cuda.synchronize(dev)
    t_up = time.perf_counter() - t_up
    t_idx = time.perf_counter()
    ctx.set_points_device(dx_, dy_, dw_)
    torch.cuda.synchronize(dev)
    t_idx = time.perf_counter() - t_idx
    del dx_, dy_, dw_
    t_set = time.perf_counter() - t_set
    d_polls = [torch.from_numpy(np.ascontiguousarray(p[lo:hi])).to(dev) for p in polls]
    d_rmax = torch.from_numpy(r_max).to(dev)
    d_best = torch.empty(2, dtype=torch.float64, device=dev)
    # cons3 (src/TDM_Constraints.jl:54-75) is part of every reference poll (extreme constraints
    # [cons1, cons3], src/TDM_STATIC_opt.jl:151-153): prev = the incumbent, d_lim = 10 m
    # (src/FullSimulation.jl:740), FOV = 100 deg (:735)
    tan_half = float(np.tan(100 / 180 * np.pi / 2))
    dlim = np.full(N, 10.0)
    d_dlim = torch.from_numpy(dlim).to(dev)
    d_prevs = [torch.from_numpy(np.ascontiguousarray(p[0])).to(dev) for p in polls]
    stream = torch.cuda.Stream(dev)
    s_handle = stream.cuda_stream

    # one bound poll per candidate set: the ctypes arguments are built once (Context.poll_step)
    steps = [ctx.poll_step(d, 3 * N, Kl, d_rmax, d_best, d_prev=pv, d_dlim=d_dlim,
                           tan_half_fov=tan_half, idx_base=idx_base, stream=s_handle)
             for d, pv in zip(d_polls, d_prevs)]

    # N > 1: the 16-B all-gather straight from d_best, ordered after the poll on its stream,
    # and one pinned host read of the world x 16-B result (dist.PollGather)
    # (RCCL: libmaxcover's own communicator, the all-gather on the poll's stream, dist.RcclExchange;
    # --exchange torch: torch's collective + the device argmin; gloo rehearsals: PollGather's host path)
    gat = None
    if distributed and coll_dev.type == "cuda" and args.exchange == "rccl":
        try:
            gat = pdist.RcclExchange(ctx, coll_dev)
        except Exception as e:   # (reported; the exchange then runs through torch's collective)
            log(f"bench.py: libmaxcover's RCCL exchange unavailable ({e}); torch.distributed's instead")
            gat = None
    if gat is None and distributed:
        gat = pdist.PollGather(coll_dev, ctx=ctx if coll_dev.type == "cuda" else None)
    xsteps = ([ctx.poll_step(d, 3 * N, Kl, d_rmax, d_best, d_prev=pv, d_dlim=d_dlim,
                             tan_half_fov=tan_half, idx_base=idx_base, stream=s_handle, fetch=False)
               for d, pv in zip(d_polls, d_prevs)] if isinstance(gat, pdist.RcclExchange) else None)
    xchg = gat.step_for(d_best, s_handle) if isinstance(gat, pdist.RcclExchange) else None
    # one GPU, armed: poll j + 1 is enqueued behind the doorbell while poll j runs (its inputs are
    # resident; a MADS driver fills them once poll j's result is known) and released right after
    # that result is read, so no launch sits between dependent polls. Consecutive polls alternate
    # two d_best buffers (each buffer's result slot follows its latest poll).
    armed = args.step_mode == "armed" and not distributed and K > 1
    if armed:
        d_best2 = [d_best, torch.empty(2, dtype=torch.float64, device=dev)]
        nb = len(d_polls) * 2 // np.gcd(len(d_polls), 2)
        arm, fire, fetch = ctx.armed_steps(
            [dict(d_cands=d_polls[j % len(d_polls)], three_n=3 * N, K=Kl, d_rmax=d_rmax,
                  d_best=d_best2[j % 2], d_prev=d_prevs[j % len(d_polls)], d_dlim=d_dlim,
                  tan_half_fov=tan_half, idx_base=idx_base) for j in range(nb)], stream=s_handle)

    def run_armed(first, n):
        """n dependent armed polls (poll sets first, first + 1, ...): fire j, arm j + 1 while
        poll j runs, read j's result. Every armed poll is fired before returning."""
        res = None
        arm(first % nb)
        for i in range(first, first + n):
            fire(i % nb)
            if i + 1 < first + n:
                arm((i + 1) % nb)
            res = fetch(i % nb)
        return res

    def step(i):
        """One MADS poll. It ends with the best (objective, index) on the host, because the
        next poll's candidates depend on it: polls never overlap."""
        if xsteps is not None:   # two prebuilt C calls: the poll, then the exchange
            xsteps[i % len(xsteps)]()
            t_x = time.perf_counter()
            r = xchg()
            gat.seconds += time.perf_counter() - t_x
            gat.calls += 1
            return r
        if distributed:
            d = d_polls[i % len(d_polls)]
            ctx.poll_best_dev(d, 3 * N, Kl, d_rmax, d_best, d_prev=d_prevs[i % len(d_polls)],
                              d_dlim=d_dlim, tan_half_fov=tan_half, idx_base=idx_base,
                              stream=s_handle)
            with torch.cuda.stream(stream):
                return gat(d_best)
        return steps[i % len(steps)]()   # poll + the 16-B result from pinned host memory

    # the stamp slots before the warmup, so that the warmup polls lead straight into the timed ones
    stamp_timed = args.stamps == "timed"
    stamp_setup(ctx, stamp_timed)
    if armed:
        run_armed(0, args.warmup)
    else:
        for i in range(args.warmup):
            step(i)
    torch.cuda.synchronize(dev)

    def run_steps(first):
        res = None
        if armed:
            for i in range(first, first + args.steps):
                fire(i % nb)
                if i + 1 < first + args.steps:
                    arm((i + 1) % nb)
                res = fetch(i % nb)
        else:
            for i in range(args.steps):
                res = step(first + i)
        return res

    # the timed region; the in-kernel stamps (roofline, kernels) come from the same steps run once
    # more right after it with stamping on (--stamps separate, the default: the stamps' host
    # bookkeeping stays out of the timed polls), or from the timed steps themselves (--stamps timed)
    if stamp_timed:
        ctx.profile_read(reset=True)   # (the warmup polls' stamps out)
    if gat is not None:
        gat.seconds, gat.calls = 0.0, 0
    if distributed:
        dist.barrier()
    torch.cuda.synchronize(dev)
    if armed:   # (the first timed poll's chain is enqueued before the clock starts, as every
                # later poll's is enqueued while its predecessor runs)
        arm(args.warmup % nb)
    t0 = time.perf_counter()
    result = run_steps(args.warmup)
    if distributed:
        dist.barrier()
    torch.cuda.synchronize(dev)
    elapsed = time.perf_counter() - t0
    if not stamp_timed:   # the stamped pass: the same polls (the same poll sets, in order)
        ctx.profile(True)
        ctx.profile_read(reset=True)
        if armed:
            arm(args.warmup % nb)
        run_steps(args.warmup)
        torch.cuda.synchronize(dev)
    split = ctx.profile_split()
    kern = ctx.profile_kernels()
    k_ms, k_launches, k_cands, k_walk = ctx.profile_read(reset=True)
    ctx.profile(False)
    if distributed:
        t = torch.tensor([elapsed], dtype=torch.float64, device=coll_dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    if result is None:
        b = d_best.cpu()
        result = (float(b[0]), int(b.view(torch.int64)[1]))

    # (after the timed region, which follows the warmup directly) correctness guard on the timed workload: the timed poll (this rank's shard, the device's
    # walk choice, cons3) writes every objective; 16 sampled candidates plus its argmin are
    # re-evaluated by the streaming scan (an independent kernel) and must agree bit for bit
    check = None
    if K > 1 and not args.no_extras:
        d_obj = torch.empty(Kl, dtype=torch.float64, device=dev)
        ctx.poll_best_dev(d_polls[0], 3 * N, Kl, d_rmax, d_best, d_prev=d_prevs[0], d_dlim=d_dlim,
                          tan_half_fov=tan_half, idx_base=idx_base, d_obj=d_obj, stream=s_handle)
        got_best = ctx.best_fetch(d_best, stream=s_handle)
        torch.cuda.synchronize(dev)
        objs = d_obj.cpu().numpy()
        pick = np.unique(np.concatenate([
            np.floor(wl.SplitMix64(args.seed + 7).uniform(16) * Kl).astype(np.int64),
            [int(np.argmin(objs))]]))
        ctx.set_algo("scan")
        _, _, o_scan = ctx.poll_best(polls[0][lo:hi][pick], r_max, 1e5, prev=polls[0][0],
                                     d_lim=dlim, tan_half_fov=tan_half, want_all=True)
        ctx.set_algo(args.algo)
        kmin = int(np.argmin(objs))
        check = bool(np.array_equal(o_scan, objs[pick]) and got_best[1] == idx_base + kmin
                     and got_best[0] == objs[kmin])
        if not check:
            log("WARNING: timed poll vs scan disagree", pick, o_scan, objs[pick], got_best)


    total_evals = K_step * args.steps
    value = total_evals / elapsed
    ms_per_step = elapsed / args.steps * 1e3

    # roofline. The unit is one poll's device chain, timed live by in-kernel workgroup stamps
    # over the timed steps. Its algorithmic floor is what any exact culling evaluation must move:
    # the candidate matrix read once, every entry that lies in some disk's poll-wide footprint
    # box read once (xy, 16 B; w only when the weights differ), and the 16-B result.
    avg_launch_ms = k_ms / max(k_launches, 1)
    cands_per_launch = k_cands / max(k_launches, 1)
    floor = floor_bytes(x, y, w, polls[0][lo:hi], G)
    # the unit is the whole poll chain on the device: first workgroup start of its first launch
    # to the last workgroup end of its last (finalize + argmin), from the in-kernel stamps
    chain_ms = (split[0] + split[1] + split[2]) / split[3] if split[3] else None
    unit_ms = chain_ms if chain_ms else avg_launch_ms
    achieved = floor["bytes"] / (unit_ms * 1e-3) / 1e9 if (k_launches and unit_ms) else None
    b_eval = 3 * M * 8 + 3 * N * 8 + 8     # a brute-force scan per candidate
    traffic, traffic_src, pmc_per = pmc_traffic(args.config, args.disks, world, args.algo)
    kernels, dominant = kernel_table(kern, pmc_per)

    # the single-candidate closure path (src/TDM_STATIC_opt.jl:125: DirectSearch calls the
    # objective once per trial point): host-pointer mac_area_f64 latency on the timed workload
    closure = None
    if rank == 0 and not args.no_extras:
        c0 = np.ascontiguousarray(polls[0][min(1, K - 1)])
        for _ in range(20):
            ctx.area(c0)
        n_cl = 300
        t_cl = time.perf_counter()
        for _ in range(n_cl):
            a_cl = ctx.area(c0)
        closure = {"mac_area_f64_us": (time.perf_counter() - t_cl) / n_cl * 1e6, "calls": n_cl,
                   "area": a_cl, "note": "host candidate in, host double out: copy-in, the walk, "
                   "copy-out, synchronous (what a Julia ccall per trial point costs)",
                   "threads": closure_threads(ctx, polls[0], (1, 4, 16))}

    # the host-pointer poll (a DirectSearch-owned poll handed over through the C ABI from host
    # memory, src/TDM_STATIC_opt.jl:162): the whole 3N x 2n matrix (mac_poll_best_f64) against
    # the basis form (mac_poll_best_basis: incumbent + L's packed triangle + permutations + delta,
    # mac_poll_basis_f64), both with cons3, timed per call on the same poll (results must agree)
    host_poll = None
    if rank == 0 and not args.no_extras and K > 1 and args.disk_shard_of == 1:
        n = 3 * N
        Lm, rp_, cp_ = wl.ltmads_basis_parts(n, 2, wl.SplitMix64(args.seed + 11))
        Bm = Lm[rp_][:, cp_].astype(np.float64)
        Cm = np.ascontiguousarray(np.concatenate([x0[None, :] + Bm.T, x0[None, :] - Bm.T]))
        tri = np.ascontiguousarray(Lm[np.tril_indices(n)], dtype=np.int16)
        kw3 = dict(prev=x0, d_lim=dlim, tan_half_fov=tan_half)
        res_m = ctx.poll_best(Cm, r_max, 1e5, **kw3)
        res_b = ctx.poll_basis(x0, tri, rp_, cp_, 1.0, r_max, 1e5, **kw3)
        reps = 20
        t_m = time.perf_counter()
        for _ in range(reps):
            ctx.poll_best(Cm, r_max, 1e5, **kw3)
        t_m = (time.perf_counter() - t_m) / reps
        t_b = time.perf_counter()
        for _ in range(reps):
            ctx.poll_basis(x0, tri, rp_, cp_, 1.0, r_max, 1e5, **kw3)
        t_b = (time.perf_counter() - t_b) / reps
        host_poll = {
            "matrix_ms": t_m * 1e3, "basis_ms": t_b * 1e3, "candidates": int(Cm.shape[0]),
            "matrix_bytes": int(Cm.nbytes), "basis_bytes": int(8 * n + 8 * n + tri.nbytes),
            "agree": bool(res_m == res_b), "calls": reps,
            "note": "host memory in, (objective, index) out, synchronous, with cons3: "
                    "mac_poll_best_f64 ships the 3N x 2n matrix; mac_poll_basis_f64 ships the "
                    "incumbent, L's packed lower triangle (int16), rp, cp and delta and expands "
                    "the candidates on the device"}

    out = None
    if rank == 0:
        cpu = None
        if not args.no_cpu and world == 1:
            threads, cinfo = usable_cpus()
            try:
                v, desc = cpu_baseline(x, y, w, polls[0], args.cpu_seconds, threads)
                cpu = {"value": v, "unit": "evals/s", "cores": threads, "kind": "port",
                       "sample": desc, **cinfo}
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
                "disks": ("integer centres uniform over the domain, R=36" if args.disks == "uniform"
                          else "clustered: integer centres within sqrt(N)*40 m of the centre, R=36"),
                "cons3": "prev = incumbent, d_lim = 10 m, FOV 100 deg (every candidate checked)",
                "parallelism": (f"rank 0 of a {args.disk_shard_of}-way disk split (UAVs 0..{N - 1} "
                                f"of every candidate), timed alone on 1 GPU (no halo, no collective)"
                                if args.disk_shard_of > 1 and not distributed else
                                f"rank 0 of a {args.shard_of}-way candidate split, timed alone on "
                                f"1 GPU (no collective)" if args.shard_of > 1 and not distributed else
                                f"{world} GPU(s), one full poll set each, 16-B argmin all-gather"
                                if args.scaling == "weak" else
                                f"one poll's candidates sharded over {world} GPU(s), "
                                f"16-B argmin all-gather"),
                "algo": args.algo, "chain": args.chain,
                "step_mode": "armed" if armed else "plain",
                "poll_sets": args.polls,
                "poll_sets_bytes": int(args.polls * K * 3 * N * 8),
            },
            "roofline": {
                "bound": "hbm",
                "achieved": achieved,
                "peak": HBM_PEAK_GBS,
                "unit": "GB/s",
                "frac": (achieved / HBM_PEAK_GBS) if achieved else None,
                "traffic": traffic,
                "kernel": (f"poll chain ({', '.join(k for k, v in kernels.items() if v.get('launches'))}); "
                           f"dominant kernel {dominant}"),
                "chain_ms": chain_ms,
                "dominant_kernel": dominant,
                "dominant_basis": ("in-kernel stamps: first workgroup start to last workgroup end; "
                                   "rocprof's dispatch-to-completion durations add the dispatch "
                                   "ramp and the end-of-kernel release, which weigh most on the "
                                   "prep launch (512 x 512-thread workgroups, 10 MB of stores), "
                                   "and can rank it first (profiles/*rocprof*config4.csv)"),
                "avg_launch_ms": (kernels[dominant]["avg_us"] * 1e-3 if dominant else avg_launch_ms),
                "kernels": kernels,
                "walk_avg_launch_ms": avg_launch_ms,
                "evals_per_launch": cands_per_launch,
                "split_ms_per_poll": ({"prep": split[0] / split[3], "walk": split[1] / split[3],
                                       "after_walk": split[2] / split[3]} if split[3] else None),
                "floor": floor,
                "traffic_source": traffic_src,
                "traffic_frac": (traffic / (unit_ms * 1e-3) / 1e9 / HBM_PEAK_GBS
                                 if traffic and unit_ms else None),
                "brute_force_equiv": {
                    "bytes_per_eval": b_eval,
                    "achieved": b_eval * cands_per_launch / (avg_launch_ms * 1e-3) / 1e9
                    if k_launches else None,
                    "note": "SURVEY 8(d)'s full-scan bytes per evaluation: what a brute-force "
                            "scan would have to stream, not a roofline of this algorithm"},
                "timing": ("in-kernel workgroup stamps (s_memrealtime) over the timed steps"
                           if args.stamps == "timed" else
                           "in-kernel workgroup stamps (s_memrealtime) over a second pass of the "
                           "timed steps (the same polls), run right after the timed region"),
                "note": "achieved = floor.bytes / chain_ms (first workgroup start of the chain's "
                        "first launch to the last workgroup end of its last); avg_launch_ms = the "
                        "dominant (longest) kernel alone, kernels = every launch of the chain "
                        "(in-kernel stamps over the timed steps; compare with profiles/*rocprof*); "
                        "traffic = PMC-measured HBM bytes of the whole chain per poll (per kernel "
                        "in kernels.*.hbm_bytes), attached only when the kernel sources hash to "
                        "the profiled build",
            },
            "cpu_baseline": cpu,
            "closure": closure,
            "host_poll_ms": host_poll,
            "exchange": (type(gat).__name__ if gat is not None else None),
            "best": {"objective": result[0], "index": result[1]},
            "check_timed_poll_vs_scan": check,
            "setup_s": t_set,
            "setup": {
                "host_upload_s": t_up, "index_rebuild_s": t_idx,
                "note": "once per MPC step (the point list changes between MADS runs, "
                        "src/FullSimulation.jl:50-61), outside ms_per_step: host upload of the "
                        "x/y/w list, then the device tile index over it (mac_set_points_dev_f64: "
                        "bbox, tile keys, radix sort, gather, offsets). Amortised over a run's "
                        "polls: index_rebuild_s / polls per MPC step (100 in the reference)"},
        }
        if distributed:
            out["config"]["gather_host_us_per_poll"] = (gat.seconds / max(gat.calls, 1) * 1e6
                                                        if gat else None)
        ranks = dist.get_world_size() if distributed else 1
        if out["n_gpus"] != ranks or ranks != args.gpus:
            raise SystemExit(f"bench.py: n_gpus {out['n_gpus']}, {ranks} rank(s), --gpus {args.gpus}")
        print(json.dumps(out), flush=True)
    if distributed:
        dist.barrier()
        dist.destroy_process_group()
    ctx.close()


if __name__ == "__main__":
    main()
