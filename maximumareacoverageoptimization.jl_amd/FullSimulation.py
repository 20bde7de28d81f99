"""The hot-path part of src/FullSimulation.jl's MPC loop (run_simulation :23-278), on the GPU:
config 5 of BASELINE.json, a CA fire streamed into the point list every MPC step.

Per timestep t (:42-100):
  1. update_POI: new fire points appended to the device list (:50-52). The source is either the
     GPU cellular automaton (DynamicArea) or rows of a FirePoints table (src/CellFunctions.jl:59-79).
  2. drone_locs = the previous circles. rmvCoveredPOI deletes the entries they cover,
     order-preserving (:56-61).
  3. r_max update for UAVs at the 15 m altitude near the high-interest box (:64-76).
  4. cons3 around the previous circles (:78).
  5. The MADS input is drone_locs for t < 3, else the previous MADS output, unless it violates
     cons3 (:82-93).
  6. MADS (N_iter iterations) on the device: mac_mads_run, one complete LTMADS poll per
     iteration (:84-95). On P GPUs (``shard = (rank, P)``, config 5 "8 GPUs") every rank runs
     steps 1-5 itself — the fire CA is deterministic, so each GPU regenerates the same point
     list with no transfer — and polls its shard of every LTMADS poll (mac_mads_begin / _poll /
     _update); ``gather`` (dist.make_gather: a 16-B all-gather) combines the ranks' bests, so
     every rank holds the single-GPU iterates.
The trajectory stage (ALTRO, :107-251) is out of scope. The next step's circles are taken to be
the MADS output, i.e. perfect tracking, which the reference's trajectory stage aims at.
"""
from __future__ import annotations

import math
import time

import numpy as np

from ._lib import Context
from .DynamicArea import DynamicArea

FOV = 100 / 180 * math.pi          # :735
h_max = 30.0                       # :737
N_iter = 100                       # :741
x_LB, x_UB, y_LB, y_UB = [2500], [3500], [1000], [2000]   # :751-754


def r_max_update(drone_locs: np.ndarray, r_max: np.ndarray, N: int) -> None:
    """:64-76 (t != 1): a UAV flying at ~15 m that is within h_max*tan(FOV/2) of the
    high-interest box keeps r_max = 15*tan(FOV/2); otherwise r_max = h_max*tan(FOV/2)."""
    t2 = math.tan(FOV / 2)
    for i in range(N):
        if abs(15 - drone_locs[i + 2 * N] / t2) < 1:
            check = [(drone_locs[i] < xu + h_max * t2) and (drone_locs[i] > xl - h_max * t2) and
                     (drone_locs[i + N] < yu + h_max * t2) and (drone_locs[i + N] > yl - h_max * t2)
                     for xl, xu, yl, yu in zip(x_LB, x_UB, y_LB, y_UB)]
            r_max[i] = 15 * t2 if any(check) else h_max * t2


def cons3_ok(prev: np.ndarray, x: np.ndarray, d_lim: np.ndarray) -> bool:
    """src/TDM_Constraints.jl:54-75 on the host (the pre-check of :88)."""
    N = x.size // 3
    t2 = math.tan(FOV / 2)
    for i in range(N):
        dx, dy = prev[i] - x[i], prev[N + i] - x[N + i]
        dz = prev[2 * N + i] / t2 - x[2 * N + i] / t2
        if math.sqrt(dx * dx + dy * dy + dz * dz) > d_lim[i]:
            return False
    return True


class Simulation:
    """The MPC loop as a stepper (one ``step()`` per timestep t = 1, 2, ...). Point source:
    ``fire`` (GPU CA: its initial points first, one CA step per MPC step), ``firepoints`` (table
    rows: rows 1..10 initially, then row t+10), or ``initial_points`` alone (static)."""

    def __init__(self, ctx: Context, starting_circles, *, fire: DynamicArea | None = None,
                 firepoints=None, initial_points=None, N_iter: int = N_iter, d_lim=None,
                 r_max=None, seed: int = 20250216, ell0: int = 2, ell_max: int = 6,
                 shard=None, gather=None, speculate: bool | None = None, device=None):
        self.ctx = ctx
        self.x_prev = np.asarray(starting_circles, dtype=np.float64).copy()
        self.N = N = self.x_prev.size // 3
        self.tan = math.tan(FOV / 2)
        self.d_lim = np.full(N, 10.0) if d_lim is None else np.asarray(d_lim, dtype=np.float64)
        self.r_max = (np.full(N, h_max * self.tan) if r_max is None
                      else np.asarray(r_max, dtype=np.float64).copy())
        self.fire, self.firepoints = fire, firepoints
        self.N_iter, self.seed, self.ell0, self.ell_max = N_iter, seed, ell0, ell_max
        self.shard = shard          # (rank, world) or None: the whole poll on this GPU
        # P GPUs: speculate over failure branches, rank j polling the poll after j failures
        # (gather: dist.SpecGather) — the default, since sharding one poll cannot shorten its
        # latency-bound chain — or shard every poll's candidates (speculate=False,
        # gather: dist.make_gather). With no gather given, the default one is made on `device`
        # (the collective's device: the rank's GPU under RCCL, "cpu" under gloo).
        multi = shard is not None and shard[1] > 1
        if speculate is None:
            from .dist import SpecGather
            speculate = multi and (gather is None or isinstance(gather, SpecGather))
        if multi and gather is None:
            from .dist import RcclShardGather, RcclSpecGather, SpecGather, make_gather
            dev = device if device is not None else "cpu"
            if str(dev).startswith("cuda"):   # libmaxcover's own RCCL communicator on ctx
                gather = RcclSpecGather(ctx, dev) if speculate else RcclShardGather(ctx, dev)
            else:
                gather = SpecGather(dev) if speculate else make_gather(dev)
        self.gather = gather
        self.speculate = bool(speculate)
        if fire is not None:
            ctx.set_points_records(fire.initial_points())
        elif firepoints is not None:
            ctx.set_points_records(np.concatenate([np.asarray(r).reshape(-1, 5)
                                                   for r in firepoints[:10]] or [np.zeros((0, 5))]))
        else:
            ctx.set_points_records(np.asarray(initial_points, dtype=np.float64).reshape(-1, 5))
        self.t = 0
        self.outputs = []
        self.records = []

    def step(self) -> dict:
        ctx, N = self.ctx, self.N
        self.t += 1
        t = self.t
        t0 = time.perf_counter()
        added = 0
        if self.fire is not None:                                        # :50-52
            added = self.fire.fire.step(append_to=ctx)
        elif self.firepoints is not None and t != 1 and t + 10 - 1 < len(self.firepoints):
            row = np.asarray(self.firepoints[t + 10 - 1]).reshape(-1, 5)
            if row.shape[0]:
                ctx.append_points(row[:, 0], row[:, 1], row[:, 3])
                added = row.shape[0]
        t1 = time.perf_counter()
        drone_locs = self.x_prev.copy()                                  # :56-57
        kept = ctx.remove_covered(drone_locs)                            # :61
        t2 = time.perf_counter()
        if t != 1:
            r_max_update(drone_locs, self.r_max, N)                      # :64-76
        if t < 3:                                                        # :82-84
            single_input = drone_locs
        else:
            single_input = self.outputs[-1]
            if not cons3_ok(self.x_prev, single_input, self.d_lim):     # :88-90
                single_input = drone_locs
        kw = dict(prev=self.x_prev, d_lim=self.d_lim, tan_half_fov=self.tan, n_iter=self.N_iter,
                  ell0=self.ell0, ell_max=self.ell_max, seed=self.seed + t)
        if self.shard is None or self.shard[1] == 1:
            x_out, st = ctx.mads_run(single_input, self.r_max, 1e5, **kw)
        elif self.speculate:
            from .dist import mads_loop_speculative
            stepper = ctx.mads_stepper(single_input, self.r_max, 1e5, **kw)
            try:
                x_out, st = mads_loop_speculative(stepper, self.gather)
            finally:
                stepper.close()
        else:
            from .dist import mads_loop, shard_range
            lo, hi = shard_range(2 * single_input.size, *self.shard)
            stepper = ctx.mads_stepper(single_input, self.r_max, 1e5, shard=(lo, hi), **kw)
            try:
                x_out, st = mads_loop(stepper, self.gather)
            finally:
                stepper.close()
        t3 = time.perf_counter()
        self.outputs.append(x_out)
        rec = dict(t=t, points=int(ctx.num_points), added=int(added), kept=int(kept.size),
                   f=st["f"], iterations=st["iterations"], evaluations=st["evaluations"],
                   feasible_evaluations=int(st.get("feasible_evaluations", 0)),
                   rejected_polls=int(st.get("rejected_polls", 0)),
                   successes=int(st.get("successes", 0)),
                   rounds=int(st.get("rounds", st["iterations"])),
                   useful_feasible_evaluations=int(st.get("useful_feasible_evaluations",
                                                          st.get("feasible_evaluations", 0))),
                   speculative_feasible_evaluations=int(st.get("speculative_feasible_evaluations",
                                                               st.get("feasible_evaluations", 0))),
                   slot_fallbacks=int(st.get("slot_fallbacks", 0)),
                   fire_s=t1 - t0, remove_s=t2 - t1, mads_s=t3 - t2, step_s=t3 - t0,
                   mads_host_s={k: float(st.get(k, 0.0)) for k in
                                ("host_enqueue_s", "host_perm_s", "wait_s", "host_post_s")},
                   input=single_input)
        self.records.append(rec)
        self.x_prev = x_out                                              # perfect tracking
        return rec


def run_simulation(ctx: Context, starting_circles, Nt_sim: int, log=None, **kw):
    """run_simulation's optimisation side for Nt_sim steps: (records, MADS outputs)."""
    sim = Simulation(ctx, starting_circles, **kw)
    for _ in range(Nt_sim):
        rec = sim.step()
        if log:
            log(rec)
    return sim.records, sim.outputs
