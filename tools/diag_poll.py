"""Diagnostic: per-workgroup timing of the poll kernel's roles (diagnostic build
libmaxcover_diag.so).

MAXCOVER_LIB=.../libmaxcover_diag.so python tools/diag_poll.py [--config 4]
Stamps are s_memrealtime (100 MHz) per workgroup, indexed by linear block id: start, end,
(role << 56 | info), XCC. Roles: 1 = penalty chains, 2 = shared entries, 3 = disk walk.
Only the diagnostic build executes stamps; never quote its timings as kernel performance.
"""
import argparse
import ctypes
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import __graft_entry__ as ge  # noqa: E402

KPB = 1 << 30   # one walk workgroup per disk (grid row 0 only)
THREADS = 256     # kPollThreads
SHB = 256         # kSharedWG (shared-entry workgroups, spread over the grid rows)
CHAINC = 16       # kChainC (candidates per penalty-chain workgroup)


def analyze(L, N, K):
    """Role timings of the LAST poll-kernel launch (N disks, K candidates)."""
    gy = (K + KPB - 1) // KPB
    n_chain = ((K + CHAINC - 1) // CHAINC + gy - 1) // gy
    gx = n_chain + (SHB + gy - 1) // gy + N
    nb = gx * gy
    buf = (ctypes.c_uint64 * (4 * nb))()
    assert L.mac_diag_read(buf, 4 * nb) == 0
    a = np.frombuffer(buf, dtype=np.uint64).reshape(-1, 4)
    ok = a[:, 0] > 0
    a = a[ok].astype(np.int64)
    t0, t1 = a[:, 0], a[:, 1]
    role = (a[:, 2].astype(np.uint64) >> np.uint64(56)).astype(np.int64)
    info = a[:, 2] & ((1 << 56) - 1)
    # the last launch only: blocks that started within 5 ms of the latest start
    last = t0 >= t0.max() - 500000
    t0, t1, role, info = t0[last], t1[last], role[last], info[last]
    base = t0.min()
    dur = (t1 - t0) / 100.0
    out = {"blocks_stamped": int(last.sum()), "span_us": float((t1.max() - base) / 100.0)}
    for r, name in ((1, "chains"), (2, "shared"), (3, "walk")):
        m = role == r
        if not m.any():
            continue
        d = dur[m]
        out[name] = {
            "blocks": int(m.sum()),
            "dur_us": {q: float(np.percentile(d, q)) for q in (0, 50, 90, 100)},
            "start_us": float((t0[m].min() - base) / 100.0),
            "end_us": float((t1[m].max() - base) / 100.0),
            "concurrency_avg": float(d.sum() / max((t1[m].max() - t0[m].min()) / 100.0, 1e-9)),
        }
        if r == 3:
            ent = info[m] & 0xFFFFF
            pos = (info[m] >> 20) & 0xFFFFF
            out[name]["entries_median"] = float(np.median(ent))
            out[name]["entries_max"] = float(np.max(ent))
            out[name]["positions_median"] = float(np.median(pos))
            out[name]["neighbours_median"] = float(np.median(info[m] >> 40))
        if r == 2:
            out[name]["disks_with_neighbours"] = int(info[m].max())
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", type=int, default=4)
    args = ap.parse_args()
    pkg = ge.load_package()
    L = pkg.load_library()
    if not hasattr(L, "mac_diag_read"):
        raise SystemExit("not the diagnostic build (set MAXCOVER_LIB)")
    L.mac_diag_read.argtypes = [ctypes.POINTER(ctypes.c_uint64), ctypes.c_int64]
    if args.config == 5:  # the last MADS iteration's poll of the second MPC step (config 5)
        wl = pkg.workloads
        rng = wl.SplitMix64(wl.SEED)
        cfg = wl.CONFIGS[5]
        fire_kw, x0 = wl.config5_setup(rng, cfg["G"], cfg["N"], cfg["ignition"])
        ctx = pkg.Context(0, algo="poll")
        D = pkg.DynamicArea.DynamicArea(**fire_kw, seed=wl.SEED, device=0)
        sim = pkg.FullSimulation.Simulation(ctx, x0, fire=D, N_iter=100, seed=wl.SEED)
        for _ in range(2):
            rec = sim.step()
        N = x0.size // 3
        out = analyze(L, N, 2 * 3 * N)
        out["mpc_step"] = {k: rec[k] for k in ("points", "kept", "evaluations", "mads_s")}
    else:
        x, y, w, C, rmax = pkg.workloads.make_config(args.config)
        ctx = pkg.Context(0, algo="poll")
        ctx.set_points(x, y, w)
        for _ in range(3):
            ctx.poll_best(C, rmax)
        out = analyze(L, C.shape[1] // 3, C.shape[0])
        N = C.shape[1] // 3
        L.mac_diag_walk_read.argtypes = [ctypes.POINTER(ctypes.c_uint64), ctypes.c_int64]
        buf = (ctypes.c_uint64 * (8 * N))()
        assert L.mac_diag_walk_read(buf, 8 * N) == 0
        a = np.frombuffer(buf, dtype=np.uint64).reshape(N, 8).astype(np.int64)[:, :6]
        a = a[(a > 0).all(axis=1)]
        ph = np.diff(a, axis=1) / 100.0
        out["walk_phases"] = {
            "names": ["prologue (urec, lanes)", "off + prefix", "staging", "tests", "rest + write"],
            "median_us": [float(v) for v in np.median(ph, axis=0)],
            "max_us": [float(v) for v in ph.max(axis=0)],
            "start_us_pct": [float(v) for v in np.percentile((a[:, 0] - a[:, 0].min()) / 100.0,
                                                            (0, 50, 100))]}
    bb = (ctypes.c_uint64 * (8 * 4096))()
    if hasattr(L, "mac_diag_band_read") and L.mac_diag_band_read(bb, 8 * 4096) == 0:
        a = np.frombuffer(bb, dtype=np.uint64).reshape(4096, 8).astype(np.int64)
        a = a[a[:, 0] > 0]
        if a.size:
            base = a[:, 0].min()
            full = a[(a[:, 1:7] > 0).all(axis=1)]
            out["band_jobs"] = {
                "jobs": int(a.shape[0]), "with_entries": int(full.shape[0]),
                "end_us_max": float((a[:, 1:7].max() - base) / 100.0)}
            if full.size:
                ph = np.diff(full[:, :7], axis=1) / 100.0
                out["band_jobs"].update({
                    "names": ["tiles", "stage", "A masks", "neighbours+count", "rest chunks", "atomics"],
                    "median_us": [float(v) for v in np.median(ph, axis=0)],
                    "max_us": [float(v) for v in ph.max(axis=0)],
                    "ns_median": float(np.median(full[:, 7] >> 32)),
                    "nc_median": float(np.median((full[:, 7] >> 16) & 0xFFFF)),
                    "U_median": float(np.median(full[:, 7] & 0xFFFF))})
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
