"""Diagnostic: per-workgroup timeline of the fused poll (diagnostic build only).

    MAXCOVER_LIB=$PWD/maximumareacoverageoptimization.jl_amd/libmaxcover_diag.so \\
        python tools/diag_fused.py [--config 4] [--disks uniform|clustered]

Runs fused polls with in-kernel stamps on and prints, per launch and role, the workgroup
durations and the launch timeline (us)."""
import argparse, ctypes, json, os, sys
import numpy as np
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import __graft_entry__ as ge  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--config", type=int, default=4)
ap.add_argument("--disks", default="uniform")
ap.add_argument("--polls", type=int, default=5)
args = ap.parse_args()
pkg = ge.load_package()
L = pkg.load_library()
L.mac_diag_stamps.argtypes = [ctypes.c_void_p, ctypes.POINTER(ctypes.c_uint64), ctypes.c_int64,
                              ctypes.POINTER(ctypes.c_int64)]
x, y, w, C, rmax = pkg.workloads.make_config(args.config, disks=args.disks)
N = C.shape[1] // 3
K = C.shape[0]
ctx = pkg.Context(0, algo="fused")
ctx.set_points(x, y, w)
tan = float(np.tan(100 / 180 * np.pi / 2))
dl = np.full(N, 10.0)
for _ in range(2):
    ctx.poll_best(C, rmax, 1e5, prev=C[0], d_lim=dl, tan_half_fov=tan)
ctx.profile(True)
ctx.profile_read(reset=True)
for _ in range(args.polls):
    ctx.poll_best(C, rmax, 1e5, prev=C[0], d_lim=dl, tan_half_fov=tan)
n_chain = (K + 63) // 64
ndt, nct = (N + 31) // 32, (K + 63) // 64
n1 = n_chain + ndt * nct
n2 = N + 256
buf = (ctypes.c_uint64 * (2 * (n1 + n2) * args.polls))()
used = ctypes.c_int64()
assert L.mac_diag_stamps(ctx._h, buf, len(buf), ctypes.byref(used)) == 0
st = np.frombuffer(buf, dtype=np.uint64).astype(np.int64).reshape(-1, 2)
res = []
for p in range(args.polls):
    a = st[p * (n1 + n2): p * (n1 + n2) + n1]
    b = st[p * (n1 + n2) + n1: (p + 1) * (n1 + n2)]
    t0 = a[:, 0].min()
    us = lambda v: float(v) / 100.0
    dur1 = (a[:, 1] - a[:, 0]) / 100.0
    dur2 = (b[:, 1] - b[:, 0]) / 100.0
    ends1 = np.sort(a[:, 1])
    res.append({
        "launch1_span": us(a[:, 1].max() - t0),
        "launch1_last_wg_extra": us(ends1[-1] - ends1[-2]),
        "chain_dur_med_max": [float(np.median(dur1[:n_chain])), float(dur1[:n_chain].max())],
        "tile_dur_med_max": [float(np.median(dur1[n_chain:])), float(dur1[n_chain:].max())],
        "launch1_start_pct": [us(np.percentile(a[:, 0] - t0, q)) for q in (50, 90, 100)],
        "launch1_end_pct_wo_last": [us(np.percentile(ends1[:-1] - t0, q)) for q in (50, 90, 100)],
        "gap": us(b[:, 0].min() - a[:, 1].max()),
        "launch2_span": us(b[:, 1].max() - b[:, 0].min()),
        "walk_dur_med_max": [float(np.median(dur2[:N])), float(dur2[:N].max())],
        "shared_dur_med_max": [float(np.median(dur2[N:])), float(dur2[N:].max())],
        "launch2_start_pct": [us(np.percentile(b[:, 0] - b[:, 0].min(), q)) for q in (50, 90, 100)],
        "launch2_last_wg_extra": us(np.sort(b[:, 1])[-1] - np.sort(b[:, 1])[-2]),
    })
L.mac_diag_walk_read.argtypes = [ctypes.POINTER(ctypes.c_uint64), ctypes.c_int64]
wb = (ctypes.c_uint64 * (8 * N))()
assert L.mac_diag_walk_read(wb, 8 * N) == 0
ws = np.frombuffer(wb, dtype=np.uint64).astype(np.int64).reshape(N, 8)[:, :7]
ok = np.all(ws[:, :7] > 0, axis=1)
ph = np.diff(ws[ok], axis=1) / 100.0
names = ["prologue+insert", "ids", "lane constants", "staging+tests (slice 0)", "atomics issue",
         "drain"]
walk = {n: [float(np.median(ph[:, q])), float(ph[:, q].max())] for q, n in enumerate(names)}
print(json.dumps({"config": args.config, "disks": args.disks, "polls": res[-2:],
                  "walk_phases_med_max_us": walk, "walk_disks_timed": int(ok.sum())}, indent=1))
