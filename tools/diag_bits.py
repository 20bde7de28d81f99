"""Diagnostic: per-workgroup phase times of shared_bits_kernel (diagnostic build only).
MAXCOVER_LIB=.../libmaxcover_diag.so python tools/diag_bits.py [--config 4|5] [--disks clustered]"""
import argparse, ctypes, json, os, sys
import numpy as np
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import __graft_entry__ as ge  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--disks", default="clustered")
ap.add_argument("--config", type=int, default=4)
args = ap.parse_args()
pkg = ge.load_package()
L = pkg.load_library()
L.mac_diag_bits_read.argtypes = [ctypes.POINTER(ctypes.c_uint64), ctypes.c_int64]
if args.config == 5:
    # the last bit-word launch of two config-5 MPC steps (LTMADS polls generated on the device)
    wl = pkg.workloads
    rng = wl.SplitMix64(wl.SEED)
    cfg = wl.CONFIGS[5]
    fire_kw, x0 = wl.config5_setup(rng, cfg["G"], cfg["N"], cfg["ignition"])
    ctx = pkg.Context(0, algo="auto")
    D = pkg.DynamicArea.DynamicArea(**fire_kw, seed=wl.SEED, device=0)
    sim = pkg.FullSimulation.Simulation(ctx, x0, fire=D, N_iter=100, seed=wl.SEED)
    for _ in range(2):
        sim.step()
else:
    x, y, w, C, rmax = pkg.workloads.make_config(4, disks=args.disks)
    ctx = pkg.Context(0, algo="auto")
    ctx.set_points(x, y, w)
    for _ in range(3):
        ctx.poll_best(C, rmax)
buf = (ctypes.c_uint64 * (256 * 16))()
assert L.mac_diag_bits_read(buf, 256 * 16) == 0
a = np.frombuffer(buf, dtype=np.uint64).reshape(256, 16).astype(np.int64)
names = ["setup+runs", "entries+group", "staging", "tables", "combine", "write+next"]
t = a[:, :6] / 100.0
print(json.dumps({
    "wg_total_us": {"median": float(np.median(a[:, 12] / 100.0)), "max": float(a[:, 12].max() / 100.0)},
    "phase_us_sum_median": dict(zip(names, [float(v) for v in np.median(t, axis=0)])),
    "phase_us_sum_max": dict(zip(names, [float(v) for v in t.max(axis=0)])),
    "per_wg_median": {"jobs": float(np.median(a[:, 8])), "passes": float(np.median(a[:, 9])),
                      "groups": float(np.median(a[:, 10])), "blocks": float(np.median(a[:, 11]))},
    "totals": {"jobs": int(a[:, 8].sum()), "passes": int(a[:, 9].sum()), "groups": int(a[:, 10].sum()),
               "blocks": int(a[:, 11].sum())},
}, indent=1))
