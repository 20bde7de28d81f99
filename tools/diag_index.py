"""Diagnostic: per-disk phase times of disk_index_kernel (diagnostic build only).
MAXCOVER_LIB=.../libmaxcover_diag.so python tools/diag_index.py"""
import ctypes, json, os, sys
import numpy as np
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import __graft_entry__ as ge  # noqa: E402

pkg = ge.load_package()
L = pkg.load_library()
L.mac_diag_index_read.argtypes = [ctypes.POINTER(ctypes.c_uint64), ctypes.c_int64]
if "--config" in sys.argv and sys.argv[sys.argv.index("--config") + 1] == "5":
    # the last index launch of two config-5 MPC steps (LTMADS polls generated on the device)
    wl = pkg.workloads
    rng = wl.SplitMix64(wl.SEED)
    cfg = wl.CONFIGS[5]
    fire_kw, x0 = wl.config5_setup(rng, cfg["G"], cfg["N"], cfg["ignition"])
    ctx = pkg.Context(0, algo="poll")
    D = pkg.DynamicArea.DynamicArea(**fire_kw, seed=wl.SEED, device=0)
    sim = pkg.FullSimulation.Simulation(ctx, x0, fire=D, N_iter=100, seed=wl.SEED)
    for _ in range(2):
        sim.step()
    N = x0.size // 3
else:
    x, y, w, C, rmax = pkg.workloads.make_config(4)
    ctx = pkg.Context(0, algo="poll")
    ctx.set_points(x, y, w)
    for _ in range(3):
        ctx.poll_best(C, rmax)
    N = C.shape[1] // 3
buf = (ctypes.c_uint64 * (8 * N))()
assert L.mac_diag_index_read(buf, 8 * N) == 0
a = np.frombuffer(buf, dtype=np.uint64).reshape(N, 8).astype(np.int64)[:, :6]
base = a[:, 0].min()
ph = np.diff(a, axis=1) / 100.0
print(json.dumps({"span_us": float((a[:, 5].max() - base) / 100.0),
                  "phase_us_median": [float(v) for v in np.median(ph, axis=0)],
                  "phase_us_max": [float(v) for v in ph.max(axis=0)],
                  "start_us": {q: float(np.percentile((a[:, 0] - base) / 100.0, q)) for q in (0, 50, 100)},
                  "names": ["loads", "hash insert", "number+records", "map+pen+spans", "reduce"]}))
