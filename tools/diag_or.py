"""Diagnostic: per-workgroup phase times of shared_or_kernel (diagnostic build only) on the config-5
regression poll (tests/golden/c5_poll293.npz, ell = 5) and on the same stream position at ell = 4
and 3 (the common crowded polls).
MAXCOVER_LIB=.../libmaxcover_diag.so python tools/diag_or.py"""
import ctypes, importlib.util, json, os, sys
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import __graft_entry__ as ge  # noqa: E402

pkg = ge.load_package()
L = pkg.load_library()
L.mac_diag_or_read.argtypes = [ctypes.POINTER(ctypes.c_uint64), ctypes.c_int64]
spec = importlib.util.spec_from_file_location("mk", os.path.join(ROOT, "tests", "golden", "make_c5_poll_fixture.py"))
mk = importlib.util.module_from_spec(spec)
spec.loader.exec_module(mk)
d = np.load(os.path.join(ROOT, "tests", "golden", "c5_poll293.npz"))
seed, it, ell0 = (int(v) for v in d["meta"][:3])
cells = d["cells"].astype(np.float64)
x, y = cells[:, 0] * 5.0 - 2.5, cells[:, 1] * 5.0 - 2.5
w = np.full(x.size, 25.0)
ctx = pkg.Context(0, algo="poll")   # (AUTO may pick the per-candidate walk at ell = 5)
ctx.set_points(x, y, w)
ctx.set_shared("bits")
names = ["setup", "stage", "tables", "combine", "next"]
for ell in (5, 4, 3):
    X = mk.candidates(pkg.workloads, d["xinc"], seed, it, ell)
    for _ in range(3):
        ctx.profile(True)
        ctx.profile_read(reset=True)
        ctx.poll_best(X, d["rmax"], 1e5)
        k = ctx.profile_kernels()
        ctx.profile_read(reset=True)
    buf = (ctypes.c_uint64 * (1024 * 16))()
    assert L.mac_diag_or_read(buf, 1024 * 16) == 0
    a = np.frombuffer(buf, dtype=np.uint64).reshape(1024, 16).astype(np.int64)
    a = a[a[:, 12] > 0]
    t = a[:, :5] / 100.0
    print(json.dumps({
        "ell": ell, "kernels_us": {n: round(ms / c * 1e3, 1) for n, (ms, c) in k.items() if c},
        "wgs": int(a.shape[0]),
        "wg_total_us": {"median": float(np.median(a[:, 12] / 100.0)), "max": float(a[:, 12].max() / 100.0)},
        "phase_us_median": dict(zip(names, [round(float(v), 1) for v in np.median(t, axis=0)])),
        "phase_us_max": dict(zip(names, [round(float(v), 1) for v in t.max(axis=0)])),
        "jobs_total": int(a[:, 8].sum()), "disks_total": int(a[:, 9].sum()),
        "positions_total": int(a[:, 10].sum()), "live_total": int(a[:, 11].sum())}), flush=True)
ctx.close()
