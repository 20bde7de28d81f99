"""The config-5 regression poll (tests/golden/c5_poll293.npz) and the same stream position at
smaller mesh steps through each walk: per-kernel device times (in-kernel stamps) of the poll walk
+ shared-entry pass against the per-candidate walk, and that both give the same objectives.
python tools/c5_walks.py"""
import importlib.util, json, os, sys
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import __graft_entry__ as ge  # noqa: E402

pkg = ge.load_package()
spec = importlib.util.spec_from_file_location("mk", os.path.join(ROOT, "tests", "golden", "make_c5_poll_fixture.py"))
mk = importlib.util.module_from_spec(spec)
spec.loader.exec_module(mk)
d = np.load(os.path.join(ROOT, "tests", "golden", "c5_poll293.npz"))
seed, it, ell0 = (int(v) for v in d["meta"][:3])
cells = d["cells"].astype(np.float64)
x, y = cells[:, 0] * 5.0 - 2.5, cells[:, 1] * 5.0 - 2.5
w = np.full(x.size, 25.0)
ctx = pkg.Context(0)
ctx.set_points(x, y, w)
for ell in (5, 4, 3, 2, 1):
    X = mk.candidates(pkg.workloads, d["xinc"], seed, it, ell)
    row = {"ell": ell}
    ref = None
    for algo in ("poll", "tiled", "auto"):
        ctx.set_algo(algo)
        for _ in range(4):
            ctx.profile(True)
            ctx.profile_read(reset=True)
            bo, bi, objs = ctx.poll_best(X, d["rmax"], 1e5, want_all=True)
            k = ctx.profile_kernels()
            ctx.profile_read(reset=True)
        if ref is None:
            ref = objs
        us = {n: round(ms / c * 1e3, 1) for n, (ms, c) in k.items() if c}
        row[algo] = {"sum_us": round(sum(us.values()), 1), "kernels_us": us,
                     "same_objs": bool(np.array_equal(objs, ref))}
    # as the MPC loop runs it: cons3 against the step's start (failing candidates not evaluated)
    ctx.set_algo("auto")
    dl = np.full(X.shape[1] // 3, 10.0)
    tan50 = float(np.tan(100 / 180 * np.pi / 2))
    for _ in range(4):
        ctx.profile(True)
        ctx.profile_read(reset=True)
        bo, bi, objs3 = ctx.poll_best(X, d["rmax"], 1e5, prev=d["prev"], d_lim=dl, tan_half_fov=tan50,
                                      want_all=True)
        k = ctx.profile_kernels()
        ctx.profile_read(reset=True)
    us = {n: round(ms / c * 1e3, 1) for n, (ms, c) in k.items() if c}
    row["auto_cons3"] = {"sum_us": round(sum(us.values()), 1), "kernels_us": us,
                         "feasible": int(np.isfinite(objs3).sum()),
                         "same_where_feasible": bool(np.array_equal(objs3[np.isfinite(objs3)],
                                                                    ref[np.isfinite(objs3)]))}
    print(json.dumps(row), flush=True)
ctx.profile(False)
ctx.close()
