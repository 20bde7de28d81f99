"""Diagnostic: per-workgroup start / end of the prep launch (k_prep.h), config-4 poll
(ceil(K/8) workgroups); with the diagnostic build also the phases of the first 64.
python tools/diag_prep.py"""
import ctypes, json, os, sys
import numpy as np
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import __graft_entry__ as ge  # noqa: E402

pkg = ge.load_package()
L = pkg.load_library()
L.mac_diag_stamps.argtypes = [ctypes.c_void_p, ctypes.POINTER(ctypes.c_uint64), ctypes.c_int64,
                              ctypes.POINTER(ctypes.c_int64)]
x, y, w, C, rmax = pkg.workloads.make_config(4)
ctx = pkg.Context(0, algo=sys.argv[1] if len(sys.argv) > 1 else "auto")
ctx.set_points(x, y, w)
for _ in range(3):
    ctx.poll_best(C, rmax)
ctx.profile(True)
out = {}
for rep in range(3):
    ctx.profile_read(reset=True)
    ctx.poll_best(C, rmax)
    K, n3 = C.shape[0], C.shape[1]
    cap = 2 * K
    buf = (ctypes.c_uint64 * cap)()
    used = ctypes.c_int64()
    assert L.mac_diag_stamps(ctx._h, buf, cap, ctypes.byref(used)) == 0
    # the prep launch's workgroups: prep_x_kernel (K // 6 of them) for a matrix source
    nchain = K // 6 if K // 6 >= K - 6 * (K // 6) else (K + 7) // 8
    nwg = nchain
    a = np.frombuffer(buf, dtype=np.uint64)[:2 * nwg].reshape(nwg, 2).astype(np.int64)
    base = a[:, 0].min()
    s = (a[:, 0] - base) / 100.0
    e = (a[:, 1] - base) / 100.0
    d = e - s
    out[rep] = {"span_us": float(e.max()),
                "chain": {"n": nchain, "start_max": float(s[:nchain].max()),
                          "dur_median": float(np.median(d[:nchain])), "dur_max": float(d[:nchain].max()),
                          "end_max": float(e[:nchain].max()),
                          "end_p50": float(np.median(e[:nchain]))}}
if hasattr(L, "mac_diag_prep_read"):
    L.mac_diag_prep_read.argtypes = [ctypes.POINTER(ctypes.c_uint64), ctypes.c_int64]
    b2 = (ctypes.c_uint64 * (64 * 16))()
    assert L.mac_diag_prep_read(b2, 64 * 16) == 0
    p = np.frombuffer(b2, dtype=np.uint64).reshape(64, 16).astype(np.int64)
    nb = (C.shape[1] // 3 + 511) // 512
    cols = 1 + 3 * nb
    ph = np.diff(p[:, :cols], axis=1) / 100.0
    out["chain_phases_us_median"] = [float(v) for v in np.median(ph, axis=0)]
    out["chain_phases_us_max"] = [float(v) for v in ph.max(axis=0)]
    out["chain_phase_names"] = "per block: loads+terms (wave 0), barrier (wave 0), fold after the barrier (the folding wave)"
print(json.dumps(out, indent=1))
