"""Diagnostic: per-workgroup timing of the poll walk (diagnostic build libmaxcover_diag.so).

MAXCOVER_LIB=.../libmaxcover_diag.so python tools/diag_poll.py [--config 4]
Stamps are s_memrealtime (100 MHz) per workgroup: start, end, (neighbours << 32 | entries), XCC.
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


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", type=int, default=4)
    args = ap.parse_args()
    pkg = ge.load_package()
    L = pkg.load_library()
    if not hasattr(L, "mac_diag_read"):
        raise SystemExit("not the diagnostic build (set MAXCOVER_LIB)")
    L.mac_diag_read.argtypes = [ctypes.POINTER(ctypes.c_uint64), ctypes.c_int64]
    x, y, w, C, rmax = pkg.workloads.make_config(args.config)
    ctx = pkg.Context(0, algo="poll")
    ctx.set_points(x, y, w)
    for _ in range(3):
        ctx.poll_best(C, rmax)
    N = C.shape[1] // 3
    K = C.shape[0]
    nwg = N * ((K + 2047) // 2048)  # kPollKPB = 2048 candidates per workgroup
    buf = (ctypes.c_uint64 * (4 * nwg))()
    assert L.mac_diag_read(buf, 4 * nwg) == 0
    a = np.frombuffer(buf, dtype=np.uint64).reshape(-1, 4).astype(np.int64)
    t0, t1 = a[:, 0], a[:, 1]
    dur = (t1 - t0) / 100.0  # us
    start = (t0 - t0.min()) / 100.0
    end = (t1 - t0.min()) / 100.0
    nc = a[:, 2] >> 32
    ent = a[:, 2] & 0xFFFFFFFF
    xcc = a[:, 3] & 0xF
    ks = np.arange(nwg) // N  # slice
    out = {
        "workgroups": int(nwg),
        "kernel_span_us": float(end.max()),
        "dur_us": {q: float(np.percentile(dur, q)) for q in (0, 10, 50, 90, 99, 100)},
        "start_us": {q: float(np.percentile(start, q)) for q in (0, 50, 90, 100)},
        "end_us": {q: float(np.percentile(end, q)) for q in (0, 50, 90, 100)},
        "entries": {q: float(np.percentile(ent, q)) for q in (0, 50, 100)},
        "nc>0": int((nc > 0).sum()),
        "dur_nc0_median": float(np.median(dur[nc == 0])),
        "dur_nc_pos_median": float(np.median(dur[nc > 0])) if (nc > 0).any() else None,
        "dur_by_slice_median": [float(np.median(dur[ks == s])) for s in range(ks.max() + 1)],
        "concurrency_avg": float(dur.sum() / end.max()),
        "slowest": [dict(wg=int(j), dur=float(dur[j]), nc=int(nc[j]), entries=int(ent[j]),
                         slice=int(ks[j]), xcc=int(xcc[j]), start=float(start[j]))
                    for j in np.argsort(-dur)[:8]],
    }
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
