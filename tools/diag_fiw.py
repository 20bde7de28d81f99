"""Diagnostic: per-disk phase times of the fused kernel fiw_kernel (k_fiw.h), diagnostic build only
(libmaxcover_diag.so; never quote its timings as kernel performance).

MAXCOVER_LIB=.../libmaxcover_diag.so python tools/diag_fiw.py [--config 4] [--disks uniform]
"""
import argparse
import ctypes
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import __graft_entry__ as ge  # noqa: E402

NAMES = ["loads", "neighbours+hash+number", "positions", "walk", "shared", "row write"]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", type=int, default=4)
    ap.add_argument("--disks", default="uniform")
    args = ap.parse_args()
    pkg = ge.load_package()
    L = pkg.load_library()
    if not hasattr(L, "mac_diag_fiw_read"):
        raise SystemExit("not the diagnostic build (set MAXCOVER_LIB)")
    L.mac_diag_fiw_read.argtypes = [ctypes.POINTER(ctypes.c_uint64), ctypes.c_int64]
    x, y, w, C, rmax = pkg.workloads.make_config(args.config, disks=args.disks)
    ctx = pkg.Context(0)
    ctx.set_chain("fused")
    ctx.set_points(x, y, w)
    tan = float(np.tan(100 / 180 * np.pi / 2))
    N = C.shape[1] // 3
    for _ in range(4):
        ctx.poll_best(C, rmax, 1e5, prev=C[0], d_lim=np.full(N, 10.0), tan_half_fov=tan)
    buf = (ctypes.c_uint64 * (16 * N))()
    assert L.mac_diag_fiw_read(buf, 16 * N) == 0
    a = np.frombuffer(buf, dtype=np.uint64).reshape(N, 16)
    info = a[:, 7]
    t = a[:, :7].astype(np.int64)
    # the walk's first slice / chunk: lane constants, staging + compaction, hot loop, band + rest
    wk = np.concatenate([a[:, 3:4], a[:, 8:12], a[:, 4:5]], axis=1).astype(np.int64)
    ok = (t > 0).all(axis=1)
    t = t[ok]
    ph = np.diff(t, axis=1) / 100.0
    out = {"disks": int(ok.sum()), "names": NAMES,
           "median_us": [round(float(v), 2) for v in np.median(ph, axis=0)],
           "max_us": [round(float(v), 2) for v in ph.max(axis=0)],
           "total_median_us": float(np.median((t[:, 6] - t[:, 0]) / 100.0)),
           "span_us": float((t[:, 6].max() - t[:, 0].min()) / 100.0),
           "start_spread_us": float((t[:, 0].max() - t[:, 0].min()) / 100.0),
           "positions_median": float(np.median((info[ok] >> 32).astype(np.int64))),
           "neighbours_max": int(((info[ok] >> 16) & 0xFFFF).max()),
           "disks_with_neighbours": int((((info[ok] >> 16) & 0xFFFF) > 0).sum()),
           "box_tiles_median": float(np.median((info[ok] & 0xFFFF).astype(np.int64)))}
    hk = np.concatenate([a[:, 1:2], a[:, 12:13], a[:, 15:16], a[:, 13:15], a[:, 2:3]], axis=1).astype(np.int64)[ok]
    hok = (hk > 0).all(axis=1)
    if hok.any():
        hp = np.diff(hk[hok], axis=1) / 100.0
        out["index_split"] = {"names": ["bound+box+neighbours", "table clear+barrier", "mark",
                                        "miss vote", "numbering"],
                              "median_us": [round(float(v), 2) for v in np.median(hp, axis=0)],
                              "max_us": [round(float(v), 2) for v in hp.max(axis=0)]}
    wk = wk[ok]
    wok = (wk > 0).all(axis=1)
    if wok.any():
        wp = np.diff(wk[wok], axis=1) / 100.0
        out["walk_split"] = {"names": ["lane constants", "staging+compaction", "hot loop",
                                       "band+sync", "rest (more chunks, credit write)"],
                             "median_us": [round(float(v), 2) for v in np.median(wp, axis=0)],
                             "max_us": [round(float(v), 2) for v in wp.max(axis=0)],
                             "disks": int(wok.sum())}
    slow = np.argsort(-(t[:, 6] - t[:, 0]))[:5]
    out["slowest"] = [{"total_us": float((t[q, 6] - t[q, 0]) / 100.0),
                       "phases_us": [round(float(v), 2) for v in ph[q]],
                       "nc": int((info[ok][q] >> 16) & 0xFFFF)} for q in slow]
    # fin2: per block {start, rows, list, records+entries, decisions, reduction, end}, last-block flag
    L.mac_diag_f2_read.argtypes = [ctypes.POINTER(ctypes.c_uint64), ctypes.c_int64]
    nb = 4096
    fb = (ctypes.c_uint64 * (8 * nb))()
    assert L.mac_diag_f2_read(fb, 8 * nb) == 0
    f = np.frombuffer(fb, dtype=np.uint64).reshape(nb, 8).astype(np.int64)
    f = f[(f[:, 0] > 0) & (f[:, 6] >= f[:, 0])]
    f = f[f[:, 0] >= t[:, 0].min()]   # this run's blocks
    if len(f):
        g = np.maximum.accumulate(np.where(f[:, :7] > 0, f[:, :7], 0), axis=1)
        ph2 = np.diff(g, axis=1) / 100.0
        last = f[:, 7] == 1
        out["fin2"] = {"blocks": int(len(f)),
                       "names": ["rows", "list", "records+entries", "decisions", "reduction", "argmin"],
                       "median_us": [round(float(v), 2) for v in np.median(ph2, axis=0)],
                       "max_us": [round(float(v), 2) for v in ph2.max(axis=0)],
                       "last_block_us": [round(float(v), 2) for v in ph2[last][0]] if last.any() else None,
                       "gap_fiw_end_to_first_start_us": float((f[:, 0].min() - t[:, 6].max()) / 100.0),
                       "start_spread_us": float((f[:, 0].max() - f[:, 0].min()) / 100.0),
                       "span_us": float((f[:, 6].max() - f[:, 0].min()) / 100.0)}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
