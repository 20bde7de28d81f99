"""Diagnostic: where the per-poll host time goes (config 4 by default).

  enqueue   : mean wall time of one mac_poll_best_dev_f64 call (returns after enqueueing)
  sync_step : one poll + 16-B D2H + stream sync, as bench.py's step
  pipelined : 20 polls enqueued back to back, one sync (GPU-bound rate)
  raw_ctypes: the same step calling the ctypes function with prebuilt arguments
"""
import argparse
import ctypes
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import __graft_entry__ as ge  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", type=int, default=4)
    ap.add_argument("--reps", type=int, default=50)
    a = ap.parse_args()
    import torch
    pkg = ge.load_package()
    x, y, w, C, rmax = pkg.workloads.make_config(a.config)
    N = C.shape[1] // 3
    K = C.shape[0]
    dev = torch.device("cuda", 0)
    ctx = pkg.Context(0)
    ctx.set_points(x, y, w)
    dC = torch.from_numpy(np.ascontiguousarray(C)).to(dev)
    dR = torch.from_numpy(rmax).to(dev)
    dB = torch.empty(2, dtype=torch.float64, device=dev)
    hB = torch.empty(2, dtype=torch.float64).pin_memory()
    st = torch.cuda.Stream(dev)
    sp = st.cuda_stream
    for _ in range(5):
        ctx.poll_best_dev(dC, 3 * N, K, dR, dB, stream=sp)
    st.synchronize()

    t = []
    for _ in range(a.reps):
        t0 = time.perf_counter()
        ctx.poll_best_dev(dC, 3 * N, K, dR, dB, stream=sp)
        t.append(time.perf_counter() - t0)
        st.synchronize()
    enqueue = float(np.median(t)) * 1e6

    t = []
    for _ in range(a.reps):
        t0 = time.perf_counter()
        with torch.cuda.stream(st):
            ctx.poll_best_dev(dC, 3 * N, K, dR, dB, stream=sp)
            hB.copy_(dB, non_blocking=True)
        st.synchronize()
        _ = float(hB[0])
        t.append(time.perf_counter() - t0)
    sync_step = float(np.median(t)) * 1e6

    st.synchronize()
    t0 = time.perf_counter()
    for _ in range(20):
        ctx.poll_best_dev(dC, 3 * N, K, dR, dB, stream=sp)
    st.synchronize()
    pipelined = (time.perf_counter() - t0) / 20 * 1e6

    L = ctx._L
    fn = L.mac_poll_best_dev_f64
    args = (ctx._h, ctypes.c_void_p(dC.data_ptr()), ctypes.c_int64(3 * N), ctypes.c_int64(K),
            ctypes.c_void_p(dR.data_ptr()), ctypes.c_double(1e5), None, None, ctypes.c_double(1.0),
            ctypes.c_int64(0), None, ctypes.c_void_p(dB.data_ptr()), ctypes.c_void_p(sp))
    hb = np.zeros(2)
    hbp = hb.ctypes.data
    hip = ctypes.CDLL("libamdhip64.so")
    hip.hipMemcpyAsync.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int,
                                   ctypes.c_void_p]
    hip.hipStreamSynchronize.argtypes = [ctypes.c_void_p]
    t = []
    for _ in range(a.reps):
        t0 = time.perf_counter()
        fn(*args)
        hip.hipMemcpyAsync(hbp, dB.data_ptr(), 16, 2, sp)
        hip.hipStreamSynchronize(sp)
        t.append(time.perf_counter() - t0)
    raw = float(np.median(t)) * 1e6
    print(json.dumps({"config": a.config, "enqueue_us": enqueue, "sync_step_us": sync_step,
                      "pipelined_us": pipelined, "raw_ctypes_step_us": raw}))


if __name__ == "__main__":
    main()
