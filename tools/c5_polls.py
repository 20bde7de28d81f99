"""Diagnostic: per-poll kernel times of the config-5 MPC loop (the bench's sequence), to find the
polls behind the bit-word kernel's slow launches and save them for offline analysis / tests.

The native loop (mac_mads_run) is replaced by the host mirror of its stepper (TDM_STATIC_opt.
PollStepper: the same LTMADS stream and update rule, bit for bit) evaluating each poll's K x 3N
matrix with Context.poll_best, so every poll is one profiled chain. Writes gpurun_out/c5_polls.json
(per poll: kernel us, dc) and gpurun_out/c5_slow.npz (the slowest polls' candidates, cons3 inputs
and the point list they ran on).

    python tools/c5_polls.py [--steps 4] [--keep 3]
"""
import argparse
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import __graft_entry__ as ge  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--steps", type=int, default=4, help="MPC steps (bench: 1 warmup + 3 timed)")
ap.add_argument("--keep", type=int, default=3)
ap.add_argument("--seed", type=int, default=20250216)
args = ap.parse_args()

pkg = ge.load_package()
wl = pkg.workloads
TS = pkg.TDM_STATIC_opt
cfg = wl.CONFIGS[5]
rng = wl.SplitMix64(args.seed)
fire_kw, x0 = wl.config5_setup(rng, cfg["G"], cfg["N"], cfg["ignition"])
ctx = pkg.Context(0, algo="auto")
D = pkg.DynamicArea.DynamicArea(**fire_kw, seed=args.seed, device=0)
sim = pkg.FullSimulation.Simulation(ctx, x0, fire=D, N_iter=100, seed=args.seed)
N = cfg["N"]
polls = []
slow = []   # (bits us, record, X, prev, points)


def mads_host(x_in, r_max, penalty, prev, d_lim, tan_half_fov, n_iter, ell0, ell_max, seed):
    """mac_mads_run through the host stepper: one profiled poll_best chain per iteration."""
    f0 = ctx.poll_best(np.asarray(x_in)[None, :], r_max, penalty, prev=prev, d_lim=d_lim,
                       tan_half_fov=tan_half_fov)[0]
    pts = None

    def poll_fn(X):
        nonlocal pts
        ctx.profile(True)
        ctx.profile_read(reset=True)
        bo, bi = ctx.poll_best(X, r_max, penalty, prev=prev, d_lim=d_lim, tan_half_fov=tan_half_fov)
        k = ctx.profile_kernels()
        ctx.profile_read(reset=True)
        rec = {"t": sim.t, "poll": len(polls), "ell": st.ell,
               **{name: (ms / n * 1e3 if n else None) for name, (ms, n) in k.items()}}
        polls.append(rec)
        b = rec["shared_or_kernel"] or 0.0
        if len(slow) < args.keep or b > min(s[0] for s in slow):
            if pts is None:
                pts = ctx.get_points()
            slow.append((b, rec, X.copy(), prev.copy(), pts))
            slow.sort(key=lambda s: -s[0])
            del slow[args.keep:]
        return bo, bi

    st = TS.PollStepper(x_in, f0, poll_fn, N_iter=n_iter, ell0=ell0, ell_max=ell_max, seed=seed)
    while True:
        done, bo, bi = st.poll()
        if done:
            break
        st.update(bo, bi)
    x, info = st.result()
    return x, {"f": info["f"], "iterations": info["iterations"], "evaluations": info["evaluations"]}


ctx.mads_run = mads_host
for _ in range(args.steps):
    r = sim.step()
    print(json.dumps({k: r[k] for k in ("t", "points", "f", "iterations")}), flush=True)
ctx.profile(False)
os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
with open(os.path.join(ROOT, "gpurun_out", "c5_polls.json"), "w") as f:
    json.dump(polls, f)
b = np.array([p["shared_or_kernel"] or 0.0 for p in polls])
print(json.dumps({"polls": len(polls), "bits_us_mean": float(b.mean()), "bits_us_max": float(b.max()),
                  "bits_us_p50": float(np.median(b)), "slowest": [s[1] for s in slow]}), flush=True)
save = {}
for q, (bu, rec, X, prev, (x, y, w)) in enumerate(slow):
    n = X.shape[1]
    xc = X[0] - (X[0] - X[n]) / 2            # the incumbent: X = [x + B^T; x - B^T]
    dd = X - xc[None, :]
    assert np.all(np.abs(dd) < 128) and np.array_equal(xc[None, :] + dd.astype(np.int8), X)
    save.update({f"xinc{q}": xc, f"delta{q}": dd.astype(np.int8), f"prev{q}": prev, f"x{q}": x,
                 f"y{q}": y, f"w{q}": w, f"rec{q}": json.dumps(rec), f"rmax{q}": sim.r_max.copy()})
np.savez_compressed(os.path.join(ROOT, "gpurun_out", "c5_slow.npz"), **save)
D.close()
ctx.close()
