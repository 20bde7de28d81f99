"""Diagnostic: what exact per-poll routing between the poll chains could save on config 5. The
config-5 MPC loop's polls (the bench's sequence, through the host mirror of the native stepper:
TDM_STATIC_opt.PollStepper, bit for bit) are each evaluated through BOTH forced chains (the fused
three-launch chain and the five-launch chain with the union pass), and the device chain of each
(in-kernel stamps, first workgroup start to last workgroup end) is recorded with the poll's mesh
index, so the sum over polls of min(fused, five) — an oracle router — can be set against the
five-launch sum (what AUTO's history routes config 5 to). Writes gpurun_out/c5_route.json.

    python tools/c5_route.py [--steps 2]
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
ap.add_argument("--steps", type=int, default=2)
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
polls = []


def chain_us(fn):
    ctx.profile(True)
    ctx.profile_read(reset=True)
    r = fn()
    p1, p2, gap, n = ctx.profile_split()
    k = {name: (ms / c * 1e3) for name, (ms, c) in ctx.profile_kernels().items() if c}
    ctx.profile_read(reset=True)
    ctx.profile(False)
    return r, ((p1 + p2 + gap) / n * 1e3 if n else None), k


def mads_host(x_in, r_max, penalty, prev, d_lim, tan_half_fov, n_iter, ell0, ell_max, seed):
    f0 = ctx.poll_best(np.asarray(x_in)[None, :], r_max, penalty, prev=prev, d_lim=d_lim,
                       tan_half_fov=tan_half_fov)[0]

    def poll_fn(X):
        rec = {"t": sim.t, "poll": len(polls), "ell": st.ell}
        out = {}
        for ch in ("five", "fused"):
            ctx.set_chain(ch)
            # twice: the second run is timed (the first settles the lane's launch hints)
            ctx.poll_best(X, r_max, penalty, prev=prev, d_lim=d_lim, tan_half_fov=tan_half_fov)
            res, us, k = chain_us(lambda: ctx.poll_best(X, r_max, penalty, prev=prev, d_lim=d_lim,
                                                        tan_half_fov=tan_half_fov))
            out[ch] = res
            rec[ch + "_us"] = us
            rec[ch + "_kernels"] = k
        ctx.set_chain("auto")
        assert out["five"] == out["fused"], (out, rec)
        polls.append(rec)
        return out["five"]

    st = TS.PollStepper(x_in, f0, poll_fn, N_iter=n_iter, ell0=ell0, ell_max=ell_max, seed=seed)
    while True:
        done, bo, bi = st.poll()
        if done:
            break
        st.update(bo, bi)
    x, info = st.result()
    return x, {"f": info["f"], "iterations": info["iterations"], "evaluations": info["evaluations"]}


ctx.mads_run = mads_host
for s in range(args.steps):
    sim.step()
    print(f"step {s + 1}: {len(polls)} polls", flush=True)
five = np.array([p["five_us"] or 0.0 for p in polls])
fused = np.array([p["fused_us"] or 0.0 for p in polls])
ells = np.array([p["ell"] for p in polls])
summary = {
    "polls": len(polls),
    "five_sum_ms": float(five.sum() / 1e3), "fused_sum_ms": float(fused.sum() / 1e3),
    "oracle_min_sum_ms": float(np.minimum(five, fused).sum() / 1e3),
    "fused_faster": int((fused < five).sum()),
    "by_ell": {int(e): {"polls": int((ells == e).sum()),
                        "five_us_mean": float(five[ells == e].mean()),
                        "fused_us_mean": float(fused[ells == e].mean()),
                        "fused_faster": int((fused[ells == e] < five[ells == e]).sum())}
               for e in sorted(set(ells.tolist()))},
}
print(json.dumps(summary, indent=1))
os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
json.dump({"summary": summary, "polls": polls}, open(os.path.join(ROOT, "gpurun_out", "c5_route.json"), "w"))
