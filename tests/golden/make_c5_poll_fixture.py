"""Regression fixture: the config-5 poll behind the bit-word kernel's 1.1-ms launch (r03 / r04
profiles: MPC step t = 3, iteration 94 of its MADS run, ell = 5, 192,317 fire entries). Written
from tools/c5_polls.py's gpurun_out/c5_slow.npz (slowest poll first):

  * the point list as 5-m cell indices (x = 5 i - 2.5, y = 5 j - 2.5, weight 25: the CA fire's
    points, src/DynamicArea.jl:100-108), int16, list order kept;
  * the poll's incumbent, the cons3 reference (prev) and r_max;
  * the LTMADS stream position: the candidates are [x + B^T; x - B^T] with
    B = workloads.ltmads_basis(n, ell, SplitMix64 at state seed + (it - 1) * (3n + n(n-1)/2)
    * 0x9E3779B97F4A7C15) — checked here against the saved candidate deltas.

No expected values are stored: tests/test_fire.py evaluates sampled candidates with the C oracle.

    python tests/golden/make_c5_poll_fixture.py [gpurun_out/c5_slow.npz]
"""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import __graft_entry__ as ge  # noqa: E402


def candidates(wl, xinc, seed, it, ell):
    n = xinc.size
    rng = wl.SplitMix64(seed)
    step = (3 * n + n * (n - 1) // 2) * 0x9E3779B97F4A7C15
    rng.state = np.uint64((seed + (it - 1) * step) & ((1 << 64) - 1))
    B = wl.ltmads_basis(n, ell, rng).astype(np.float64)
    return np.concatenate([xinc[None, :] + B.T, xinc[None, :] - B.T], axis=0)


def main(src):
    wl = ge.load_package().workloads
    d = np.load(src)
    rec = json.loads(str(d["rec0"]))
    t, poll, ell = rec["t"], rec["poll"], rec["ell"]
    it = poll - 100 * (t - 1) + 1
    seed = wl.SEED + t   # Simulation: seed + t per MPC step
    xinc = d["xinc0"]
    X = candidates(wl, xinc, seed, it, ell)
    assert np.array_equal(X, xinc[None, :] + d["delta0"]), "stream position does not reproduce the poll"
    x, y, w = d["x0"], d["y0"], d["w0"]
    ci, cj = (x + 2.5) / 5.0, (y + 2.5) / 5.0
    assert np.all(ci == np.round(ci)) and np.all(cj == np.round(cj)) and np.all(w == 25.0)
    out = os.path.join(ROOT, "tests", "golden", "c5_poll293.npz")
    np.savez_compressed(out, cells=np.stack([ci, cj], axis=1).astype(np.int16), xinc=xinc,
                        prev=d["prev0"], rmax=d["rmax0"],
                        meta=np.array([seed, it, ell, t, poll], dtype=np.int64))
    print(out, os.path.getsize(out), "bytes;", rec)


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else os.path.join(ROOT, "gpurun_out", "c5_slow.npz"))
