"""Config 1 (BASELINE.json configs[0]): 5 UAVs on the FirePoints table through the MPC loop's
optimisation side (src/FullSimulation.jl:42-100), three timesteps.

Reference side, replayed with the oracle only: the list starts as FirePoints rows 1..10
(src/CellFunctions.jl:35-49), row t+10 is appended for t != 1 (:59-79; row 11 is never read),
the entries the previous circles cover are deleted in order (rmvCoveredPOI :81-108 ->
ref_remove_covered), and the MADS run is the Python driver TDM_STATIC_opt.mads over the C
oracle's objective (src/TDM_STATIC_opt.jl:82-100) with cons1 / cons3 per trial point. The
library side is FullSimulation.Simulation: the device list (mac_append_points_f64,
mac_remove_covered_f64) and the native MADS loop (mac_mads_run)."""
import math

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

FOV = 100 / 180 * math.pi


def test_config1_firepoints_mpc_steps(ctx, pkg, orc, firepoints):
    FS = pkg.FullSimulation
    TS = pkg.TDM_STATIC_opt
    TC = pkg.TDM_Constraints
    N, N_iter, seed = 5, 30, 20250216
    x0 = np.round(pkg.Base_Functions.allocate_even_circles(15.0, N, 10 * math.tan(FOV / 2),
                                                           250.0, 250.0))
    sim = FS.Simulation(ctx, x0, firepoints=firepoints, N_iter=N_iter, seed=seed)

    rec = np.concatenate([np.asarray(r).reshape(-1, 5) for r in firepoints[:10]])
    assert rec.shape[0] == 455                    # rows 1..10
    x_prev = x0.copy()
    r_max = np.full(N, 30.0 * math.tan(FOV / 2))
    d_lim = np.full(N, 10.0)
    outputs = []
    moved = False
    for t in (1, 2, 3):
        got = sim.step()
        # -- the reference's list for step t, replayed on the host
        if t != 1 and t + 10 - 1 < len(firepoints):
            rec = np.concatenate([rec, np.asarray(firepoints[t + 10 - 1]).reshape(-1, 5)])
        drone_locs = x_prev.copy()
        rec = rec[orc.ref_remove_covered(drone_locs, rec)]
        gx, gy, gw = ctx.get_points()
        assert np.array_equal(gx, rec[:, 0]) and np.array_equal(gy, rec[:, 1])
        assert np.array_equal(gw, rec[:, 3])      # the weight is column 4 (:72)
        assert got["points"] == rec.shape[0]
        # -- the reference's MADS input and run for step t
        if t != 1:
            FS.r_max_update(drone_locs, r_max, N)
        single_input = drone_locs if t < 3 else outputs[-1]
        if t >= 3 and not FS.cons3_ok(x_prev, single_input, d_lim):
            single_input = drone_locs
        assert np.array_equal(got["input"], single_input)
        c3 = TC.create_cons3(x_prev, FOV, d_lim)
        rr = r_max.copy()

        def oracle_objective(v, rec=rec, rr=rr):
            return orc.ref_objective(v, rec, rr, 1e5)

        res = TS.mads(single_input, oracle_objective, [TC.cons1, c3], N_iter=N_iter, ell0=2,
                      ell_max=6, seed=seed + t)
        want = res.x if res.x is not None else res.i
        assert np.array_equal(sim.outputs[-1], want), t
        assert got["f"] == res.x_cost, t
        assert got["iterations"] == res.status.iteration, t
        moved |= not np.array_equal(want, single_input)
        outputs.append(want)
        x_prev = want
    assert moved
