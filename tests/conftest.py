"""Shared fixtures. `-m "not gpu"` runs here (no GPU); `-m gpu` runs on an MI355X box."""
import math
import os
import sys

import numpy as np
import pytest
# torch before libmaxcover: one HIP runtime per process (the GPU tests mix torch tensors and
# streams with the library's launches; _lib.check_one_runtime)
import torch  # noqa: F401,E402

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

import __graft_entry__ as ge  # noqa: E402


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through libmaxcover on HIP)")


@pytest.fixture(scope="session")
def pkg():
    return ge.load_package()


@pytest.fixture(scope="session")
def orc():
    return ge.load_oracle()


@pytest.fixture(scope="session")
def golden():
    with np.load(os.path.join(ROOT, "tests", "golden", "golden.npz"), allow_pickle=False) as z:
        return {k: z[k] for k in z.files}


@pytest.fixture(scope="session")
def firepoints(pkg):
    return pkg.workloads.load_firepoints(os.path.join(ROOT, "tests", "golden", "firepoints.csv"))


@pytest.fixture(scope="session")
def ctx(pkg):
    """One GPU context for the whole GPU session (tests reset the point list themselves)."""
    if pkg.device_count() < 1:
        pytest.fail("no HIP device visible: GPU tests must run on the MI355X box")
    c = pkg.Context(0)
    yield c
    c.close()


def _quadrotor_run():
    path = os.path.join(ROOT, "tests", "golden", "quadrotor_run.csv")
    return np.loadtxt(path, delimiter=",", comments="#")


@pytest.fixture(scope="session")
def quadrotor_steps(pkg):
    """(prev, target) per MPC step of the reference's static N = 5 run for UAV 1, as [x; y; R]
    (N = 1): prev = where the step's MADS started (the initial ring for step 1,
    src/FullSimulation.jl:803; else the previous step's end state, R = z tan(FOV/2), :238-251);
    target = the MADS output the reference recorded (z back to R = z tan(FOV/2))."""
    D = _quadrotor_run()
    tan = math.tan(100 / 180 * math.pi / 2)
    x0 = pkg.Base_Functions.allocate_even_circles(15.0, 5, 10 * tan, 250.0, 250.0)
    out = []
    for t in range(D.shape[0]):
        prev = (np.array([x0[0], x0[5], x0[10]]) if t == 0
                else np.array([D[t - 1, 3], D[t - 1, 4], D[t - 1, 5] * tan]))
        out.append((prev, np.array([D[t, 0], D[t, 1], D[t, 2] * tan])))
    return out, tan

