"""Shared fixtures. `-m "not gpu"` runs here (no GPU); `-m gpu` runs on an MI355X box."""
import os
import sys

import numpy as np
import pytest

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
