import os
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if REPO not in sys.path:
    sys.path.insert(0, REPO)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs the HIP kernels)")
    config.addinivalue_line("markers", "slow: BASELINE-size inputs")


@pytest.fixture(scope="session")
def golden():
    import numpy as np

    d = os.path.join(REPO, "tests", "golden")
    return {name: np.load(os.path.join(d, f"{name}.npz")) for name in ("solvers", "spmv", "lartg")}


@pytest.fixture(scope="session")
def oracle_lib():
    """The C oracle (test infrastructure), built on demand with gcc."""
    import ctypes
    import subprocess

    so = os.path.join(REPO, "oracle", "build", "liboracle.so")
    if not os.path.exists(so):
        subprocess.check_call(["make", "-s", "-C", os.path.join(REPO, "oracle")])
    return ctypes.CDLL(so)
