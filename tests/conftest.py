import importlib
import os
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if REPO not in sys.path:
    sys.path.insert(0, REPO)
ORACLE_DIR = os.path.join(REPO, "oracle")
if ORACLE_DIR not in sys.path:
    sys.path.insert(0, ORACLE_DIR)
GOLDEN = os.path.join(REPO, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (gfx950) device")
    config.addinivalue_line("markers", "slow: long CPU test")


def load_pkg():
    return importlib.import_module("zig-raytracing-weekend_amd")


@pytest.fixture(scope="session")
def rtw():
    return load_pkg()


@pytest.fixture(scope="session")
def oracle():
    import oracle as O  # noqa: E402  (oracle/oracle.py: test infrastructure)
    O.lib()
    return O


@pytest.fixture(scope="session")
def earth_rgba():
    import numpy as np
    with np.load(os.path.join(GOLDEN, "earthmap_rgba.npz"), allow_pickle=False) as z:
        return np.ascontiguousarray(z["rgba"])
