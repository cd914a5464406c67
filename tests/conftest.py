import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG_DIR = os.path.join(ROOT, "risk-aware-hybrid-lqr-mpc-navigation-for-autonomous-systems_amd")
GOLDEN = os.path.join(ROOT, "tests", "golden")
for p in (ROOT, PKG_DIR):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (HIP device)")
    config.addinivalue_line("markers", "slow: long-running CPU test")


@pytest.fixture(scope="session")
def golden():
    import numpy as np

    def load(name):
        return np.load(os.path.join(GOLDEN, name))
    return load


@pytest.fixture(scope="session")
def lib():
    """The native C-ABI library (librmpc.so) -- built by __graft_entry__.build()."""
    from rmpc import _native
    return _native.load()


@pytest.fixture(scope="session")
def gpu_lib(lib):
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    return lib
