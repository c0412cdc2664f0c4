import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through the HIP C ABI)")


@pytest.fixture(scope="session")
def lib():
    import rsmt2d_amd
    if not os.path.exists(rsmt2d_amd.LIB_PATH):
        rsmt2d_amd.build()
    return rsmt2d_amd.library()


@pytest.fixture
def rng():
    return np.random.default_rng(0x52534D543244)


def rand_shares(rng, n, S):
    return [rng.integers(0, 256, S, dtype=np.uint8).tobytes() for _ in range(n)]


def const_share(v, S=512):
    return bytes([v]) * S
