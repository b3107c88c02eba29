import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs on the GPU box via gpurun)")
    config.addinivalue_line("markers", "slow: long-running")


@pytest.fixture(scope="session")
def golden_ops():
    import numpy as np
    return np.load(os.path.join(ROOT, "tests", "golden", "ops.npz"))


@pytest.fixture(scope="session")
def golden_e2e():
    import numpy as np
    return np.load(os.path.join(ROOT, "tests", "golden", "e2e_tiny.npz"))
