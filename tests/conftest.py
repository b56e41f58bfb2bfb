import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG_DIR = os.path.join(ROOT, "videoprism-mlx_amd")
for p in (ROOT, PKG_DIR, os.path.join(ROOT, "tests"), os.path.join(ROOT, "tools")):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through libvideoprism_hip.so)")
    config.addinivalue_line("markers", "slow: long-running")


@pytest.fixture(scope="session")
def cuda():
    import torch
    if not torch.cuda.is_available():
        pytest.fail("GPU test selected but no HIP device is visible")
    from videoprism import _native
    _native.load()  # fail loudly if the HIP library is missing
    return torch.device("cuda:0")
