import os
import sys
from pathlib import Path

import numpy as np
import pytest

ROOT = Path(__file__).resolve().parent.parent
PKG = ROOT / "3dgs_study_amd"
for p in (str(PKG), str(ROOT)):
    if p not in sys.path:
        sys.path.insert(0, p)

REFERENCE = Path("/root/reference")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs the HIP library)")
    config.addinivalue_line("markers", "slow: long-running")


@pytest.fixture(scope="session")
def oracle():
    from oracle import oracle as o

    o.build()
    return o


@pytest.fixture(scope="session")
def dev():
    """cuda:0 with the native library loaded; fails (never skips) without a GPU."""
    import torch

    assert torch.cuda.is_available(), "gpu-marked test needs a ROCm device"
    from diff_gaussian_rasterization import _C

    _C.load_library()
    return torch.device("cuda:0")


def golden(name):
    return np.load(ROOT / "tests" / "golden" / name)
