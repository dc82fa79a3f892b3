"""Test configuration.

Markers: ``gpu`` -- needs an MI355X (runs through the C ABI of libsamq_hip.so).  Everything
else runs on the CPU (oracle vs golden vectors, host logic, ABI exports, gloo multi-process).
The oracle (``oracle/``) is used here only as the checker.
"""
import os
import sys
from pathlib import Path

import pytest

REPO = Path(__file__).resolve().parent.parent
PKG = REPO / "sam-quantization_amd"
GOLDEN = Path(__file__).resolve().parent / "golden"
for p in (str(REPO), str(PKG)):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an AMD Instinct MI355X (gfx950) GPU")
    config.addinivalue_line("markers", "slow: CPU test that takes more than ~20 s")


def gpu_available() -> bool:
    try:
        import torch
        return torch.cuda.is_available()
    except Exception:
        return False


@pytest.fixture(scope="session")
def golden_dir():
    return GOLDEN


@pytest.fixture(scope="session")
def cuda():
    import torch
    if not torch.cuda.is_available():
        pytest.fail("GPU test selected but no HIP device is visible")
    torch.manual_seed(0)
    return torch.device("cuda:0")
