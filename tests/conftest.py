import os
import sys
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parent.parent
if str(ROOT) not in sys.path:
    sys.path.insert(0, str(ROOT))


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a ROCm GPU (MI355X); parity of the HIP kernels")


def pytest_sessionstart(session):
    # build the native library in-tree if it is missing or stale (hipcc cross-compiles w/o a GPU)
    import __graft_entry__

    __graft_entry__.build()


@pytest.fixture(scope="session")
def gpu_device():
    import torch

    if not torch.cuda.is_available():
        pytest.skip("no ROCm GPU visible")
    return "cuda:0"
