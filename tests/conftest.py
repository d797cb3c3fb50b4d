import json
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


def pytest_terminal_summary(terminalreporter):
    """One line per parity config measured in this session (tests/_parity.py summarize): bad and
    certified envs, the largest certified cut-off margin, max |diff|, the 1-ulp band's max."""
    try:
        from tests import _parity
    except Exception:  # noqa: BLE001
        return
    def short(v):
        if isinstance(v, float):
            return float(f"{v:.3g}")
        if isinstance(v, dict):
            return {k: short(x) for k, x in v.items()}
        return v

    if _parity.SUMMARY:
        terminalreporter.section("parity summary")
        # the full-size configs last: they are what a reader of the log's tail needs
        for rec in sorted(_parity.SUMMARY, key=lambda r: r.get("envs", 0)):
            terminalreporter.write_line("PARITY " + json.dumps(short(rec), separators=(",", ":")))
