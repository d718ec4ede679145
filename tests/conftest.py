import os
import sys
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))
sys.path.insert(0, str(ROOT / "oracle"))


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through libklf.so on the device)")
    # build the native pieces in-tree if they are missing or stale (hipcc cross-compiles on CPU)
    from klogs_amd import _build
    _build.build_all(quiet=True)


def gpu_available() -> bool:
    try:
        import torch
        return torch.cuda.is_available()
    except Exception:
        return False


@pytest.fixture(scope="session")
def gpu():
    if not gpu_available():
        pytest.skip("no GPU")
    return 0
