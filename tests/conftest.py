"""Test configuration: registers the `gpu` marker and puts the product
package (bulletproof-perm_amd/) and the oracle on sys.path."""
import os
import sys
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parent.parent
# a host-side fault inside libbpperm prints its native backtrace before
# Python's faulthandler report (ctx.hip segv_trace)
os.environ.setdefault("BPP_SEGV_TRACE", "1")
sys.path.insert(0, str(ROOT / "bulletproof-perm_amd"))
sys.path.insert(0, str(ROOT))


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through libbpperm.so on cuda:0)")


def gpu_available() -> bool:
    try:
        import torch
        return torch.cuda.is_available()
    except Exception:
        return False


@pytest.fixture(scope="session")
def ctx():
    import bpperm
    c = bpperm.Context(0)
    yield c
    c.close()
