import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (HIP) device")
    config.addinivalue_line("markers", "slow: long-running test")


@pytest.fixture(scope="session")
def hip_lib():
    """The in-tree HIP library; on a GPU box it MUST load (no silent eager fallback)."""
    import torch
    from distributedpytorch_amd.ops import _lib
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    assert _lib.available(), f"HIP kernel library missing: {_lib.LIB_PATH}"
    return _lib.lib()
