import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)
# the service tests drive the app through starlette's TestClient (not a loopback peer); auth itself is covered by
# tests/test_auth.py, which sets its own mode
os.environ.setdefault("DXA_AUTH", "off")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: test needs a real MI355X (HIP device)")
    config.addinivalue_line("markers", "slow: long-running test")


@pytest.fixture(scope="session")
def gpu():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from dxa.ops import native
    native.lib()          # the native library must load on a GPU box — never silently skip it
    return torch.device("cuda:0")
