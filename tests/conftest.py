import os
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if REPO not in sys.path:
    sys.path.insert(0, REPO)
os.environ.setdefault("TQDM_DISABLE", "1")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a HIP device (MI355X); parity tests of the HIP path")


def pytest_sessionfinish(session, exitstatus):
    from tests import parity
    parity.dump()


@pytest.fixture(scope="session")
def gpu_device():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    from gaussian_splatting_lightning_amd import _native
    _native.load()
    return torch.device("cuda", 0)
