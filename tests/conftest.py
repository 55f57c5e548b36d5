import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs via gpurun on the GPU box)")
    config.addinivalue_line("markers", "slow: long-running")


@pytest.fixture(scope="session")
def C():
    import hpcjoin
    return hpcjoin.require_native()


@pytest.fixture(scope="session")
def cuda():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    torch.cuda.set_device(0)
    return torch.device("cuda", 0)


def devices():
    """cpu always; cuda only on the GPU box (marked gpu)."""
    return [pytest.param("cpu", id="host"), pytest.param("cuda", id="device", marks=pytest.mark.gpu)]
