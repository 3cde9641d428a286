import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (HIP kernels / RCCL)")
    config.addinivalue_line("markers", "slow: longer CPU integration test")


@pytest.fixture(scope="session")
def cuda():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from ml_recipe_distributed_pytorch_amd import _native
    _native.kernels()  # fail loudly if the HIP library is missing on a GPU box
    return torch.device("cuda", 0)
