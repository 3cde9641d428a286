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


@pytest.fixture(scope="session")
def host_lib():
    """The C++ host runtime (tokenizers, synth, crc32c); built on demand (g++, no GPU needed)."""
    from ml_recipe_distributed_pytorch_amd import _native
    if not _native.host_available():
        from ml_recipe_distributed_pytorch_amd.csrc.build import build_host
        build_host(verbose=False)
        _native.reset_cache()
    return _native.host()


FIXTURES = os.path.join(os.path.dirname(os.path.abspath(__file__)), "fixtures")


def free_port() -> int:
    import socket
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]
