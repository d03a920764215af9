import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG_DIR = os.path.join(ROOT, "swarmacb-isaaclab_amd")
for p in (ROOT, PKG_DIR, os.path.join(ROOT, "tests")):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (HIP device) and libswarmstep.so")


@pytest.fixture(scope="session")
def gpu_device():
    import torch

    if not torch.cuda.is_available():
        pytest.skip("no HIP device in this container")
    from SwarmACB_isaac import _native

    _native.load()  # a GPU box without the built extension must fail, not skip
    return torch.device("cuda:0")
