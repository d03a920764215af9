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


@pytest.fixture(autouse=True)
def _fp32_matmul_precision():
    """The learned-OC trainer applies its config's matmul precision process-wide (as the
    reference does, learned_option_critic_trainer.py); restore torch's defaults (fp32 GEMMs) after every
    test so no later comparison runs its torch reference on reduced-precision GEMMs."""
    yield
    import torch

    torch.set_float32_matmul_precision("highest")
    torch.backends.cuda.matmul.allow_tf32 = False
    torch.backends.cudnn.allow_tf32 = True     # torch's default


@pytest.fixture(scope="session")
def gpu_device():
    import torch

    if not torch.cuda.is_available():
        pytest.skip("no HIP device in this container")
    from SwarmACB_isaac import _native

    _native.load()  # a GPU box without the built extension must fail, not skip
    return torch.device("cuda:0")
