import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

GOLDEN = os.path.join(ROOT, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a ROCm GPU (MI355X); runs the HIP path through the C-ABI")
    config.addinivalue_line("markers", "slow: takes more than ~20 s on the CPU")


@pytest.fixture(scope="session")
def gpu_device():
    import torch  # noqa: F401  (before libyk: one HIP runtime)
    if not torch.cuda.is_available():
        pytest.fail("gpu test collected without a GPU (run with -m 'not gpu' on CPU hosts)")
    from core_amd.device import Device
    d = Device(0)
    yield d
    d.close()
