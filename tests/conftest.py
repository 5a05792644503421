import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a ROCm (MI355X) device and the built HIP library")
    config.addinivalue_line("markers", "slow: long-running CPU test")


def _gpu_available() -> bool:
    import torch

    return torch.cuda.is_available()


def pytest_collection_modifyitems(config, items):
    if any("gpu" in item.keywords for item in items) and not _gpu_available():
        skip = pytest.mark.skip(reason="no ROCm GPU in this environment")
        for item in items:
            if "gpu" in item.keywords:
                item.add_marker(skip)


@pytest.fixture(autouse=True)
def _device_sync(request):
    """Every GPU test ends with a device synchronisation, so an asynchronous kernel error surfaces in
    the test that launched the kernel."""
    yield
    if "gpu" in request.keywords and _gpu_available():
        import torch

        torch.cuda.synchronize()
