import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (HIP kernels); skipped in CPU CI")
    config.addinivalue_line("markers", "unit: hermetic CPU unit test")
    config.addinivalue_line("markers", "integration: multi-component test against in-process fakes")
    config.addinivalue_line("markers", "end_to_end: full worker/app flow against LocalHypha")
    config.addinivalue_line("markers", "requires_gpu: alias used by reference app tests")
    config.addinivalue_line("markers", "slow: long-running test")


def pytest_collection_modifyitems(config, items):
    import torch

    if torch.cuda.is_available():
        return
    skip = pytest.mark.skip(reason="no GPU visible")
    for it in items:
        if "gpu" in it.keywords:
            it.add_marker(skip)


@pytest.fixture(scope="session")
def gpu():
    import torch

    from bioengine_worker_amd.ops import _native

    assert torch.cuda.is_available()
    _native.hip()  # must load: GPU tests never run on a silent fallback
    return torch.device("cuda:0")
