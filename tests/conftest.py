import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs the HIP kernels)")
    config.addinivalue_line("markers", "slow: long CPU test")


@pytest.fixture(scope="session")
def dev():
    import torch
    if not torch.cuda.is_available():
        pytest.fail("GPU test selected but no GPU is visible")
    return torch.device("cuda:0")


@pytest.fixture
def engine():
    """engine.use(True): the convs of this test run on the implicit-GEMM engine also where
    a direct kernel serves the geometry (ops.engine_only, TMR_IO_ENGINE); use(False): the product
    routing.  Reset when the test ends."""
    from tmrnet_amd import ops

    class _Switch:
        def use(self, on):
            ops._ENGINE[0] = bool(on)

    yield _Switch()
    ops._ENGINE[0] = False
