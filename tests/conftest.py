import os
import sys

import pytest

# record every kernel the library launches in this process (tests/test_zz_kernel_coverage.py)
os.environ.setdefault("GSRAST_LAUNCH_LOG", "1")

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "gaussian-splatting-skysphere_amd")
for p in (ROOT, PKG, os.path.join(ROOT, "tests")):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a HIP device (MI355X); parity tests through the C ABI")
    config.addinivalue_line("markers", "spawn_first: starts child processes on the GPU; runs before any other test, "
                                       "while this process has not touched the GPU")
    config.addinivalue_line("markers", "last: runs after every other test of the session")
    # autograd accumulating one leaf's gradient from backwards on several streams (multi-stream
    # views without a GradBucket): an error, not a warning, so no test relies on it
    config.addinivalue_line("filterwarnings", "error:The AccumulateGrad node's stream does not match:UserWarning")


def pytest_collection_modifyitems(config, items):
    # stable: keeps the rest in order; the kernel-coverage check runs after everything else
    items.sort(key=lambda it: 0 if it.get_closest_marker("spawn_first") else 2 if it.get_closest_marker("last") else 1)


@pytest.fixture(scope="session")
def oracle():
    from oracle import gs_oracle

    gs_oracle.build()
    return gs_oracle


def gpu_available():
    try:
        import torch

        return torch.cuda.is_available()
    except Exception:
        return False


@pytest.fixture(scope="session")
def device():
    import torch

    if not torch.cuda.is_available():
        pytest.fail("gpu test requested but no HIP device is visible")
    return torch.device("cuda:0")
