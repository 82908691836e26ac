import os
import sys

import pytest

# torch first: it brings its own HIP runtime, and libsift_hip.so must bind to
# the one already loaded (if the library's HIP initialises first, torch's
# lazy init finds no device)
import torch  # noqa: F401

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
sys.path.insert(0, HERE)
sys.path.insert(0, os.path.join(ROOT, "sift-project_amd"))


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through the HIP C-ABI)")
    config.addinivalue_line("markers", "slow: long-running (large images / many ranks)")


@pytest.fixture(scope="session")
def gpu_ctx():
    from sift_hip import Context

    ctx = Context(0)
    yield ctx
    ctx.close()
