import os
import sys

import pytest

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
