import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (runs through the HIP C-ABI)")


@pytest.fixture(autouse=True)
def _device_check_after_gpu_test(request):
    """After every GPU test that loaded the library: gcs_device_check(0) --
    every stream drained without a fault (looked at twice, 1 ms apart: a
    fault reaches the process asynchronously) and no burst-server grid left
    resident without a ring.  A fault is then charged, as a teardown error, to
    the test whose work caused it instead of surfacing in a later one."""
    yield
    if request.node.get_closest_marker("gpu") is None:
        return
    from mtcp_amd import gpucsum
    if gpucsum._lib is None:
        return
    gpucsum.device_check(0)
