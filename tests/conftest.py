import os
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if REPO not in sys.path:
    sys.path.insert(0, REPO)
TESTS = os.path.dirname(os.path.abspath(__file__))
if TESTS not in sys.path:
    sys.path.insert(0, TESTS)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through libvpcsum.so on cuda:0)")


@pytest.fixture(scope="session")
def orc():
    from oracle import oracle as O
    O.build()
    return O.Oracle()


@pytest.fixture(autouse=True)
def _sync_after_gpu_test(request):
    """VPCSUM_SYNC_EACH_TEST=1 (debugging): synchronise the device after every GPU test, so that a
    fault from asynchronous work (a service grid still polling, a kernel on another stream) is
    reported against the test that started it, not the next one."""
    yield
    if os.environ.get("VPCSUM_SYNC_EACH_TEST") == "1" and request.node.get_closest_marker("gpu"):
        import torch
        torch.cuda.synchronize()
