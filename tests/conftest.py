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
    # the binding checks every release of a page-locked range against HIP (_audit_registrations)
    os.environ.setdefault("VPCSUM_AUDIT_REGISTRATIONS", "1")


@pytest.fixture(scope="session")
def orc():
    from oracle import oracle as O
    O.build()
    return O.Oracle()


@pytest.fixture(autouse=True)
def _sync_after_gpu_test(request):
    """Every GPU test ends with a device synchronise (and a garbage collection first, so contexts
    the test dropped are destroyed -- their service grids stopped -- inside it): a fault from
    asynchronous work (a service grid still polling, a kernel on another stream) is reported against
    the test that started it, not a later one.  VPCSUM_SYNC_EACH_TEST=0 turns it off."""
    yield
    if os.environ.get("VPCSUM_SYNC_EACH_TEST", "1") != "0" and request.node.get_closest_marker("gpu"):
        import gc
        import torch
        gc.collect()
        if torch.cuda.is_available():
            torch.cuda.synchronize()
            _audit_registrations()


def _audit_registrations():
    """Every host range the binding page-locked and released during the test (unregister, or its
    context / group destroyed) was no longer registered with HIP right after the release
    (vpcsum.py: VPCSUM_AUDIT_REGISTRATIONS).  A registration that outlived its release would make a
    later pageable copy from whatever is allocated there read through a dead mapping
    (DESIGN_HISTORY.md "Round 6: the intermittent fault"): caught in the test that made it."""
    import sys
    V = sys.modules.get("vproxy_amd.vpcsum")
    if V is None:
        return
    stale = [(hex(p), n) for p, n in V._stale]
    V._stale.clear()
    assert not stale, f"HIP still held released ranges as registered: {stale[:4]}"
