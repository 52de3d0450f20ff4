import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "mpistragglers.jl_amd"), os.path.join(ROOT, "oracle")):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (HIP device); run with -m gpu")
    config.addinivalue_line("markers", "timing: checks host-time latencies against the oracle's clock; "
                                       "runs after the other tests (pytest_collection_modifyitems)")


def pytest_collection_modifyitems(session, config, items):
    """Order: every other test, then the multi-process GPU tests (test_gpu_procs.py), then the
    timing checks (latency against the oracle's virtual clock, marker `timing`): a stall of the
    box inflates those, so they go where a miss under `-x` costs no other test.  (Round 4's
    first order put them before the multi-process tests, which had disturbed them in round 3;
    with the queue cap and the one-wave doorbell wait they now pass right after them:
    profiles/r04_gated_stall.txt, r04order.)  The sort is stable: file and definition order are
    kept inside each group."""
    def group(item):
        if item.get_closest_marker("timing"):
            return 2
        return 1 if item.fspath.basename == "test_gpu_procs.py" else 0
    items.sort(key=group)


@pytest.fixture(scope="session")
def built():
    """Build the oracle (gcc) and the HIP library (hipcc) once per session if missing."""
    import subprocess
    if not os.path.exists(os.path.join(ROOT, "oracle", "_build", "liboracle.so")):
        subprocess.check_call(["make", "-s", "-C", os.path.join(ROOT, "oracle"), "all"])
    if not os.path.exists(os.path.join(ROOT, "mpistragglers.jl_amd", "_build", "libmpiasyncpools.so")):
        subprocess.check_call(["make", "-s", "-j8", "-C", os.path.join(ROOT, "mpistragglers.jl_amd")])
    return True


@pytest.fixture(autouse=True)
def _release_comms(request):
    """After a GPU test, collect the comms it left unclosed: their streams go back to the
    process's capped queue set (MPA_MAX_QUEUES), or the next comm's workers would share them."""
    yield
    if request.node.get_closest_marker("gpu"):
        import gc
        gc.collect()
