"""The timing harness's own helpers (tests/gated.py), on CPU: the host watchdog process and
the GC-off context the device latency checks run in."""
import gc
import time

import gated


def test_no_gc_disables_and_restores_the_collector():
    assert gc.isenabled()
    with gated.no_gc():
        assert not gc.isenabled()
    assert gc.isenabled()
    gc.disable()
    try:
        with gated.no_gc():
            assert not gc.isenabled()
        assert not gc.isenabled()  # left as it was found
    finally:
        gc.enable()


def test_host_watchdog_reports_its_oversleep():
    w = gated.HostWatchdog()
    try:
        w.take()
        time.sleep(0.2)
        worst, over = w.take()
        assert 0.0 <= worst < 1000.0 and over >= 0
    finally:
        w.close()
