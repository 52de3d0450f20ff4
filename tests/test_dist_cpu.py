"""N > 1 control plane on CPU: world_size-2 (and 3) process groups over gloo, the
coordinator on rank 0 and workers served by other processes through the shared-memory
mailboxes (MPA_TRANSPORT_HOST: the HIP transport's protocol with host-executed test
workers).  Checks the test/kmap2.jl properties across processes, pause/resume between
serve() sessions, waitall!, the predicate form of nwait, and shutdown."""
import multiprocessing as mp

import pytest

import dist_worker


def _run(world, placement):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = dist_worker.free_port()
    procs = [ctx.Process(target=dist_worker.kmap2_dist, args=(r, world, port, "host", placement, q))
             for r in range(world)]
    for p in procs:
        p.start()
    try:
        status, payload = q.get(timeout=180)
    finally:
        for p in procs:
            p.join(timeout=60)
            if p.is_alive():
                p.kill()
    assert status == "ok", payload
    assert payload == [], payload
    assert all(p.exitcode == 0 for p in procs), [p.exitcode for p in procs]


@pytest.mark.parametrize("placement", [[0, 1, 1, 1], [1, 1, 1]])
def test_kmap2_two_processes(built, placement):
    _run(2, placement)


def test_kmap2_three_processes(built):
    _run(3, [0, 1, 2, 1, 2])
