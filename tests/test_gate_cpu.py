"""Gated replay on the CPU: every golden scenario (tests/golden/traces.json) and random
schedules replayed through the product's state machine over the HOST transport (the
multi-process mailbox protocol with host-executed test workers), workers split between
the coordinator's process and a server, the server's tasks finishing in a scrambled
physical order.  With the oracle's gate schedule the trace (repochs, sepochs, active,
recvbuf after every call) must equal the oracle's bit for bit.  The device version of the
same replay is tests/test_gpu_gated.py."""
import threading
import uuid

import numpy as np
import pytest

import gated
import mpiasyncpools as M

SCEN = gated.scenarios()


@pytest.fixture(scope="module", autouse=True)
def _built(built):
    return built


def _run_host(sc, seed=0):
    _, sched = gated.oracle_gate(sc)
    comm_n = sc.get("comm_workers", sc["n"])
    placement = [0 if w % 3 == 0 else 1 for w in range(comm_n)]  # workers 1, 4, 7 on rank 0
    name = f"/mpa_gate_{uuid.uuid4().hex[:10]}"
    coord = M.DistComm(comm_n, placement, 0, name, 256, transport="host")
    server = M.DistComm(comm_n, placement, 1, name, 256, transport="host")
    rng = np.random.default_rng(seed)
    for w in range(1, comm_n + 1):
        c = coord if placement[w - 1] == 0 else server
        c.set_task(w, "kmap2")
        if placement[w - 1] == 1:  # physical completions in an order unrelated to the schedule
            c.set_delays(w, rng.integers(0, 300, size=37) * 1000)
    th = threading.Thread(target=server.serve, daemon=True)
    th.start()
    try:
        coord.set_gate(*sched)
        got, pool = gated.replay(M, sc, coord, lambda k: np.zeros(k), lambda b: b, gated.make_golden().predicate,
                                 snap=np.copy)
    finally:
        coord.shutdown()
        th.join(timeout=60)
    assert not th.is_alive()
    server.close()
    coord.close()
    return got, pool


@pytest.mark.parametrize("name", [s["name"] for s in SCEN])
def test_golden_scenario_gated_on_host_transport(name):
    sc = next(s for s in SCEN if s["name"] == name)
    got, _ = _run_host(sc, seed=len(name))
    assert gated.mismatches(name, got, sc["results"]) == []


@pytest.mark.parametrize("seed", range(8))
def test_random_scenario_gated_on_host_transport(seed):
    sc = gated.random_scenario(seed)
    ref, _ = gated.oracle_gate(sc)
    got, _ = _run_host(sc, seed=seed)
    assert gated.mismatches(sc["name"], got, ref) == []


def test_gate_schedule_covers_every_observation():
    """The schedule has one step per observation point and releases each harvested task
    exactly once: on tag_ties it holds steps that release several workers at once (the
    ties Waitany! resolves lowest index first)."""
    sc = next(s for s in SCEN if s["name"] == "tag_ties")
    ref, (kinds, offs, ranks) = gated.oracle_gate(sc)
    assert len(offs) == len(kinds) + 1 and offs[-1] == len(ranks)
    assert int((kinds == M.MPA_GATE_CALL).sum()) == sum(op["op"] == "asyncmap" for op in sc["ops"])
    sizes = np.diff(offs)[kinds == M.MPA_GATE_WAIT]
    assert sizes.max() >= 2, "tag_ties should release tied completions together"


def test_gate_errors():
    """A schedule of the wrong shape is refused; a step of the wrong kind fails the call."""
    name = f"/mpa_gate_{uuid.uuid4().hex[:10]}"
    coord = M.DistComm(2, [0, 0], 0, name, 256, transport="host")
    for w in (1, 2):
        coord.set_task(w, "kmap2")
    with pytest.raises(M.ArgumentError):
        coord.set_gate([0], [0, 1], [3])        # rank 3 is not a worker
    with pytest.raises(M.ArgumentError):
        coord.set_gate([0, 7], [0, 0, 0], [])   # unknown kind
    coord.set_gate([M.MPA_GATE_WAIT], [0, 0], [])
    pool = M.MPIAsyncPool(2)
    with pytest.raises(M.ErrorException, match="gated replay"):
        M.asyncmap_(pool, np.zeros(1), np.zeros(6), np.zeros(2), np.zeros(6), coord, nwait=1)
    # the failed step closed the call (pool.cpp gate_step): the comm serves the next call
    coord.set_gate([], [], [])
    rep = M.asyncmap_(pool, np.zeros(1), np.zeros(6), np.zeros(2), np.zeros(6), coord, nwait=2)
    assert rep.tolist() == [pool.epoch, pool.epoch] and not pool.active.any()
    coord.shutdown()
    coord.close()
    sim = M.SimComm(2)
    with pytest.raises(M.ArgumentError):
        sim.set_gate([0], [0, 0], [])
