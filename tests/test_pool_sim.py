"""Host logic of the product (libmpiasyncpools.so state machine) on the SIM transport,
checked bit for bit against the committed golden traces and against the oracle on
randomised schedules.  No GPU is used: SimComm is the library's virtual-clock transport
(test-only, never selected implicitly)."""
import json
import os

import numpy as np
import pytest

import mpiasyncpools as M
import oracle as O

GOLDEN = os.path.join(os.path.dirname(__file__), "golden")


@pytest.fixture(scope="module", autouse=True)
def _built(built):
    return built


def _load_make_golden():
    import importlib.util
    spec = importlib.util.spec_from_file_location("make_golden", os.path.join(GOLDEN, "make_golden.py"))
    mg = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mg)
    return mg


def run_product(sc, predicate):
    """Replay a golden scenario on the product's SimComm; same record layout as the oracle's."""
    n, comm_n = sc["n"], sc.get("comm_workers", sc["n"])
    ranks = sc.get("ranks", list(range(1, n + 1)))
    dur = np.asarray(sc["durations_ns"], dtype=np.int64).reshape(comm_n, -1)
    comm = M.SimComm(comm_n)
    comm.set_compute(sc.get("compute_ns", 0))
    for r in range(1, comm_n + 1):
        comm.set_task(r, sc["worker"])
        comm.set_delays(r, dur[r - 1])
    pool = M.MPIAsyncPool(ranks, epoch0=sc.get("epoch0", 0), nwait=sc.get("default_nwait"))
    send = np.zeros(sc.get("send_elems", 1))
    isend = np.zeros(n * send.size)
    chunk = sc.get("chunk_elems", 3)
    recv, irecv = np.zeros(n * chunk), np.zeros(n * chunk)
    out = []
    for op in sc["ops"]:
        if op.get("advance_ns"):
            comm.advance(op["advance_ns"])
        t0 = comm.now
        if op["op"] == "waitall":
            M.waitall_(pool, recv, irecv)
        else:
            send[0] = op.get("send", 0)
            nw = op.get("nwait")
            nw = predicate(nw) if isinstance(nw, str) else nw
            M.asyncmap_(pool, send, recv, isend, irecv, comm, nwait=nw, epoch=op.get("epoch"), tag=0)
        out.append({"repochs": pool.repochs.tolist(), "sepochs": pool.sepochs.tolist(),
                    "active": pool.active.astype(int).tolist(), "epoch": int(pool.epoch),
                    "latency_ns": [int(round(v * 1e9)) for v in pool.latency],
                    "t_start": int(t0), "t_end": int(comm.now), "recv": recv.tolist()})
    return out


GOLD = json.load(open(os.path.join(GOLDEN, "traces.json")))["scenarios"]


@pytest.mark.parametrize("name", [s["name"] for s in GOLD])
def test_product_matches_golden_traces(name):
    mg = _load_make_golden()
    sc = next(s for s in GOLD if s["name"] == name)
    got = run_product(sc, mg.predicate)
    for k, (g, r) in enumerate(zip(got, sc["results"])):
        # sepochs of never-dispatched workers are `undef` in the reference (:39); compare active ones
        for key in ("repochs", "active", "epoch", "latency_ns", "t_start", "t_end", "recv"):
            assert g[key] == r[key], (name, k, key)


@pytest.mark.parametrize("seed", range(12))
def test_product_matches_oracle_random(seed):
    """Random pools, delays (with ties), nwait kinds, explicit epochs and waitall!s."""
    mg = _load_make_golden()
    rng = np.random.default_rng(1000 + seed)
    n = int(rng.integers(1, 12))
    ops = []
    for e in range(int(rng.integers(5, 60))):
        r = rng.random()
        if r < 0.08:
            ops.append({"op": "waitall"})
            continue
        op = {"op": "asyncmap", "send": int(rng.integers(0, 1000)),
              "advance_ns": int(rng.integers(0, 3)) * 1_000_000 if rng.random() < 0.3 else 0}
        k = rng.random()
        if k < 0.6:
            op["nwait"] = int(rng.integers(0, n + 1))
        elif k < 0.8:
            op["nwait"] = f"count_{int(rng.integers(0, n + 1))}"
        else:
            op["nwait"] = "first"
        if rng.random() < 0.2:
            op["epoch"] = int(rng.integers(-3, 40))
        ops.append(op)
    d = rng.integers(0, 6, size=(n, 8)) * 1_000_000
    sc = {"name": f"rand{seed}", "n": n, "worker": "kmap2", "durations_ns": d.ravel().tolist(),
          "compute_ns": int(rng.integers(0, 2)) * 500_000, "ops": ops}
    ref = mg.run_scenario(sc)
    got = run_product(sc, mg.predicate)
    for k, (g, r) in enumerate(zip(got, ref)):
        for key in ("repochs", "active", "epoch", "latency_ns", "t_start", "t_end", "recv"):
            assert g[key] == r[key], (seed, k, key)


def test_reference_error_messages():
    comm = M.SimComm(2)
    for r in (1, 2):
        comm.set_task(r, "echo")
    pool = M.MPIAsyncPool(2)
    s, i_s, r, i_r = np.zeros(1), np.zeros(2), np.zeros(2), np.zeros(2)
    with pytest.raises(M.ArgumentError, match=r"nwait must be in the range \[0, length\(pool.ranks\)\], but is -1"):
        M.asyncmap_(pool, s, r, i_s, i_r, comm, nwait=-1)
    with pytest.raises(M.DimensionMismatch, match="sendbuf is of size 8 bytes, but isendbuf is of size 8 bytes when 16 bytes are needed"):
        M.asyncmap_(pool, s, r, np.zeros(1), i_r, comm, nwait=1)
    with pytest.raises(M.DimensionMismatch, match="recvbuf is of size 16 bytes, but irecvbuf is of size 24 bytes"):
        M.asyncmap_(pool, s, r, i_s, np.zeros(3), comm, nwait=1)
    with pytest.raises(M.DimensionMismatch, match="The length of recvbuf and irecvbuf must be a multiple of the number of workers"):
        M.asyncmap_(pool, s, np.zeros(3), i_s, np.zeros(3), comm, nwait=1)
    with pytest.raises(M.ArgumentError, match="The eltype of sendbuf must be isbits, but is object"):
        M.asyncmap_(pool, np.array([None], dtype=object), r, i_s, i_r, comm, nwait=1)
    with pytest.raises(M.ArgumentError, match="The eltype of sendbuf must be isbits, but is object"):
        M.waitall_(pool, np.array([None, None], dtype=object), i_r)
    assert pool.epoch == 0 and not pool.active.any()
    with pytest.raises(M.ErrorException, match="nwait must be either an Integer or a Function, but is a float"):
        M.asyncmap_(pool, s, r, i_s, i_r, comm, nwait=1.5)
    assert pool.active.all() and pool.epoch == 1  # dispatch happened before the error (:156-158)
    M.waitall_(pool, r, i_r)
    assert not pool.active.any()


def test_predicate_exception_propagates_and_state_is_consistent():
    comm = M.SimComm(3)
    for r in (1, 2, 3):
        comm.set_task(r, "kmap2")
        comm.set_delays(r, [r * 1_000_000])
    pool = M.MPIAsyncPool(3)
    s, i_s, r, i_r = np.zeros(1), np.zeros(3), np.zeros(9), np.zeros(9)

    def bad(epoch, repochs):
        raise KeyError("boom")
    with pytest.raises(KeyError):
        M.asyncmap_(pool, s, r, i_s, i_r, comm, nwait=bad)
    assert pool.active.all()
    M.waitall_(pool, r, i_r)
    assert (pool.repochs == 1).all()


def test_unsatisfiable_predicate_is_an_error():
    """All workers inactive and the predicate false: MPI_Waitany would return
    MPI_UNDEFINED (undefined in the reference); the build raises."""
    comm = M.SimComm(2)
    for r in (1, 2):
        comm.set_task(r, "echo")
    pool = M.MPIAsyncPool(2)
    s, i_s, r, i_r = np.zeros(1), np.zeros(2), np.zeros(2), np.zeros(2)
    with pytest.raises(M.ErrorException, match="unsatisfiable"):
        M.asyncmap_(pool, s, r, i_s, i_r, comm, nwait=lambda e, rep: False)


def test_zero_workers_and_empty_messages():
    comm = M.SimComm(1)
    comm.set_task(1, "echo")
    pool = M.MPIAsyncPool(1)
    s = np.zeros(0)
    rep = M.asyncmap_(pool, s, np.zeros(0), np.zeros(0), np.zeros(0), comm, nwait=1)
    assert list(rep) == [1]
    pool0 = M.MPIAsyncPool(0)
    with pytest.raises(M.ErrorException, match="DivideError"):  # mod(length(recvbuf), 0) throws in Julia
        M.asyncmap_(pool0, s, np.zeros(0), np.zeros(0), np.zeros(0), comm, nwait=0)


def test_pool_fields_and_alias():
    pool = M.MPIAsyncPool([1, 4, 5], epoch0=7, nwait=2)
    assert list(pool.ranks) == [1, 4, 5] and pool.nwait == 2 and pool.epoch == 7
    assert list(pool.repochs) == [7, 7, 7] and not pool.active.any()
    comm = M.SimComm(5)
    for r in range(1, 6):
        comm.set_task(r, "kmap1")
    s, i_s, r, i_r = np.zeros(1), np.zeros(3), np.zeros(3), np.zeros(3)
    a = M.asyncmap_(pool, s, r, i_s, i_r, comm)
    assert a is pool.repochs
    assert pool.epoch == 8 and (r == [1, 4, 5]).sum() >= 2
