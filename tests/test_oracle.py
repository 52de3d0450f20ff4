"""Pin the ORACLE: the reference's own tests, restated against the C oracle.

The reference has no golden vectors; its tests are multi-process property tests
(test/kmap1.jl, test/kmap2.jl, run by test/runtests.jl with 3 and 10 MPI ranks).  Every
assertion of those files is restated here against the oracle's virtual-clock workers,
which run the same worker programs (test/kmap1.jl:23-33, test/kmap2.jl:76-99) and sleep
the same distribution (`max(rand()/10, 0.005)` s, test/kmap2.jl:95).
"""
import json
import os

import numpy as np
import pytest

import lsq
import oracle as O

GOLDEN = os.path.join(os.path.dirname(__file__), "golden")


@pytest.fixture(scope="module", autouse=True)
def _built(built):
    return built


@pytest.mark.parametrize("nranks", [3])  # test/runtests.jl:20-27
def test_kmap1(nranks):
    nworkers = nranks - 1
    pool = O.OraclePool(nworkers)
    sim = O.OracleSim(nworkers, O.ORC_WORKER_KMAP1)
    sendbuf = np.repeat([3.14], 1)                          # kmap1.jl:16
    isendbuf = np.zeros(nworkers * len(sendbuf))            # :17
    recvbuf = np.empty(nworkers)                            # :18
    irecvbuf = recvbuf.copy()                               # :19
    O.asyncmap(pool, sim, sendbuf, recvbuf, isendbuf, irecvbuf, nwait=nworkers, tag=0)  # :20-21
    np.testing.assert_allclose(recvbuf, np.arange(1, nworkers + 1))  # :22
    # :30 every worker received 3.14: the bytes it was sent are isendbuf's slots
    np.testing.assert_allclose(isendbuf, np.repeat([3.14], nworkers))


def _kmap2(nworkers, seed):
    rng = np.random.default_rng(seed)
    d = np.maximum(rng.random((nworkers, 512)) / 10, 0.005)   # kmap2.jl:95
    sim = O.OracleSim(nworkers, O.ORC_WORKER_KMAP2, (d * 1e9).astype(np.int64))
    pool = O.OraclePool(nworkers)
    assert list(pool.ranks) == list(range(1, nworkers + 1))   # kmap2.jl:22
    sendbuf = np.empty(1)                                     # :58
    isendbuf = np.zeros(nworkers)                             # :59
    recvbuf = np.empty(3 * nworkers)                          # :60
    recvbufs = [recvbuf[3 * i:3 * i + 3] for i in range(nworkers)]  # :61
    irecvbuf = recvbuf.copy()                                 # :62
    nwait = 2                                                 # :63
    for epoch in range(1, 101):                               # :66
        sendbuf[0] = epoch                                    # :67
        repochs = O.asyncmap(pool, sim, sendbuf, recvbuf, isendbuf, irecvbuf, nwait=nwait, tag=0)  # :69
        from_this_epoch = 0
        for i in range(nworkers):
            wrank, t, wepoch = recvbufs[i]                    # :73
            if repochs[i] == 0:                               # :76-78
                continue
            if repochs[i] == epoch:                           # :79-81
                from_this_epoch += 1
            assert wepoch == repochs[i]                       # :84
            assert wrank == i + 1
        assert from_this_epoch >= nwait                       # :87
    for epoch in range(1, 101):                               # :91
        O.asyncmap(pool, sim, sendbuf, recvbuf, isendbuf, irecvbuf, nwait=1, tag=0)  # :92
        O.waitall(pool, sim, recvbuf, irecvbuf)               # :93
        assert not pool.active.any()                          # :94
    f = lambda epoch, repochs: repochs[0] == epoch            # :99
    for _ in range(101, 201):                                 # :100
        t0 = sim.now
        repochs = O.asyncmap(pool, sim, sendbuf, recvbuf, isendbuf, irecvbuf, nwait=f, tag=0)  # :102
        delay = (sim.now - t0) / 1e9
        assert repochs[0] == pool.epoch                       # :104
        assert abs(delay - pool.latency[0]) <= 1e-3           # :105
    return pool, sim


@pytest.mark.parametrize("nranks", [3, 10])  # test/runtests.jl:29-45
@pytest.mark.parametrize("seed", [0, 1, 2])
def test_kmap2(nranks, seed):
    _kmap2(nranks - 1, seed)


def test_kmap2_fifo_t_counts():
    """The worker's message counter t (kmap2.jl:82-84) equals the tasks it served."""
    pool, sim = _kmap2(9, 5)
    for i in range(9):
        assert sim.tasks(i) >= 1


def test_asyncmap_returns_alias():
    """`return pool.repochs` (:187): the returned vector is the pool's, mutated later."""
    pool = O.OraclePool(3)
    sim = O.OracleSim(3, O.ORC_WORKER_ECHO, np.array([[1], [2], [3]]) * 1000)
    s, i_s, r, i_r = np.zeros(1), np.zeros(3), np.zeros(3), np.zeros(3)
    a = O.asyncmap(pool, sim, s, r, i_s, i_r, nwait=3)
    first = a.copy()
    O.asyncmap(pool, sim, s, r, i_s, i_r, nwait=3)
    assert (a == pool.repochs).all() and not (a == first).all()


def test_errors_and_messages():
    pool = O.OraclePool(2)
    sim = O.OracleSim(2, O.ORC_WORKER_ECHO)
    s, i_s, r, i_r = np.zeros(1), np.zeros(2), np.zeros(2), np.zeros(2)
    with pytest.raises(O.ArgumentError, match=r"nwait must be in the range \[0, length\(pool.ranks\)\], but is 3"):
        O.asyncmap(pool, sim, s, r, i_s, i_r, nwait=3)
    with pytest.raises(O.DimensionMismatch, match="sendbuf is of size 8 bytes, but isendbuf is of size 8 bytes when 16 bytes are needed"):
        O.asyncmap(pool, sim, s, r, np.zeros(1), i_r, nwait=1)
    with pytest.raises(O.DimensionMismatch, match="recvbuf is of size 16 bytes, but irecvbuf is of size 24 bytes"):
        O.asyncmap(pool, sim, s, r, i_s, np.zeros(3), nwait=1)
    with pytest.raises(O.DimensionMismatch, match="must be a multiple of the number of workers"):
        O.asyncmap(pool, sim, s, np.zeros(3), i_s, np.zeros(3), nwait=1)
    # state untouched by validation failures (:69-77 run before :87)
    assert pool.epoch == 0 and not pool.active.any()
    # a non-Integer non-Function nwait errors only after dispatch (:156-158)
    with pytest.raises(O.ErrorException, match="nwait must be either an Integer or a Function, but is a float"):
        O.asyncmap(pool, sim, s, r, i_s, i_r, nwait=1.5)
    assert pool.active.all() and pool.epoch == 1


def test_philox_kat():
    kat = json.load(open(os.path.join(GOLDEN, "philox_kat.json")))["vectors"]
    import ctypes as C
    L = O.lib()
    for ctr, key, want in kat:
        got = lsq.philox4x32_10(*[np.array([c], dtype=np.uint32) for c in ctr], key[0], key[1])
        assert [int(v[0]) for v in got] == want
        out = (C.c_uint32 * 4)()
        L.orc_philox((C.c_uint32 * 4)(*ctr), (C.c_uint32 * 2)(*key), out)
        assert list(out) == want


def test_datagen_numpy_matches_c():
    import ctypes as C
    L = O.lib()
    L.orc_gen_f32.argtypes = [C.c_uint64, C.c_uint32, C.c_uint64, C.c_int64, C.c_float, C.c_void_p]
    for e0, cnt in ((0, 1000), (3, 517), (2**33 + 1, 64)):
        ref = lsq.gen_vector(99, e0, cnt, "f32", stream=lsq.STREAM_A, scale=0.03125)
        out = np.empty(cnt, dtype=np.float32)
        L.orc_gen_f32(99, lsq.STREAM_A, e0, cnt, 0.03125, out.ctypes.data)
        assert np.array_equal(out.view(np.uint32), ref.view(np.uint32))
    u = lsq.unit_f32(lsq.philox_words(1, 0, np.arange(100000, dtype=np.uint64)))
    assert u.min() >= -1.0 and u.max() < 1.0 and abs(float(u.mean())) < 0.01


def test_lsq_small_golden():
    z = np.load(os.path.join(GOLDEN, "lsq_small.npz"))
    seed = int(z["seed"])
    A = lsq.gen_matrix(seed, 0, z["A"].shape[0], z["A"].shape[1], "f32")
    assert np.array_equal(A.view(np.uint32), z["A"].view(np.uint32))
    g = lsq.shard_gradient(z["A"], z["b"], z["x"])
    assert np.array_equal(g, z["g"])
    # g = A^T (A x - b) by the definition, written out
    A64 = z["A"].astype(np.float64)
    g2 = sum((A64[r] @ z["x"] - z["b"][r]) * A64[r] for r in range(A64.shape[0]))
    assert lsq.rel_err(g2, g) < 1e-12


def test_golden_traces_regenerate():
    """The committed traces are exactly what the oracle produces now."""
    import importlib.util
    spec = importlib.util.spec_from_file_location("make_golden", os.path.join(GOLDEN, "make_golden.py"))
    mg = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mg)
    ref = json.load(open(os.path.join(GOLDEN, "traces.json")))["scenarios"]
    for sc in ref:
        got = mg.run_scenario(sc)
        assert got == sc["results"], sc["name"]


def test_golden_traces_satisfy_kmap2_properties():
    """kmap2.jl:50/:53/:60 hold on every committed trace (chunk epoch == repochs, >= nwait
    fresh, all inactive after waitall!)."""
    ref = json.load(open(os.path.join(GOLDEN, "traces.json")))["scenarios"]
    for sc in ref:
        ranks = sc.get("ranks", list(range(1, sc["n"] + 1)))
        consistent = True  # every dispatch so far sent its own epoch number
        for op, res in zip(sc["ops"], sc["results"]):
            if op["op"] == "asyncmap":
                consistent &= op.get("send") == res["epoch"]
            rep = res["repochs"]
            recv = np.asarray(res["recv"]).reshape(sc["n"], 3)
            for i, r in enumerate(rep):
                if r != sc.get("epoch0", 0):
                    assert recv[i, 0] == ranks[i]
                    if consistent:
                        assert recv[i, 2] == r
            if op["op"] == "waitall":
                assert not any(res["active"])
            elif isinstance(op["nwait"], int) and "epoch" not in op:
                assert sum(1 for r in rep if r == res["epoch"]) >= op["nwait"]
