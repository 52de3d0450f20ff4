"""Generate the committed golden fixtures under tests/golden/ from the ORACLE.

    python tests/golden/make_golden.py

The reference (Julia + MPI.jl) cannot run in this image, so these vectors come from the C
restatement in oracle/ (pinned by the reference's own kmap1/kmap2 properties, see
tests/test_oracle.py).  They freeze the oracle's behaviour so that (1) any change to it is
visible and (2) the product can be checked against fixed vectors without the oracle.

Files:
  philox_kat.json   published Random123 known-answer vectors for Philox4x32-10 (input data)
  traces.json       asyncmap!/waitall! traces of seeded scenarios (virtual clock)
  lsq_small.npz     a small least-squares shard: A, b, x and g = A^T(Ax - b) in fp64
"""
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(ROOT, "oracle"))

import lsq  # noqa: E402
import oracle as O  # noqa: E402

# Random123 kat_vectors, philox4x32 with 10 rounds: (ctr[4], key[2]) -> out[4]
PHILOX_KAT = [
    [[0x00000000, 0x00000000, 0x00000000, 0x00000000], [0x00000000, 0x00000000],
     [0x6627e8d5, 0xe169c58d, 0xbc57ac4c, 0x9b00dbd8]],
    [[0xffffffff, 0xffffffff, 0xffffffff, 0xffffffff], [0xffffffff, 0xffffffff],
     [0x408f276d, 0x41c83b0e, 0xa20bc7c6, 0x6d5451fd]],
    [[0x243f6a88, 0x85a308d3, 0x13198a2e, 0x03707344], [0xa4093822, 0x299f31d0],
     [0xd16cfe09, 0x94fdcceb, 0x5001e420, 0x24126ea1]],
]

MS = 1_000_000


def predicate(name):
    """nwait::Function variants used by the scenarios."""
    if name == "first":  # test/kmap2.jl:65
        return lambda epoch, repochs: bool(repochs[0] == epoch)
    if name.startswith("first_plus_"):  # BASELINE c4: worker 1 + any k others
        k = int(name.rsplit("_", 1)[1])
        return lambda epoch, repochs: bool(repochs[0] == epoch and int(np.sum(repochs == epoch)) >= k + 1)
    if name.startswith("count_"):
        k = int(name.rsplit("_", 1)[1])
        return lambda epoch, repochs: bool(int(np.sum(repochs == epoch)) >= k)
    raise KeyError(name)


def kmap2_ops(epochs=100):
    """test/kmap2.jl:20-73: 100 epochs nwait=2, 100x (nwait=1 + waitall!), 100 epochs f."""
    ops = [{"op": "asyncmap", "nwait": 2, "send": e} for e in range(1, epochs + 1)]
    for _ in range(epochs):
        ops.append({"op": "asyncmap", "nwait": 1, "send": epochs})
        ops.append({"op": "waitall"})
    ops += [{"op": "asyncmap", "nwait": "first", "send": epochs} for _ in range(epochs)]
    return ops


def run_scenario(sc, return_sim=False):
    """Run a scenario on the oracle; returns the list of per-op records (and the oracle's
    sim, whose observation log gives the gated-replay schedule, with return_sim)."""
    n, comm_n = sc["n"], sc.get("comm_workers", sc["n"])
    ranks = sc.get("ranks", list(range(1, n + 1)))
    kind = {"kmap2": O.ORC_WORKER_KMAP2, "tag": O.ORC_WORKER_TAG, "echo": O.ORC_WORKER_ECHO,
            "kmap1": O.ORC_WORKER_KMAP1}[sc["worker"]]
    dur = np.asarray(sc["durations_ns"], dtype=np.int64).reshape(comm_n, -1)
    # the oracle's sim addresses workers by pool position: give it the rows of the pool's ranks
    sim = O.OracleSim(n, kind, dur[np.asarray(ranks) - 1], sc.get("compute_ns", 0))
    pool = O.OraclePool(ranks, epoch0=sc.get("epoch0", 0), nwait=sc.get("default_nwait"))
    elems = sc.get("send_elems", 1)
    send = np.zeros(elems, dtype=np.float64)
    isend = np.zeros(n * elems)
    chunk = sc.get("chunk_elems", 3)
    recv = np.zeros(n * chunk)
    irecv = np.zeros(n * chunk)
    out = []
    for op in sc["ops"]:
        if op.get("advance_ns"):
            sim.advance(op["advance_ns"])
        t0 = sim.now
        if op["op"] == "waitall":
            O.waitall(pool, sim, recv, irecv)
        else:
            send[0] = op.get("send", 0)
            nw = op.get("nwait")
            nw = predicate(nw) if isinstance(nw, str) else nw
            O.asyncmap(pool, sim, send, recv, isend, irecv, nwait=nw, epoch=op.get("epoch"), tag=0)
        out.append({"repochs": pool.repochs.tolist(), "sepochs": pool.sepochs.tolist(),
                    "active": pool.active.astype(int).tolist(), "epoch": int(pool.epoch),
                    "latency_ns": [int(round(v * 1e9)) for v in pool.latency],
                    "t_start": int(t0), "t_end": int(sim.now),
                    "recv": recv.view(np.int64).tolist() if sc["worker"] == "tag" else recv.tolist()})
    return (out, sim) if return_sim else out


def _events(sc):
    n = sc["n"]
    sim_dur = np.asarray(sc["durations_ns"], dtype=np.int64).reshape(n, -1)
    sim = O.OracleSim(n, O.ORC_WORKER_TAG, sim_dur, sc.get("compute_ns", 0))
    pool = O.OraclePool(n)
    send, isend, recv, irecv = np.zeros(1), np.zeros(n), np.zeros(3 * n), np.zeros(3 * n)
    for op in sc["ops"]:
        if op["op"] == "waitall":
            O.waitall(pool, sim, recv, irecv)
        else:
            nw = op.get("nwait")
            O.asyncmap(pool, sim, send, recv, isend, irecv, nwait=predicate(nw) if isinstance(nw, str) else nw)
    return sim.events()


def min_completion_gap(sc):
    """Smallest distance between two task completion times of a scenario (virtual clock)."""
    done = sorted(e[3] for e in _events(sc))
    return int(min(np.diff(done))) if len(done) > 1 else 10**18


def separate(sc, gap):
    """Repair a schedule until every two completion times are >= gap apart: the later task
    of a close pair is lengthened by 2*gap, then the scenario is re-simulated."""
    n = sc["n"]
    d = np.asarray(sc["durations_ns"], dtype=np.int64).reshape(n, -1)
    for _ in range(5000):
        sc["durations_ns"] = d.ravel().tolist()
        ev = sorted(_events(sc), key=lambda e: e[3])
        bad = [(a, b) for a, b in zip(ev, ev[1:]) if b[3] - a[3] < gap]
        if not bad:
            return sc
        w, t = bad[0][1][0], bad[0][1][1]
        assert t - 1 < d.shape[1], "schedule too short for the scenario"
        d[w, t - 1] += 2 * gap
    raise RuntimeError("could not separate the schedule")


def scenarios():
    rng = np.random.default_rng(20261015)
    sc = []
    for n in (2, 9):  # test/runtests.jl:29-45 runs kmap2 with 3 and 10 ranks
        # sleep(max(rand()/10, 0.005)) (test/kmap2.jl:95), microsecond resolution
        d = np.maximum(rng.random((n, 128)) / 10, 0.005)
        sc.append({"name": f"kmap2_n{n}", "n": n, "worker": "kmap2",
                   "durations_ns": (np.round(d * 1e6).astype(np.int64) * 1000).ravel().tolist(),
                   "ops": kmap2_ops()})
    # ties everywhere: durations from {1,2,3} ms
    n = 5
    d = rng.integers(1, 4, size=(n, 16)) * MS
    sc.append({"name": "tag_ties", "n": n, "worker": "kmap2", "durations_ns": d.ravel().tolist(),
               "ops": [{"op": "asyncmap", "nwait": 3, "send": e} for e in range(1, 41)] + [{"op": "waitall"}]})
    # nwait = 0 and nwait = n, with coordinator time between calls
    d = rng.integers(1, 20, size=(n, 16)) * MS
    ops = []
    for e in range(1, 31):
        ops.append({"op": "asyncmap", "nwait": int(e % 3 == 0) * n, "send": e, "advance_ns": int(rng.integers(0, 8)) * MS})
    ops.append({"op": "waitall"})
    sc.append({"name": "tag_nwait_0_and_n", "n": n, "worker": "kmap2", "durations_ns": d.ravel().tolist(), "ops": ops})
    # MPIAsyncPool([1, 4, 5]) on a 5-worker comm (src/MPIAsyncPools.jl:21 docstring)
    d = rng.integers(1, 30, size=(5, 16)) * MS
    sc.append({"name": "tag_rank_subset", "n": 3, "comm_workers": 5, "ranks": [1, 4, 5], "worker": "kmap2",
               "durations_ns": d.ravel().tolist(),
               "ops": [{"op": "asyncmap", "nwait": 2, "send": e} for e in range(1, 31)]})
    # explicit epochs that repeat and go backwards (:68, :87 do not validate epoch)
    d = rng.integers(1, 30, size=(n, 16)) * MS
    eps = [1, 1, 2, 5, 3, 3, 3, 4, 10, 2, 2, 7, 7, 8, 9, 9, 1, 12, 12, 13]
    sc.append({"name": "tag_epoch_games", "n": n, "worker": "kmap2", "durations_ns": d.ravel().tolist(),
               "epoch0": 0, "ops": [{"op": "asyncmap", "nwait": 2, "epoch": e, "send": e} for e in eps]})
    # predicate: worker 1 + any 3 others (BASELINE c4), one slow straggler
    d = rng.integers(2, 12, size=(6, 32)) * MS
    d[3] *= 7
    sc.append({"name": "tag_pred_first_plus_3", "n": 6, "worker": "kmap2", "durations_ns": d.ravel().tolist(),
               "ops": [{"op": "asyncmap", "nwait": "first_plus_3", "send": e} for e in range(1, 51)]})
    # heavy stragglers: stale re-dispatch in phase 3 (:177-184)
    d = rng.integers(1, 10, size=(8, 32)) * MS
    d[[2, 5]] *= 13
    sc.append({"name": "tag_stale_redispatch", "n": 8, "worker": "kmap2", "durations_ns": d.ravel().tolist(),
               "ops": [{"op": "asyncmap", "nwait": 6, "send": e} for e in range(1, 61)] + [{"op": "waitall"}]})
    # GPU-timeable scenarios: every completion time >= 4 ms from every other one
    for name, n, nw, k in (("gpu_sep_nwait2", 4, 2, 24), ("gpu_sep_pred", 4, "count_3", 20),
                           ("gpu_sep_nwait6of8", 8, 6, 16)):
        d = rng.integers(5, 41, size=(n, 64)) * MS
        s = {"name": name, "n": n, "worker": "kmap2", "durations_ns": d.ravel().tolist(),
             "ops": [{"op": "asyncmap", "nwait": nw, "send": e} for e in range(1, k + 1)] + [{"op": "waitall"}]}
        separate(s, 4 * MS)
        s["min_gap_ns"] = min_completion_gap(s)
        sc.append(s)
    # BASELINE configs[3] (c4: worker 1 + 5 of the other 7, stale results folded in),
    # configs[0] (c1: 3 workers, nwait 2, the 10 epochs of examples/iterative_example.jl:37)
    # and configs[2] (c3: 6 of 8)
    # replayed on device with least-squares workers (tests/test_gpu_configs.py); own seed so
    # the scenarios above stay unchanged
    rng2 = np.random.default_rng(20261016)
    for name, n, nw, k, drain in (("gpu_sep_c4_first_plus_5", 8, "first_plus_5", 12, True),
                                  ("gpu_sep_c1", 3, 2, 10, False),
                                  ("gpu_sep_c3", 8, 6, 12, False)):
        d = rng2.integers(5, 41, size=(n, 64)) * MS
        s = {"name": name, "n": n, "worker": "kmap2", "durations_ns": d.ravel().tolist(),
             "ops": [{"op": "asyncmap", "nwait": nw, "send": e} for e in range(1, k + 1)] +
                    ([{"op": "waitall"}] if drain else [])}
        separate(s, 4 * MS)
        s["min_gap_ns"] = min_completion_gap(s)
        sc.append(s)
    return sc


def main():
    with open(os.path.join(HERE, "philox_kat.json"), "w") as f:
        json.dump({"source": "Random123 kat_vectors, philox4x32 R=10", "vectors": PHILOX_KAT}, f, indent=1)
    out = []
    for s in scenarios():
        s = dict(s)
        s["results"] = run_scenario(s)
        out.append(s)
    with open(os.path.join(HERE, "traces.json"), "w") as f:
        json.dump({"generator": "tests/golden/make_golden.py (oracle/asyncpool_oracle.c)", "scenarios": out}, f)
    seed, rows, cols = 7, 96, 256
    A = lsq.gen_matrix(seed, 0, rows, cols, "f32")
    b = lsq.gen_vector(seed, 0, rows, "f32")
    x = lsq.gen_vector(seed, 0, cols, "f32", stream=lsq.STREAM_X, scale=0.25)
    g = lsq.shard_gradient(A, b, x)
    np.savez_compressed(os.path.join(HERE, "lsq_small.npz"), seed=seed, A=A, b=b, x=x, g=g)
    print("wrote", len(out), "scenarios")


if __name__ == "__main__":
    main()
