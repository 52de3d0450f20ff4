"""Gated device replays (mpa_comm_set_gate on the HIP transport), against the oracle.

The oracle runs each scenario on its virtual clock; its observation log gives the gate
schedule (tests/gated.py): at every Test!/Waitany!/Waitall! the device shows exactly the
completions the oracle saw there, so the HIP transport must reproduce the oracle's trace
bit for bit whatever order its kernels finish in -- ties included (released together,
Waitany! takes the lowest index, src/MPIAsyncPools.jl:161), stale harvests and
re-dispatches in the wait loop (:177-184), phase-1 harvests (:91-114) and waitall!
(:195-224).

  * every golden scenario of tests/golden/traces.json (14: kmap2 at 3 and 10 ranks, ties,
    nwait 0 and n, rank subsets, explicit epochs, predicates, stale re-dispatch, the six
    GPU-timeable schedules) with kmap2 device workers whose injected delays ARE the
    committed durations (no scaling): repochs / sepochs / active / recvbuf bit-exact after
    every call, latency = host time dispatch -> harvest close to the oracle's;
  * random schedules with ties, run with no delays and with scrambling delays;
  * BASELINE configs[4]'s shape (c5): 8 batched bf16 least-squares workers on uneven shards,
    nwait 7 of 8, undelayed, so stale replies arrive inside the wait loop and their
    re-dispatches are HELD for the next batched launch (transport_hip.cpp flush_stale);
    run with the hold (default) and MPA_HOLD=0: the oracle's repochs / active after every
    call, every chunk equal to the gradient of the X sent at its epoch, the iterate equal to
    a numpy replay of the update, and both runs on the same trace and iterate (1e-5);
  * the same for fp32 least-squares workers (c2's kernel) on uneven shards, nwait 5 of 8.
"""
import numpy as np
import pytest

import gated

pytestmark = pytest.mark.gpu
SCEN = gated.scenarios()
MS = 1_000_000


@pytest.fixture(scope="module")
def M(built):
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU visible")
    import mpiasyncpools
    gated.warm_kernels(mpiasyncpools, torch, 4)
    return mpiasyncpools


@pytest.fixture(scope="module")
def watchdog():
    w = gated.HostWatchdog()
    yield w
    w.close()


def _kmap2_run(M, sc, delays, own_stream=False):
    """One gated replay of a kmap2 scenario in this process (gated.kmap2_replay)."""
    got, counters = gated.kmap2_replay(M, sc, delays, own_stream)
    _TRACE[0] = counters.pop("trace", None)
    _LAST.clear()
    _LAST.update(counters)
    return got


_LAST = {}  # the transport's counters of the last replay (failure messages)
_TRACE = [None]  # the task trace of the last replay (mpa_comm_trace)


def _latency_check(name, sc, got):
    """(ok, summary) of a replay's latencies: every hop on the device's own clock within 1 ms
    (gated.hop_check: the latency is harvest - dispatch, each task completes its schedule
    duration after its dispatch, each harvest follows the device event the oracle harvested it
    at), and the latencies themselves against the oracle's: median |device - oracle| < 0.2 ms
    (their maximum is reported: it holds the coordinator chain's drift, see hop_check)."""
    trace = _TRACE[0]
    dev = []
    for g, r in zip(got, sc["results"]):
        for v, lat in zip(g["latency_s"], r["latency_ns"]):
            if lat > 0:
                dev.append(abs(v - lat / 1e9))
    dev = np.asarray(dev)
    bad, hops = gated.hop_check(sc, got, trace)
    msg = "%s: hops p50/p99/max ms %s, misses %s; latency |device - oracle| median %.3f ms, max %.3f ms" % (
        name, hops, bad[:6], 1e3 * np.median(dev), 1e3 * dev.max())
    if bad:  # the transport's view and the split of the missed harvests
        import os
        msg += "; counters %s; loadavg %s; task trace of the misses %s" % (
            dict(_LAST), tuple(round(x, 1) for x in os.getloadavg()),
            gated.explain_misses(got, trace, [(k, i, d, t) for _, k, i, d, t in bad if d is not None]))
    msg += "; trace p50/p99/max ms %s" % gated.trace_stats(trace)
    return not bad and np.median(dev) < 0.2e-3, msg


@pytest.mark.timing
@pytest.mark.parametrize("name", [s["name"] for s in SCEN])
def test_golden_scenario_gated_on_device(M, watchdog, name):
    """Every golden scenario at its committed durations: the trace bit-exact; every hop of the
    device timeline within 1 ms on the device's own clock -- latency = harvest - dispatch
    (src/MPIAsyncPools.jl:105,164,215), each task's completion its schedule duration after its
    dispatch, each harvest right after the device event the oracle harvested it at
    (_latency_check, gated.hop_check) -- and the median |device - oracle| latency < 0.2 ms.
    Round 4 compared each latency with the oracle's directly (1 ms + 50 us per completion in its
    window) and re-ran misses up to eight times: the task trace showed its steady miss
    (gpu_sep_nwait2, -1.3 ms every run) to be the drift between two chains of the timeline, not a
    late task or harvest (hop_check).  A miss now gets ONE rerun, in this process, after a 10 s
    pause (a stall of the box: the message carries the host watchdog's reading and the split of
    each missed hop from the task trace).  The harness runs on a non-blocking stream of its own
    (gated.kmap2_replay), so the injected delays run as device deadlines (deadline_kernel, round
    6: no host thread wakes for them; the 4 misses of round 5 were the host timer waking 1.3-18
    ms late on loaded boxes); the NULL-stream caller (host timer) is covered by the random
    scenarios and the config replays.  The test is marked `timing` and runs last (tests/conftest.py)."""
    sc = next(s for s in SCEN if s["name"] == name)
    comm_n = sc.get("comm_workers", sc["n"])
    dur = np.asarray(sc["durations_ns"], dtype=np.int64).reshape(comm_n, -1)
    import time
    msgs = []
    watchdog.take()
    for attempt in range(2):
        if attempt:
            time.sleep(10)
            watchdog.take()
        got = _kmap2_run(M, sc, dur, own_stream=True)
        assert gated.mismatches(name, got, sc["results"]) == []
        ok, msg = _latency_check(name, sc, got)
        worst, over = watchdog.take()
        msg += "; host watchdog worst oversleep %.2f ms (%d over 2 ms)" % (worst, over)
        msgs.append(msg)
        print(msg)
        if ok:
            break
    assert ok, msgs


@pytest.mark.parametrize("seed", range(6))
def test_random_scenario_gated_on_device(M, seed):
    """Random schedules full of ties: with no delays, and with 0-400 us delays that scramble
    the physical completion order against the schedule."""
    sc = gated.random_scenario(seed)
    ref, _ = gated.oracle_gate(sc)
    rng = np.random.default_rng(seed)
    for delays in (None, rng.integers(0, 400, size=(sc["n"], 23)) * 1000):
        got = _kmap2_run(M, sc, delays)
        assert gated.mismatches(sc["name"], got, ref) == []


# ---- least-squares workers, k-of-n with stale replies in the wait loop -------------------

ROWS = [2000, 3100, 1500, 4113, 2500, 1000, 3500, 2200]  # uneven shards (8 workers)


def _straggler_scenario(n, nwait, epochs, seed):
    """A schedule (oracle durations) with stragglers that miss an epoch and reply inside a
    later call's wait loop, so that call harvests a stale chunk and re-dispatches."""
    rng = np.random.default_rng(seed)
    d = rng.integers(4, 10, size=(n, 64)) * MS
    slow = rng.random((n, 64)) < 0.2
    d[slow] *= rng.integers(2, 4, size=int(slow.sum()))
    ops = [{"op": "asyncmap", "nwait": nwait, "send": e} for e in range(1, epochs + 1)] + [{"op": "waitall"}]
    return {"name": f"straggle{seed}", "n": n, "worker": "kmap2", "durations_ns": d.ravel().tolist(), "ops": ops}


def _stale_redispatches(sc):
    """Posts the oracle made inside a wait loop (a stale harvest's re-dispatch, :177-184)."""
    import oracle as O
    mg = gated.make_golden()
    _, sim = mg.run_scenario(sc, return_sim=True)
    count, in_wait = 0, False
    for kind, *_ in sim.observations():
        if kind == O.OBS_WAIT:
            in_wait = True
        elif kind in (O.OBS_CALL, O.OBS_WAITALL):
            in_wait = False
        elif kind == O.OBS_POST and in_wait:
            count += 1
    return count


def _gated_descent(M, torch, batched, sc, hold, monkeypatch):
    """Python coordinator loop (examples/iterative_example.jl:37-47 with nwait k) over the
    gated schedule; checks every call against the oracle, then every chunk and the iterate."""
    import lsq
    if hold:
        monkeypatch.delenv("MPA_HOLD", raising=False)
    else:
        monkeypatch.setenv("MPA_HOLD", "0")
    ref, sched = gated.oracle_gate(sc)
    n, K, seed, eta = sc["n"], 64, 77, 1e-4
    cols = 256 if batched else 512
    tot = sum(ROWS)
    off = np.concatenate([[0], np.cumsum(ROWS)])
    if batched:
        A = lsq.gen_matrix(seed, 0, tot, cols, "bf16")
        B = lsq.gen_matrix(seed, 0, tot, K, "bf16", stream=lsq.STREAM_B, scale=np.float32(1.0))
    else:
        A = lsq.gen_matrix(seed, 0, tot, cols, "f32")
        B = lsq.gen_vector(seed, 0, tot, "f32")
    comm = M.DeviceComm(n)
    keep = []
    for r in range(1, n + 1):
        a, b = A[off[r - 1]:off[r]], B[off[r - 1]:off[r]]
        if batched:
            Ad = torch.from_numpy(np.ascontiguousarray(a).view(np.int16)).cuda().view(torch.bfloat16)
            Bd = torch.from_numpy(np.ascontiguousarray(b).view(np.int16)).cuda().view(torch.bfloat16)
            comm.set_task_lsq_batch(r, Ad, Bd)
        else:
            Ad, Bd = torch.from_numpy(np.ascontiguousarray(a)).cuda(), torch.from_numpy(np.ascontiguousarray(b)).cuda()
            comm.set_task_lsq(r, Ad, Bd)
        keep.append((Ad, Bd))
    comm.set_gate(*sched)
    pool = M.MPIAsyncPool(n)
    m = cols * (K if batched else 1)
    x = torch.zeros(m, dtype=torch.float32, device="cuda")
    msg = torch.zeros(m, dtype=torch.bfloat16, device="cuda") if batched else x
    isend = torch.zeros(n * m, dtype=msg.dtype, device="cuda")
    recv = torch.zeros(n * m, dtype=torch.float32, device="cuda")
    irecv = torch.zeros_like(recv)
    sent, got, reps, ws = {}, [], [], []
    steps = [(op, r) for op, r in zip(sc["ops"], ref) if op["op"] == "asyncmap"]
    for k, (op, r) in enumerate(steps):
        epoch = k + 1
        sent[epoch] = msg.clone()
        rep = M.asyncmap_(pool, msg, recv, isend, irecv, comm, nwait=op["nwait"]).copy()
        assert rep.tolist() == r["repochs"], (sc["name"], hold, k, rep.tolist(), r["repochs"])
        assert pool.active.astype(int).tolist() == r["active"], (sc["name"], hold, k)
        got.append(recv.clone())
        w = (rep == epoch).astype(np.float64)
        w *= n / w.sum()
        if batched:
            comm.lsqb_update(x, msg, recv, n, w, eta)
        else:
            comm.lsq_update(x, recv, n, w, eta)
        reps.append(rep)
        ws.append(w)
    M.waitall_(pool, recv, irecv)
    assert pool.repochs.tolist() == ref[-1]["repochs"] and not pool.active.any()
    torch.cuda.synchronize()
    # every chunk is the gradient of the message of its epoch (kmap2.jl:50, numerically)
    x_np, worst = np.zeros(m), 0.0
    for k, (rep, w, rcv) in enumerate(zip(reps, ws, got)):
        epoch = k + 1
        chunks = rcv.cpu().numpy().reshape(n, m).astype(np.float64)
        for i in range(n):
            if rep[i] == 0:
                continue
            s = sent[int(rep[i])]
            if batched:
                X = s.cpu().view(torch.int16).numpy().view(np.uint16).reshape(cols, K)
                g = lsq.batched_shard_gradient(A[off[i]:off[i + 1]], B[off[i]:off[i + 1]], X).ravel()
            else:
                g = lsq.shard_gradient(A[off[i]:off[i + 1]], B[off[i]:off[i + 1]], s.cpu().numpy())
            err = lsq.rel_err(chunks[i], g)
            worst = max(worst, err)
            assert err <= 1e-5, (sc["name"], hold, k, i, err)
        x_np = x_np - eta * (w[:, None] * chunks).sum(0)
    assert lsq.rel_err(x.cpu().numpy().astype(np.float64), x_np) <= 1e-5
    held = {k: comm.counter(k) for k in ("held", "held_joined", "held_alone", "gate_steps")}
    comm.shutdown()
    comm.close()
    return x, reps, worst, held


@pytest.mark.parametrize("batched", [True, False], ids=["c5_bf16_nwait7", "f32_nwait5"])
def test_gated_lsq_k_of_n_with_held_redispatch(M, monkeypatch, batched):
    import lsq
    import torch
    nwait = 7 if batched else 5
    sc = _straggler_scenario(8, nwait, 24, seed=31 if batched else 32)
    nstale = _stale_redispatches(sc)
    assert nstale >= 3, nstale  # the schedule exercises the stale re-dispatch path
    x_hold, reps_hold, worst, held = _gated_descent(M, torch, batched, sc, True, monkeypatch)
    x_now, reps_now, _, held_now = _gated_descent(M, torch, batched, sc, False, monkeypatch)
    # the hold ran: stale re-dispatches were held, and some joined a later batched launch
    assert held["held"] >= 1 and held["held_joined"] >= 1, held
    assert held["held"] == held["held_joined"] + held["held_alone"], held
    assert held_now["held"] == 0, held_now
    assert [r.tolist() for r in reps_hold] == [r.tolist() for r in reps_now]
    # the same chunks feed the same updates, but not bit for bit: a launch deals its grid
    # over the tasks it carries, and holding changes which tasks share a launch, so a
    # gradient's reduction order (not its inputs) differs between the two runs
    d = lsq.rel_err(x_hold.cpu().numpy().astype(np.float64), x_now.cpu().numpy().astype(np.float64))
    assert d <= 1e-5, d
    print("%s: %d stale re-dispatches, %s, worst chunk rel err %.3e, iterate hold vs MPA_HOLD=0 rel %.3e"
          % (sc["name"], nstale, held, worst, d))


def test_gated_native_descent_defers_held_redispatch(M, monkeypatch):
    """The native descent loop (mpa_lsq_descent) under the same gated k-of-n schedule: its
    held stale re-dispatches do not launch an exchange of their own -- their messages (the
    iterate before the next update) and the pending harvests join the next epoch step
    (EpochArgs dst0) -- and it ends where the Python loop over the same schedule ends: the
    same repochs, the iterate within the gradients' reduction-order tolerance."""
    import lsq
    import torch
    n, nwait, epochs = 8, 5, 24
    sc = _straggler_scenario(n, nwait, epochs, seed=32)
    assert _stale_redispatches(sc) >= 3
    x_py, reps_py, _, _ = _gated_descent(M, torch, False, sc, True, monkeypatch)
    monkeypatch.delenv("MPA_HOLD", raising=False)
    monkeypatch.setenv("MPA_WAIT_TIMEOUT_S", "30")
    ref, sched = gated.oracle_gate(sc)
    seed, eta, cols = 77, 1e-4, 512
    off = np.concatenate([[0], np.cumsum(ROWS)])
    A = lsq.gen_matrix(seed, 0, int(off[-1]), cols, "f32")
    B = lsq.gen_vector(seed, 0, int(off[-1]), "f32")
    comm = M.DeviceComm(n)
    keep = []
    for r in range(1, n + 1):
        Ad = torch.from_numpy(np.ascontiguousarray(A[off[r - 1]:off[r]])).cuda()
        Bd = torch.from_numpy(np.ascontiguousarray(B[off[r - 1]:off[r]])).cuda()
        comm.set_task_lsq(r, Ad, Bd)
        keep.append((Ad, Bd))
    comm.set_gate(*sched)
    pool = M.MPIAsyncPool(n)
    x = torch.zeros(cols, dtype=torch.float32, device="cuda")
    isend = torch.zeros(n * cols, dtype=torch.float32, device="cuda")
    recv = torch.zeros(n * cols, dtype=torch.float32, device="cuda")
    irecv = torch.zeros_like(recv)
    M.lsq_descent(pool, comm, x, recv, isend, irecv, nwait, eta, epochs)
    deferred = comm.counter("stale_deferred")
    assert pool.repochs.tolist() == reps_py[-1].tolist()
    M.waitall_(pool, recv, irecv)
    torch.cuda.synchronize()
    assert pool.repochs.tolist() == ref[-1]["repochs"] and not pool.active.any()
    assert deferred >= 1, deferred
    d = lsq.rel_err(x.cpu().numpy().astype(np.float64), x_py.cpu().numpy().astype(np.float64))
    assert d <= 1e-5, d
    comm.shutdown()
    comm.close()
