"""Gated replay (mpa_comm_set_gate), shared by the CPU test on the HOST transport
(tests/test_gate_cpu.py) and the device tests on the HIP transport (tests/test_gpu_gated.py).

The oracle runs a scenario on its virtual clock and logs, at every observation point of
the state machine (before phase 1 of asyncmap!, each Waitany!, each Waitall!), which task
completions it could see there (oracle/oracle.py OracleSim.gate_schedule).  The product
is handed that schedule: a request reads as complete only once its task has finished AND
the schedule has released it, so every Test!/Waitany!/Waitall! sees the oracle's set of
completions and the product must reproduce the oracle's trace bit for bit, whatever order
the tasks really finish in (ties included: released together, Waitany! must take the
lowest index, src/MPIAsyncPools.jl:161 over MPICH's array scan).
"""
import contextlib
import gc
import importlib.util
import json
import os
import time

import numpy as np

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def make_golden():
    spec = importlib.util.spec_from_file_location("make_golden", os.path.join(GOLDEN, "make_golden.py"))
    mg = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mg)
    return mg


def scenarios():
    return json.load(open(os.path.join(GOLDEN, "traces.json")))["scenarios"]


def oracle_gate(sc):
    """(oracle records, gate schedule) of a scenario; the schedule is in comm ranks."""
    mg = make_golden()
    out, sim = mg.run_scenario(sc, return_sim=True)
    n = sc["n"]
    return out, sim.gate_schedule(sc.get("ranks", list(range(1, n + 1))))


def latency_tolerance(sc, slack_s=1e-3, per_event_s=50e-6):
    """Per (op, pool position) of every harvest: how far the device's latency (host time,
    dispatch -> harvest) may sit from the oracle's.  The oracle's coordinator spends no time
    and its tasks no launch overhead; on the device every task completion between a task's
    dispatch and its harvest carries ~+-50 us (a launch's overhead against the 35 us taken out
    of its sleep, the harness's time between calls), and the gate releases the harvest only
    once those completions it waits for have happened.  So: 1 ms + 50 us per task completion
    on the oracle's clock inside the harvested task's dispatch -> harvest window."""
    mg = make_golden()
    out, sim = mg.run_scenario(sc, return_sim=True)
    ev = sim.events()
    done = np.sort(np.asarray([e[3] for e in ev], dtype=np.int64))
    by_lat = {}
    for w, t, post, d, seen in ev:
        by_lat.setdefault((w, seen - post), (post, seen))
    tol = {}
    for k, r in enumerate(out):
        for i, lat in enumerate(r["latency_ns"]):
            if lat <= 0:
                continue
            post, seen = by_lat[(i, lat)]
            inside = int(np.searchsorted(done, seen, side="right") - np.searchsorted(done, post, side="right"))
            tol[(k, i)] = slack_s + per_event_s * max(inside - 1, 0)
    return tol


@contextlib.contextmanager
def no_gc():
    """Python's cyclic garbage collector off for a timed stretch (collected once before): a
    generation-2 pass over the heap of a long pytest process takes milliseconds to tens of
    them and pauses the thread that dispatches and harvests, which the pool's host-time
    latencies then record (r04final3: 5-46 ms misses with the host watchdog and the
    transport's timer on time, profiles/r04_gated_stall.txt)."""
    gc.collect()
    was = gc.isenabled()
    gc.disable()
    try:
        yield
    finally:
        if was:
            gc.enable()


def replay(M, sc, comm, buf, host, predicate, snap=None):
    """Run a scenario's ops on the product through `comm`; the oracle's record layout.
    `buf(k)` makes a float64 buffer of k elements, `host(b)` reads one back as numpy,
    `snap(b)` (default: host) keeps a copy of recvbuf after each call -- a device clone, read
    back after the last call, so the harness adds no host sync between calls (its time
    between calls delays the next dispatch, which the oracle's coordinator does not)."""
    snap = snap or host
    n = sc["n"]
    ranks = sc.get("ranks", list(range(1, n + 1)))
    pool = M.MPIAsyncPool(ranks, epoch0=sc.get("epoch0", 0), nwait=sc.get("default_nwait"))
    elems, chunk = sc.get("send_elems", 1), sc.get("chunk_elems", 3)
    send, isend = buf(elems), buf(n * elems)
    recv, irecv = buf(n * chunk), buf(n * chunk)
    out = []
    for op in sc["ops"]:
        if op.get("advance_ns"):  # the coordinator's own time between calls (make_golden.py run_scenario)
            t_end = time.perf_counter_ns() + int(op["advance_ns"])
            while time.perf_counter_ns() < t_end:
                pass
        t0 = time.perf_counter()
        t0_ns = time.perf_counter_ns()  # CLOCK_MONOTONIC, the transport's steady clock (task trace)
        if op["op"] == "waitall":
            M.waitall_(pool, recv, irecv)
        else:
            send[0] = float(op.get("send", 0))
            nw = op.get("nwait")
            nw = predicate(nw) if isinstance(nw, str) else nw
            M.asyncmap_(pool, send, recv, isend, irecv, comm, nwait=nw, epoch=op.get("epoch"), tag=0)
        call_ms = (time.perf_counter() - t0) * 1e3
        out.append({"repochs": pool.repochs.tolist(), "sepochs": pool.sepochs.tolist(),
                    "active": pool.active.astype(int).tolist(), "epoch": int(pool.epoch),
                    "latency_s": pool.latency.tolist(), "recv": snap(recv), "call_ms": call_ms,
                    "t_ns": (t0_ns, time.perf_counter_ns()), "ranks": list(ranks),
                    "stimestamps": pool.stimestamps.tolist()})
    for r in out:
        r["recv"] = np.asarray(host(r["recv"])).tolist()
    return out, pool


KEYS = ("repochs", "sepochs", "active", "epoch", "recv")


def mismatches(name, got, ref):
    """Every (op, field) where the product's trace differs from the oracle's."""
    bad = []
    for k, (g, r) in enumerate(zip(got, ref)):
        for key in KEYS:
            if g[key] != r[key]:
                bad.append((name, k, key, g[key], r[key]))
    if len(got) != len(ref):
        bad.append((name, "ops", len(got), len(ref)))
    return bad


def kmap2_replay(M, sc, delays, own_stream=False):
    """One gated replay of a kmap2 scenario on device workers whose injected delays are
    `delays` (workers x tasks, ns; None: none): (the oracle-layout record, the transport's
    counters).  own_stream: the harness (its buffers, the send writes, the recvbuf snapshots)
    and the coordinator's copies run on a non-blocking stream of their own, as a GPU caller
    of the pool would keep them: on the legacy NULL stream every harness op between two calls
    also orders against every worker stream.  The whole replay runs with Python's GC off."""
    import torch
    ctx = torch.cuda.stream(torch.cuda.Stream()) if own_stream else contextlib.nullcontext()
    with ctx, no_gc():
        _, sched = oracle_gate(sc)
        comm_n = sc.get("comm_workers", sc["n"])
        comm = M.DeviceComm(comm_n)
        for r in range(1, comm_n + 1):
            comm.set_task(r, "kmap2")
            if delays is not None:
                comm.set_delays(r, delays[r - 1])
        comm.set_gate(*sched)
        comm.set_trace(TRACE_CAP)

        def buf(k):
            return torch.zeros(k, dtype=torch.float64, device="cuda")
        got, pool = replay(M, sc, comm, buf, lambda t: t.cpu().numpy(), make_golden().predicate,
                           snap=lambda t: t.clone())
        counters = {k: comm.counter(k) for k in ("timer_late", "queues", "shared_worker_streams")}
        counters["trace"] = comm.trace(TRACE_CAP)
        comm.shutdown()
        comm.close()
        torch.cuda.current_stream().synchronize()
    return got, counters


TRACE_CAP = 1 << 14
F = {k: j for j, k in enumerate(("rank", "seq", "post", "due", "call", "ret", "start", "pub", "gate", "seen", "harvest"))}
LEAD_NS = 35_000  # the transport's default MPA_DELAY_LEAD_NS (host timer)
DEADLINE_LEAD_NS = 8_000  # ... MPA_DEADLINE_LEAD_NS (a task queued behind a device deadline)


def task_parts(e):
    """(ms) where a task's time went against the oracle's clock: timer (the launch call against
    its due time less the launch lead; a task queued behind a device deadline at its post has
    none: its `deadline` part is the kernel's start against its due time less that lead), launch
    (the call itself), queue (call returned -> kernel started), kernel, visible (completion store,
    or the gate step's start if that came later -> the gate saw it: the coordinator's own
    lateness), harvest (seen -> taken); `late` = completion store - due (the task's own
    lateness)."""
    ms = lambda a, b: round((e[F[a]] - e[F[b]]) / 1e6, 3) if e[F[a]] and e[F[b]] else None
    due = e[F["due"]]
    delayed = due - e[F["post"]] > LEAD_NS
    # launched at its post, long before its due time: it waited behind a deadline_kernel
    on_device = delayed and e[F["call"]] and e[F["call"]] < due - LEAD_NS - 500_000
    p = {"task": "r%d#%d" % (e[F["rank"]], e[F["seq"]]),
         "timer": round((e[F["call"]] - (due - LEAD_NS)) / 1e6, 3) if delayed and e[F["call"]] and not on_device else None,
         "deadline": round((e[F["start"]] - (due - DEADLINE_LEAD_NS)) / 1e6, 3) if on_device and e[F["start"]] else None,
         "launch": ms("ret", "call"), "queue": ms("start", "ret"), "kernel": ms("pub", "start"),
         "visible": (round((e[F["seen"]] - max(e[F["pub"]], e[F["gate"]])) / 1e6, 3)
                     if e[F["seen"]] and e[F["pub"]] else None),
         "harvest": ms("harvest", "seen"), "late": ms("pub", "due")}
    return p


def hop_check(sc, got, trace, task_tol=1e-3, obs_tol=1e-3, lat_tol=50e-6):
    """Per-hop latency fidelity of a gated device replay against the oracle (tests/test_gpu_gated.py).

    The device's latency of a harvest, like the reference's, is (harvest time) - (dispatch time)
    (src/MPIAsyncPools.jl:105,164,215).  Its distance to the oracle's is the difference of two
    drifts of the device timeline against the virtual clock -- at the dispatch and at the
    harvest -- and those drifts accumulate along DIFFERENT chains: a re-dispatch inside the wait
    loop (:177-184) runs on its worker's own chain of completions, a call's posts on the
    coordinator's chain (the oracle's coordinator takes no time).  gpu_sep_nwait2's final
    Waitall! harvests worker 1 at worker 4's completion: -1.3 ms against the oracle at every run
    on the device (-3.4 ms over the HOST transport on CPU, where each hop costs more) with every
    task and every observation on time (round 4's "residual miss", round 5's task trace).  So
    the check is per hop, on the device's own clock (the task trace, mpa_comm_trace), for every
    harvested task:

      * latency semantics: pool.latency = trace harvest - trace post (within lat_tol);
      * the task: its completion store - (its dispatch + its schedule duration)  (task_tol)
        -- the injected straggler delay IS the schedule;
      * the harvest: its time - the latest of the device time of the event the oracle harvested
        it at (the completion store of the task(s) whose virtual completion is the oracle's
        observation time; where none is, a phase-1 Test!, the call's start), the start of the
        call that harvested it and the call's previous harvest (obs_tol): a call that starts after
        its trigger because the coordinator's chain drifted (the previous calls' hops), or a
        harvest held back by the one before it (whose task the drift posted late), is not this
        hop's lateness.

    The coordinator's own time between calls (the harness's, beside the oracle's advance_ns)
    is reported in the stats ("between_calls"), not held to a bound.

    Every traced task the device harvested is matched to the oracle's event of the same worker
    and task number (no matching by latency value: one worker's tasks can share a latency), and
    the op that harvested it is the call whose host-time window holds its harvest.

    Returns (misses, stats): misses are (kind, op, pool position, ms, tolerance ms); stats the
    p50 / p99 of |hop| / max of |hop| of each hop in ms."""
    mg = make_golden()
    _, sim = mg.run_scenario(sc, return_sim=True)
    events, done_at = {}, {}
    for w, t, post, d, seen in sim.events():
        events[(w, t)] = (post, d, seen)
        done_at.setdefault(d, []).append((w, t))
    n = sc["n"]
    ranks = list(sc.get("ranks", list(range(1, n + 1))))
    pos_of = {r: i for i, r in enumerate(ranks)}
    tr = {(int(e[F["rank"]]), int(e[F["seq"]])): e for e in trace}
    starts = np.asarray([g["t_ns"][0] for g in got], dtype=np.int64)
    bad = []
    hops = {"latency": [], "task": [], "harvest": []}
    # the call that harvested each task; a worker harvested twice in one call (a stale harvest,
    # its re-dispatch and the fresh one, :161-184) shows the later latency after the call
    last = {}
    for (rank, t), e in tr.items():
        if e[F["harvest"]] and rank in pos_of:
            k = int(np.searchsorted(starts, e[F["harvest"]], side="right")) - 1
            if k >= 0 and e[F["harvest"]] >= last.get((k, pos_of[rank]), (0, 0))[0]:
                last[(k, pos_of[rank])] = (e[F["harvest"]], t)
    for (rank, t), e in sorted(tr.items()):
        if not e[F["harvest"]] or rank not in pos_of or (pos_of[rank], t) not in events:
            continue  # never harvested (still in flight at the end), or another pool's
        i = pos_of[rank]
        post, d, seen = events[(i, t)]
        k = int(np.searchsorted(starts, e[F["harvest"]], side="right")) - 1  # the call that harvested it
        if not e[F["pub"]] or k < 0:
            bad.append(("untraced", k, i, None, None))
            continue
        lat_dev = got[k]["latency_s"][i] - (e[F["harvest"]] - e[F["post"]]) / 1e9 if last[(k, i)][1] == t else 0.0
        task_dev = (e[F["pub"]] - e[F["post"]] - (d - post)) / 1e9
        trig = [tr.get((ranks[w2], t2)) for w2, t2 in done_at.get(seen, [])]
        trig = [x[F["pub"]] for x in trig if x is not None and x[F["pub"]]]
        # the coordinator's previous harvest in the same call: the state machine harvests one
        # completion at a time in the oracle's order, so a harvest cannot precede the one before
        # it -- whose own hop (and its task's) is checked on its own.  (A task posted late by the
        # chain drift completes late and holds the next harvest back: kmap2_n9 op 356, r06g.)
        before = [x[F["harvest"]] for x in tr.values()
                  if got[k]["t_ns"][0] <= x[F["harvest"]] < e[F["harvest"]]]
        t_trig = max(max(trig) if trig else 0, got[k]["t_ns"][0], max(before) if before else 0)
        obs_dev = (e[F["harvest"]] - t_trig) / 1e9
        hops["latency"].append(lat_dev)
        hops["task"].append(task_dev)
        hops["harvest"].append(obs_dev)
        if abs(lat_dev) > lat_tol:
            bad.append(("latency", k, i, round(lat_dev * 1e3, 3), lat_tol * 1e3))
        if abs(task_dev) > task_tol:
            bad.append(("task", k, i, round(task_dev * 1e3, 3), task_tol * 1e3))
        if obs_dev > obs_tol or obs_dev < -0.1e-3:
            bad.append(("harvest", k, i, round(obs_dev * 1e3, 3), obs_tol * 1e3))
    hops["between_calls"] = [(got[k]["t_ns"][0] - got[k - 1]["t_ns"][1] - sc["ops"][k].get("advance_ns", 0)) / 1e9
                             for k in range(1, len(got))]
    stats = {key: (round(float(np.median(v)) * 1e3, 3), round(float(np.percentile(np.abs(v), 99)) * 1e3, 3),
                   round(float(np.max(np.abs(v))) * 1e3, 3))
             for key, v in hops.items() if v}
    return sorted(bad, key=lambda b: (b[1], b[2])), stats


def explain_misses(got, trace, bad):
    """For each missed harvest (op k, pool position i): the harvested task's split, and the
    latest task (completion store - due) the gate waited for during that call."""
    out = []
    if trace is None or len(trace) == 0:
        return out
    for k, i, d, _tol in bad[:6]:
        t0, t1 = got[k]["t_ns"]
        rank = got[k]["ranks"][i]
        mine = [e for e in trace if e[F["rank"]] == rank and t0 <= e[F["harvest"]] <= t1]
        during = [e for e in trace if e[F["seen"]] and t0 <= e[F["seen"]] <= t1 and e[F["pub"]]]
        worst = max(during, key=lambda e: e[F["pub"]] - e[F["due"]], default=None)
        # the coordinator's activity before the late harvest: every task posted, launched or
        # harvested in the 3 ms before it (ms relative to the harvest)
        h = mine[-1][F["harvest"]] if mine else t1
        rel = lambda v: round((v - h) / 1e6, 3) if v else None  # noqa: E731
        near = [e for e in trace if any(h - 3_000_000 <= e[F[f]] <= h for f in ("post", "call", "harvest", "pub"))]
        act = [{"task": "r%d#%d" % (e[F["rank"]], e[F["seq"]]), "post": rel(e[F["post"]]), "call": rel(e[F["call"]]),
                "ret": rel(e[F["ret"]]), "pub": rel(e[F["pub"]]), "seen": rel(e[F["seen"]]), "harvest": rel(e[F["harvest"]])}
               for e in sorted(near, key=lambda e: e[F["post"]])][-8:]
        out.append({"op": k, "pos": i, "dev_ms": d, "harvested": task_parts(mine[-1]) if mine else None,
                    "latest_in_call": task_parts(worst) if worst is not None else None, "activity": act})
    return out


def trace_stats(trace):
    """Percentiles (p50 / p99 / max, ms) of each part over every traced task."""
    parts = [task_parts(e) for e in trace]
    st = {}
    for key in ("timer", "deadline", "launch", "queue", "kernel", "visible", "harvest", "late"):
        v = np.asarray([p[key] for p in parts if p[key] is not None])
        if len(v):
            st[key] = (round(float(np.median(v)), 3), round(float(np.percentile(v, 99)), 3), round(float(v.max()), 3))
    return st


def random_scenario(seed):
    """A random pool / schedule / op mix (ties from 0-5 ms durations, nwait integers,
    counting predicates and test/kmap2.jl:65's predicate, explicit epochs, waitall!s)."""
    rng = np.random.default_rng(5000 + seed)
    n = int(rng.integers(1, 10))
    ops = []
    for _ in range(int(rng.integers(5, 50))):
        if rng.random() < 0.08:
            ops.append({"op": "waitall"})
            continue
        op = {"op": "asyncmap", "send": int(rng.integers(0, 1000)),
              "advance_ns": int(rng.integers(0, 3)) * 1_000_000 if rng.random() < 0.3 else 0}
        k = rng.random()
        op["nwait"] = int(rng.integers(0, n + 1)) if k < 0.6 else f"count_{int(rng.integers(0, n + 1))}" if k < 0.8 else "first"
        if rng.random() < 0.2:
            op["epoch"] = int(rng.integers(-3, 40))
        ops.append(op)
    d = rng.integers(0, 6, size=(n, 8)) * 1_000_000
    return {"name": f"rand{seed}", "n": n, "worker": "kmap2", "durations_ns": d.ravel().tolist(), "ops": ops}


def _watchdog_loop(conn):
    """Sleep 0.5 ms at a time; on each request reply (worst oversleep in ms, how many > 2 ms)
    since the previous request."""
    worst, over = 0.0, 0
    while True:
        if conn.poll():
            if conn.recv() is None:
                return
            conn.send((round(worst, 3), over))
            worst, over = 0.0, 0
        t0 = time.perf_counter()
        time.sleep(0.0005)
        d = (time.perf_counter() - t0 - 0.0005) * 1e3
        worst = max(worst, d)
        over += d > 2.0


class HostWatchdog:
    """A process beside the test (same cgroup, no GPU) that measures how late its own 0.5 ms
    sleeps wake: a host-wide stall (CPU throttling, descheduling by other tenants of the
    machine) shows there as well as in the pool's host-time latencies.  take() returns the
    worst oversleep (ms) and the count over 2 ms since the previous take()."""

    def __init__(self):
        import multiprocessing as mp
        ctx = mp.get_context("spawn")
        self._conn, child = ctx.Pipe()
        self._proc = ctx.Process(target=_watchdog_loop, args=(child,), daemon=True)
        self._proc.start()

    def take(self):
        self._conn.send(1)
        return self._conn.recv()

    def close(self):
        try:
            self._conn.send(None)
        except OSError:
            pass
        self._proc.join(5)


def warm_kernels(M, torch, n):
    """Load the task / deadline / exchange code objects before a timing-sensitive trace (a
    first launch loads its code object): delayed tasks by the host timer (the caller on the NULL
    stream) and behind device deadlines (on a stream of its own)."""
    for own in (False, True):
        ctx = torch.cuda.stream(torch.cuda.Stream()) if own else contextlib.nullcontext()
        with ctx:
            comm = M.DeviceComm(n)
            for r in range(1, n + 1):
                comm.set_task(r, "kmap2")
                comm.set_delays(r, [100_000, 0])
            pool = M.MPIAsyncPool(n)
            s = torch.zeros(1, dtype=torch.float64, device="cuda")
            rb = torch.zeros(3 * n, dtype=torch.float64, device="cuda")
            for _ in range(3):
                M.asyncmap_(pool, s, rb, torch.zeros(n, dtype=torch.float64, device="cuda"), torch.zeros_like(rb), comm,
                            nwait=n)
            torch.cuda.synchronize()
            comm.close()
