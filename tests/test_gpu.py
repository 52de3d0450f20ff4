"""GPU parity tests: the HIP path (libmpiasyncpools.so through its C ABI) against the oracle.

  * the reference's own tests (test/kmap1.jl, test/kmap2.jl) on device workers;
  * (the golden traces replay on device in tests/test_gpu_gated.py, gated by the oracle's
    schedule);
  * the least-squares shard kernel against the fp64 numpy oracle (rel 1e-5 fp32,
    1e-12 fp64, BASELINE.json north_star), small shapes incl. ragged rows and masked
    columns, and the full BASELINE c2 shape against a torch fp64 reference;
  * the device data generator bit-exact against oracle/lsq.py.
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def M(built):
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU visible")
    import mpiasyncpools
    return mpiasyncpools


@pytest.fixture(scope="module")
def torch_mod(M):
    import torch
    return torch


def _dev(torch, a):
    return torch.from_numpy(np.ascontiguousarray(a)).cuda()


def test_kmap1(M, torch_mod):
    torch = torch_mod
    nworkers = 2
    comm = M.DeviceComm(nworkers)
    for r in range(1, nworkers + 1):
        comm.set_task(r, "kmap1")
    pool = M.MPIAsyncPool(nworkers)
    sendbuf = torch.full((1,), 3.14, dtype=torch.float64, device="cuda")
    isendbuf = torch.zeros(nworkers, dtype=torch.float64, device="cuda")
    recvbuf = torch.empty(nworkers, dtype=torch.float64, device="cuda")
    irecvbuf = recvbuf.clone()
    M.asyncmap_(pool, sendbuf, recvbuf, isendbuf, irecvbuf, comm, nwait=nworkers, tag=0)
    assert recvbuf.cpu().tolist() == [1.0, 2.0]                    # kmap1.jl:22
    assert isendbuf.cpu().tolist() == [3.14, 3.14]                 # kmap1.jl:30


def test_task_trace(M, torch_mod):
    """mpa_comm_set_trace / mpa_comm_trace: every posted task's life on one clock, in order --
    post <= due, call <= ret (the timer thread's launch of a delayed task), the kernel's
    device-clock start <= completion store (mapped to host time; calibration error well under
    0.1 ms), harvest after the completion; a delayed task's launch call within a few ms of its
    due time less the launch lead."""
    torch = torch_mod
    n = 4
    comm = M.DeviceComm(n)
    for r in range(1, n + 1):
        comm.set_task(r, "kmap2")
        comm.set_delays(r, [2_000_000 * r, 0])
    comm.set_trace(64)
    pool = M.MPIAsyncPool(n)
    s = torch.ones(1, dtype=torch.float64, device="cuda")
    rb = torch.zeros(3 * n, dtype=torch.float64, device="cuda")
    for _ in range(4):
        M.asyncmap_(pool, s, rb, torch.zeros(n, dtype=torch.float64, device="cuda"), torch.zeros_like(rb), comm, nwait=n)
    tr = comm.trace()
    assert tr.shape == (4 * n, 11)
    F = {k: j for j, k in enumerate(M.DeviceComm.TRACE_FIELDS)}
    slack = 100_000  # ns: the device clock's calibration
    for e in tr:
        assert 1 <= e[F["rank"]] <= n and e[F["seq"]] >= 1
        assert 0 < e[F["post"]] <= e[F["due"]] and e[F["post"]] <= e[F["call"]] <= e[F["ret"]]
        assert e[F["start"]] and e[F["start"]] <= e[F["pub"]] + slack
        assert e[F["call"]] - slack <= e[F["start"]] and e[F["pub"]] <= e[F["harvest"]] + slack
        delay = e[F["due"]] - e[F["post"]]
        if delay:
            assert delay == 2_000_000 * e[F["rank"]]
            assert abs(e[F["call"]] - (e[F["due"]] - 35_000)) < 5_000_000
    comm.set_trace(0)
    assert len(comm.trace()) == 0
    comm.shutdown()


@pytest.mark.timing
@pytest.mark.parametrize("nranks", [3, 10])
def test_kmap2(M, torch_mod, nranks):
    """test/kmap2.jl end to end on device workers; delays = the reference's distribution / 10."""
    import time
    torch = torch_mod
    nworkers = nranks - 1
    rng = np.random.default_rng(nranks)
    comm = M.DeviceComm(nworkers)
    for r in range(1, nworkers + 1):
        comm.set_task(r, "kmap2")
        comm.set_delays(r, (np.maximum(rng.random(256) / 10, 0.005) * 1e8).astype(np.int64))
    pool = M.MPIAsyncPool(nworkers)
    assert list(pool.ranks) == list(range(1, nworkers + 1))
    sendbuf = torch.empty(1, dtype=torch.float64, device="cuda")
    isendbuf = torch.zeros(nworkers, dtype=torch.float64, device="cuda")
    recvbuf = torch.empty(3 * nworkers, dtype=torch.float64, device="cuda")
    irecvbuf = recvbuf.clone()
    nwait = 2
    for epoch in range(1, 101):
        sendbuf.fill_(epoch)
        repochs = M.asyncmap_(pool, sendbuf, recvbuf, isendbuf, irecvbuf, comm, nwait=nwait, tag=0)
        rb = recvbuf.cpu().numpy().reshape(nworkers, 3)
        fresh = 0
        for i in range(nworkers):
            if repochs[i] == 0:
                continue
            if repochs[i] == epoch:
                fresh += 1
            assert rb[i, 2] == repochs[i]
            assert rb[i, 0] == i + 1
        assert fresh >= nwait
    for _ in range(100):
        M.asyncmap_(pool, sendbuf, recvbuf, isendbuf, irecvbuf, comm, nwait=1, tag=0)
        M.waitall_(pool, recvbuf, irecvbuf)
        assert not pool.active.any()
    f = lambda epoch, repochs: bool(repochs[0] == epoch)
    # kmap2.jl:71 (atol 1e-3) at every call of a 100-call run (round 3 allowed two calls up to
    # 5 ms: launches stalled on a process holding more HSA queues than the GPU maps,
    # profiles/r04_gated_stall.txt); a run with a miss gets one rerun (a stall of the box),
    # every call's repochs checked in each
    for attempt in range(2):
        if attempt:
            time.sleep(10)  # a noisy spell of the box passes (profiles/r04_gated_stall.txt)
        dev = []
        with gated_mod().no_gc():  # a GC pass inside the call's Python wrapper is call time, not latency
            for _ in range(100):
                t0 = time.perf_counter()
                repochs = M.asyncmap_(pool, sendbuf, recvbuf, isendbuf, irecvbuf, comm, nwait=f, tag=0)
                delay = time.perf_counter() - t0
                assert repochs[0] == pool.epoch
                dev.append(abs(delay - pool.latency[0]))
        dev = np.sort(np.asarray(dev))
        print("kmap2.jl:71 run %d: |call time - latency| max %.3f ms" % (attempt, 1e3 * dev[-1]))
        if dev[-1] <= 1e-3:
            break
    assert dev[-1] <= 1e-3, dev[-5:]
    # t counts the tasks each worker served (kmap2.jl:82-84)
    M.waitall_(pool, recvbuf, irecvbuf)
    rb = recvbuf.cpu().numpy().reshape(nworkers, 3)
    for i in range(nworkers):
        assert rb[i, 1] == comm.tasks_done(i + 1)
    comm.shutdown()


def gated_mod():
    import gated
    return gated


def _warm_kernels(M, torch, n):
    import gated
    gated.warm_kernels(M, torch, n)


def test_queue_cap(M, torch_mod):
    """The process holds at most MPA_MAX_QUEUES (10) CU-masked streams per device: a comm of
    24 workers shares them, and a 9-worker comm after it gets a stream of its own per worker
    beside its coordinator stream (past ~20 queues the GPU time-slices them and launches stall
    ~10 ms, profiles/r04_queue_latency.txt)."""
    big = M.DeviceComm(24)
    for r in range(1, 25):
        big.set_task(r, "kmap2")
    assert big.counter("queues") <= 10
    assert big.counter("shared_worker_streams") >= 14
    big.close()
    c = M.DeviceComm(9)
    for r in range(1, 10):
        c.set_task(r, "kmap2")
        c.set_delays(r, [1000])
    assert c.counter("queues") <= 10 and c.counter("shared_worker_streams") == 0
    pool = M.MPIAsyncPool(9)
    torch = torch_mod
    rb = torch.zeros(27, dtype=torch.float64, device="cuda")
    M.asyncmap_(pool, torch.ones(1, dtype=torch.float64, device="cuda"), rb,
                torch.zeros(9, dtype=torch.float64, device="cuda"), torch.zeros_like(rb), c, nwait=9)
    assert c.counter("sleeps") == 0 and c.counter("timer_late") == 0  # the host timer launched them
    assert rb.cpu().numpy().reshape(9, 3)[:, 0].tolist() == list(range(1, 10))
    c.close()


_PAST_CAP_CHILD = r"""
import sys
sys.path.insert(0, sys.argv[1])
import torch
import mpiasyncpools as M
c = M.DeviceComm(2)          # its coordinator stream takes the one queue MPA_MAX_QUEUES=1 allows
for r in (1, 2):
    c.set_task(r, "kmap2")   # worker 1: a kind with no stream yet -> one queue past the cap
pool = M.MPIAsyncPool(2)     # worker 2: shares worker 1's
rb = torch.zeros(6, dtype=torch.float64, device="cuda")
M.asyncmap_(pool, torch.ones(1, dtype=torch.float64, device="cuda"), rb, torch.zeros(2, dtype=torch.float64, device="cuda"),
            torch.zeros_like(rb), c, nwait=2)
print("RESULT", c.counter("queues"), c.counter("queues_past_cap"), c.counter("shared_worker_streams"),
      rb.cpu().numpy().reshape(2, 3)[:, 0].tolist())
c.close()
"""


def test_queue_past_cap_is_counted_and_said(M):
    """past MPA_MAX_QUEUES a stream kind that has no stream yet still gets a queue
    (a coordinator or worker stream cannot share another kind's), but no longer silently: the
    process says so once on stderr and counts it (counter queues_past_cap).  The cap is read once
    per process: a child with MPA_MAX_QUEUES=1."""
    import os
    import subprocess
    import sys
    pkg = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "mpistragglers.jl_amd")
    r = subprocess.run([sys.executable, "-c", _PAST_CAP_CHILD, pkg], env=dict(os.environ, MPA_MAX_QUEUES="1"),
                       capture_output=True, text=True, timeout=180)
    assert r.returncode == 0, r.stderr[-2000:]
    line = [ln for ln in r.stdout.splitlines() if ln.startswith("RESULT")][-1].split(maxsplit=4)
    queues, past, shared = int(line[1]), int(line[2]), int(line[3])
    assert (queues, past, shared) == (2, 1, 2), line
    assert line[4] == "[1.0, 2.0]", line
    assert "one more for a stream kind that has none yet" in r.stderr


def test_device_delays_only_on_unshared_streams(M, torch_mod, monkeypatch):
    """MPA_DELAY=device (forced; by default only where no caller work on the NULL stream can meet
    it): a delayed task waits behind a one-wave deadline kernel ahead of it on its worker's
    stream -- but only where that stream is the worker's own: past the queue cap workers share
    streams, and a wait there would hold the other worker's tasks, so those delays stay on the
    host timer.  16 workers over 9 streams: one deadline kernel per unshared worker, every reply
    correct."""
    monkeypatch.setenv("MPA_DELAY", "device")
    torch = torch_mod
    c = M.DeviceComm(16)
    for r in range(1, 17):
        c.set_task(r, "kmap2")
        c.set_delays(r, [200_000])
    pool = M.MPIAsyncPool(16)
    rb = torch.zeros(48, dtype=torch.float64, device="cuda")
    M.asyncmap_(pool, torch.ones(1, dtype=torch.float64, device="cuda"), rb,
                torch.zeros(16, dtype=torch.float64, device="cuda"), torch.zeros_like(rb), c, nwait=16)
    shared = c.counter("shared_worker_streams")  # the streams were in place before the launches
    assert 0 < shared < 16 and c.counter("queues") <= 10
    assert c.counter("sleeps") == 16 - shared, (c.counter("sleeps"), shared)
    assert rb.cpu().numpy().reshape(16, 3)[:, 0].tolist() == list(range(1, 17))
    c.close()


def _straggler_hold(M, torch):
    """Three nwait = 1 calls while worker 2's 400 ms delay sleeps ON THE DEVICE (a deadline kernel
    on its worker stream): the wall time of each call."""
    import time
    c = M.DeviceComm(2)
    for r in (1, 2):
        c.set_task(r, "kmap2")
    c.set_delays(2, [400_000_000])
    pool = M.MPIAsyncPool(2)
    f64 = dict(dtype=torch.float64, device="cuda")
    s, rb, isb = torch.ones(1, **f64), torch.zeros(6, **f64), torch.zeros(2, **f64)
    irb = torch.zeros_like(rb)
    t = []
    for _ in range(3):
        t0 = time.perf_counter()
        M.asyncmap_(pool, s, rb, isb, irb, c, nwait=1)
        t.append(time.perf_counter() - t0)
    sleeps = c.counter("sleeps")
    M.waitall_(pool, rb, irb)
    ok = rb.cpu().numpy().reshape(2, 3)[:, 0].tolist() == [1.0, 2.0]
    c.close()
    return t, sleeps, ok


def test_running_straggler_does_not_hold_the_coordinator(M, torch_mod, monkeypatch):
    """k-of-n: a straggler's task RUNNING on its worker stream must not hold the coordinator's
    work.  The Python API hands the comm torch's default stream, HIP's NULL stream, and HIP runs
    a NULL-stream command only after everything queued on the device's blocking streams: the
    exchange that re-dispatched worker 1 waited for worker 2's running kernel (c3: 0.1-0.6 ms per
    epoch step, up to 5.7 ms per harvest; profiles/r05_null_stream.txt).  The comm coordinates on
    a stream of its own instead (hip_transport.hpp set_stream): calls 2 and 3 re-dispatch worker 1
    in milliseconds while worker 2's 400 ms deadline kernel runs."""
    monkeypatch.setenv("MPA_DELAY", "device")
    torch = torch_mod
    t, sleeps, ok = _straggler_hold(M, torch)
    assert sleeps == 1 and ok
    assert max(t[1:]) < 0.1, t
    monkeypatch.setenv("MPA_OWN_COORD", "0")  # the NULL stream, for the record
    print("re-dispatch call times (s): own stream %s; NULL stream %s" % (t, _straggler_hold(M, torch)[0]))


@pytest.mark.timing
@pytest.mark.parametrize("path", ["timer", "deadline"])
def test_delay_calibration(M, torch_mod, path):
    """An injected delay of d ms shows up as a latency of d ms (within 0.5 ms), by either path:
    the host timer (the caller on torch's default stream, HIP's NULL stream: a device deadline
    would hold every NULL-stream command) and a device deadline (the caller on a stream of its
    own: deadline_kernel queued ahead of the task, no host thread involved; within 0.2 ms)."""
    import contextlib
    torch = torch_mod
    _warm_kernels(M, torch, 2)
    comm = M.DeviceComm(2)
    for r, d in ((1, 20_000_000), (2, 7_000_000)):
        comm.set_task(r, "echo")
        comm.set_delays(r, [d])
    pool = M.MPIAsyncPool(2)
    tol = 0.5e-3 if path == "timer" else 0.2e-3
    ctx = torch.cuda.stream(torch.cuda.Stream()) if path == "deadline" else contextlib.nullcontext()
    with ctx:
        s = torch.zeros(2, device="cuda")
        # three calls in a row; a run with a miss gets one rerun (a stall of the box inflates one
        # call's latency, profiles/r04_gated_stall.txt)
        for attempt in range(2):
            if attempt:
                __import__("time").sleep(10)  # a noisy spell of the box passes
            lat = []
            with gated_mod().no_gc():
                for _ in range(3):
                    M.asyncmap_(pool, s, torch.zeros(4, device="cuda"), torch.zeros(4, device="cuda"),
                                torch.zeros(4, device="cuda"), comm, nwait=2)
                    # the delay is dispatch -> reply (the task's launch overhead is inside it)
                    lat.append((float(pool.latency[0]), float(pool.latency[1])))
            ok = all(abs(a - 0.020) < tol and abs(b - 0.007) < tol for a, b in lat)
            print("delay calibration (%s) run %d: %s" % (path, attempt, lat))
            if ok:
                break
        torch.cuda.current_stream().synchronize()
    assert ok, lat
    # which path ran: deadline kernels (and the clock samples behind them) or the timer
    if path == "deadline":
        assert comm.counter("sleeps") >= 6 and comm.counter("clock_samples") >= 1
    else:
        assert comm.counter("sleeps") == 0


def _lsq_case(M, torch, dtype, rows, cols, lda=None, seed=3, nworkers=1, grid=None):
    import lsq
    lda = cols if lda is None else lda
    tname = "f32" if dtype == "f32" else "f64"
    tdt = torch.float32 if dtype == "f32" else torch.float64
    A = np.zeros((rows, lda), dtype=np.float32 if dtype == "f32" else np.float64)
    A[:, :cols] = lsq.gen_matrix(seed, 0, rows, cols, tname)
    b = lsq.gen_vector(seed, 0, rows, tname)
    x = lsq.gen_vector(seed, 0, cols, tname, stream=lsq.STREAM_X, scale=0.5)
    comm = M.DeviceComm(nworkers)
    Ad, bd = _dev(torch, A), _dev(torch, b)
    for r in range(1, nworkers + 1):
        comm.set_task_lsq(r, Ad, bd, cols=cols, lda=lda)
    pool = M.MPIAsyncPool(nworkers)
    send = _dev(torch, x)
    isend = torch.zeros(nworkers * cols, dtype=tdt, device="cuda")
    recv = torch.zeros(nworkers * cols, dtype=tdt, device="cuda")
    irecv = torch.zeros_like(recv)
    M.asyncmap_(pool, send, recv, isend, irecv, comm, nwait=nworkers)
    g_ref = lsq.shard_gradient(A[:, :cols], b, x)
    out = recv.cpu().numpy().reshape(nworkers, cols)
    return out, g_ref, (comm, pool, send, recv, isend, irecv)


@pytest.mark.parametrize("rows,cols", [(1, 256), (37, 256), (1000, 512), (4099, 1024), (2048, 2048),
                                       (777, 1000), (513, 100), (5000, 1536)])
def test_lsq_f32(M, torch_mod, rows, cols):
    out, g_ref, _ = _lsq_case(M, torch_mod, "f32", rows, cols, lda=((cols + 3) // 4) * 4)
    err = np.linalg.norm(out[0] - g_ref) / np.linalg.norm(g_ref)
    assert err <= 1e-5, err


@pytest.mark.parametrize("rows,cols", [(4099, 2048), (5000, 1536), (3, 2048)])
def test_lsq_f32_batched_2048(M, torch_mod, rows, cols):
    """Several fp32 tasks of up to 2048 columns in ONE launch take the four-row tile
    (lsq_kernel.hip launch_lsq): every worker's gradient against the fp64 oracle at 1e-5, the
    same bits for every worker (they share the shard)."""
    out, g_ref, _ = _lsq_case(M, torch_mod, "f32", rows, cols, lda=((cols + 3) // 4) * 4, nworkers=3)
    for w in range(3):
        err = np.linalg.norm(out[w] - g_ref) / np.linalg.norm(g_ref)
        assert err <= 1e-5, (w, err)
    assert np.array_equal(out[0], out[1]) and np.array_equal(out[0], out[2])


@pytest.mark.parametrize("rows,cols", [(1, 128), (300, 256), (1025, 1024), (999, 2048), (64, 130)])
def test_lsq_f64(M, torch_mod, rows, cols):
    out, g_ref, _ = _lsq_case(M, torch_mod, "f64", rows, cols, lda=((cols + 1) // 2) * 2)
    err = np.linalg.norm(out[0] - g_ref) / np.linalg.norm(g_ref)
    assert err <= 1e-12, err


@pytest.mark.parametrize("dtype,rows,cols,lda", [("f32", 1000, 4096, 4096), ("f32", 333, 3000, 3004),
                                                  ("f32", 2500, 8200, 8200), ("f32", 5, 65536, 65536),
                                                  ("f64", 700, 2050, 2050), ("f64", 1201, 6000, 6002)])
def test_lsq_wide_rows(M, torch_mod, dtype, rows, cols, lda):
    """Rows wider than the narrow kernel's 2048 columns (lsqw_kernel.hip, two passes): three
    workers on the same shard in one batched launch against the fp64 oracle (1e-5 fp32 /
    1e-12 fp64), identical bits across workers and across repeated launches."""
    torch = torch_mod
    out, g_ref, st = _lsq_case(M, torch, dtype, rows, cols, lda=lda, nworkers=3)
    comm, pool, send, recv, isend, irecv = st
    tol = 1e-5 if dtype == "f32" else 1e-12
    for i in range(3):
        err = np.linalg.norm(out[i] - g_ref) / np.linalg.norm(g_ref)
        assert err <= tol, (i, err)
    u = np.uint32 if dtype == "f32" else np.uint64
    assert np.array_equal(out[0].view(u), out[1].view(u)) and np.array_equal(out[0].view(u), out[2].view(u))
    first = recv.clone()
    for _ in range(2):
        M.asyncmap_(pool, send, recv, isend, irecv, comm, nwait=3)
        assert torch.equal(first, recv)
    comm.close()


def test_lsq_padded_lda_and_determinism(M, torch_mod):
    torch = torch_mod
    out, g_ref, st = _lsq_case(M, torch, "f32", 3000, 1000, lda=1024, nworkers=3)
    comm, pool, send, recv, isend, irecv = st
    assert np.linalg.norm(out[0] - g_ref) / np.linalg.norm(g_ref) <= 1e-5
    # every worker computed the same shard: identical bits (fixed-order reduction)
    assert np.array_equal(out[0].view(np.uint32), out[1].view(np.uint32))
    assert np.array_equal(out[0].view(np.uint32), out[2].view(np.uint32))
    first = recv.clone()
    for _ in range(3):
        M.asyncmap_(pool, send, recv, isend, irecv, comm, nwait=3)
        assert torch.equal(first.view(torch.int32), recv.view(torch.int32))


@pytest.mark.parametrize("cols", [512, 3000])
def test_lsq_gradient_descent_chunks_match_their_epochs(M, torch_mod, cols):
    """Asyncmap with least-squares workers and stragglers: each chunk i equals the
    gradient of the iterate sent at epoch repochs[i] (kmap2.jl:50, numerically); narrow and
    wide rows."""
    import lsq
    torch = torch_mod
    n, rows, seed = 4, 2048, 11
    comm = M.DeviceComm(n)
    A = lsq.gen_matrix(seed, 0, n * rows, cols, "f32")
    b = lsq.gen_vector(seed, 0, n * rows, "f32")
    keep = []
    rng = np.random.default_rng(5)
    for r in range(1, n + 1):
        Ad, bd = _dev(torch, A[(r - 1) * rows:r * rows]), _dev(torch, b[(r - 1) * rows:r * rows])
        keep.append((Ad, bd))
        comm.set_task_lsq(r, Ad, bd)
        comm.set_delays(r, rng.integers(0, 6, size=16) * 1_000_000)
    pool = M.MPIAsyncPool(n)
    x = torch.zeros(cols, dtype=torch.float32, device="cuda")
    isend = torch.zeros(n * cols, dtype=torch.float32, device="cuda")
    recv = torch.zeros(n * cols, dtype=torch.float32, device="cuda")
    irecv = torch.zeros_like(recv)
    sent = {}
    for epoch in range(1, 16):
        sent[epoch] = x.cpu().numpy().copy()
        rep = M.asyncmap_(pool, x, recv, isend, irecv, comm, nwait=2)
        chunks = recv.cpu().numpy().reshape(n, cols)
        for i in range(n):
            if rep[i] == 0:
                continue
            xs = sent[int(rep[i])]
            g = lsq.shard_gradient(A[i * rows:(i + 1) * rows], b[i * rows:(i + 1) * rows], xs)
            assert lsq.rel_err(chunks[i], g) <= 1e-5, (epoch, i)
        w = (rep == epoch).astype(np.float64) * (n / max(1, int((rep == epoch).sum())))
        comm.lsq_update(x, recv, n, w, 0.05)
    M.waitall_(pool, recv, irecv)


def test_aggregate_and_update(M, torch_mod):
    torch = torch_mod
    rng = np.random.default_rng(0)
    comm = M.DeviceComm(1)
    for dt, tdt, tol in ((np.float32, torch.float32, 1e-6), (np.float64, torch.float64, 1e-15)):
        n, c = 7, 1000
        chunks = rng.standard_normal((n, c)).astype(dt)
        w = rng.standard_normal(n)
        w[2] = 0.0
        out = torch.zeros(c, dtype=tdt, device="cuda")
        comm.aggregate(_dev(torch, chunks.ravel()), n, w, out)
        ref = (w[:, None] * chunks.astype(np.float64)).sum(0)
        assert np.max(np.abs(out.cpu().numpy() - ref)) <= tol * np.max(np.abs(ref)) * 10
        x0 = rng.standard_normal(c).astype(dt)
        x = _dev(torch, x0)
        comm.lsq_update(x, _dev(torch, chunks.ravel()), n, w, 0.1)
        assert np.max(np.abs(x.cpu().numpy() - (x0 - 0.1 * ref))) <= tol * 10 * (1 + np.max(np.abs(ref)))


@pytest.mark.parametrize("dtype", ["f32", "f64", "bf16"])
def test_generate_bit_exact(M, torch_mod, dtype):
    import lsq
    torch = torch_mod
    tdt = {"f32": torch.float32, "f64": torch.float64, "bf16": torch.bfloat16}[dtype]
    for e0, cnt, scale in ((0, 4096, 1 / 32), (5, 1001, 0.7), (2**35 + 3, 333, 1.0)):
        out = torch.empty(cnt, dtype=tdt, device="cuda")
        M.generate(out, 42, 0, e0, scale)
        ref = lsq.gen_vector(42, e0, cnt, dtype, stream=0,
                             scale=np.float64(scale) if dtype == "f64" else np.float32(scale))
        got = out.cpu()
        if dtype == "bf16":
            assert np.array_equal(got.view(torch.int16).numpy().view(np.uint16), ref)
        elif dtype == "f32":
            assert np.array_equal(got.numpy().view(np.uint32), ref.view(np.uint32))
        else:
            assert np.array_equal(got.numpy().view(np.uint64), ref.view(np.uint64))


def test_full_size_c2_against_torch_fp64(M, torch_mod):
    """BASELINE c2 shape (A 2^20 x 1024 fp32, 8 workers): every worker's g_i against a
    torch fp64 computation of A_i^T(A_i x - b_i) on the same device data (rel 1e-5)."""
    torch = torch_mod
    n, rows, cols, seed = 8, 1 << 20, 1024, 1234
    per = rows // n
    comm = M.DeviceComm(n)
    A = torch.empty(rows, cols, dtype=torch.float32, device="cuda")
    b = torch.empty(rows, dtype=torch.float32, device="cuda")
    M.generate(A, seed, 0, 0, float(np.float32(1 / np.sqrt(cols))))
    M.generate(b, seed, 1, 0, 1.0)
    for r in range(1, n + 1):
        comm.set_task_lsq(r, A[(r - 1) * per:r * per], b[(r - 1) * per:r * per])
    x = torch.empty(cols, dtype=torch.float32, device="cuda")
    M.generate(x, seed, 2, 0, 0.5)
    pool = M.MPIAsyncPool(n)
    isend = torch.zeros(n * cols, dtype=torch.float32, device="cuda")
    recv = torch.zeros(n * cols, dtype=torch.float32, device="cuda")
    irecv = torch.zeros_like(recv)
    M.asyncmap_(pool, x, recv, isend, irecv, comm, nwait=n)
    got = recv.view(n, cols).double()
    x64 = x.double()
    for i in range(n):
        Ai = A[i * per:(i + 1) * per].double()
        g = Ai.t() @ (Ai @ x64 - b[i * per:(i + 1) * per].double())
        err = (torch.linalg.norm(got[i] - g) / torch.linalg.norm(g)).item()
        assert err <= 1e-5, (i, err)
        del Ai
    # isendbuf holds n copies of x (the reference's isendbufs[i] .= sendbuf, :130)
    assert torch.equal(isend.view(n, cols), x.expand(n, cols))


@pytest.mark.parametrize("env,cols", [({}, 1024), ({"MPA_TAIL": "0"}, 1024), ({"MPA_AHEAD": "0"}, 1024),
                                      ({"MPA_AHEAD": "0", "MPA_HEAD": "0"}, 1024), ({"MPA_FUSE": "0"}, 1024),
                                      ({}, 4096)])
def test_lsq_descent_native_loop_matches_python_loop(M, torch_mod, monkeypatch, env, cols):
    """mpa_lsq_descent makes the same calls as the Python loop: identical iterates (bitwise,
    nwait = n so every epoch is fresh and every kernel is deterministic), with launch-ahead
    and the epoch step fused into the previous launch's tail (default), launch-ahead with a
    separate epoch kernel, no launch-ahead (the step at the head of the task launch, or as
    its own epoch kernel), and unfused."""
    import lsq
    torch = torch_mod
    for k, v in env.items():
        monkeypatch.setenv(k, v)
    n, rows, seed = 4, 2048, 17
    A = _dev(torch, lsq.gen_matrix(seed, 0, n * rows, cols, "f32"))
    b = _dev(torch, lsq.gen_vector(seed, 0, n * rows, "f32"))
    xs = []
    for native in (False, True):
        comm = M.DeviceComm(n)
        for r in range(1, n + 1):
            comm.set_task_lsq(r, A[(r - 1) * rows:r * rows], b[(r - 1) * rows:r * rows])
        pool = M.MPIAsyncPool(n)
        x = torch.zeros(cols, device="cuda")
        isend = torch.zeros(n * cols, device="cuda")
        recv = torch.zeros(n * cols, device="cuda")
        irecv = torch.zeros_like(recv)
        if native:
            comm.set_timing(True)
            M.lsq_descent(pool, comm, x, recv, isend, irecv, n, 0.01, 6)
            xl = comm.exchange_timing()[0]
            comm.set_timing(False)
            # epoch kernels: with the fused tail only the first ahead step (update 1) and the
            # final update (6) run as their own launches; updates 2-5 ride in launch tails
            if not env and cols <= 2048:
                assert xl == 2, xl
            elif env == {"MPA_TAIL": "0"}:
                assert xl == 6, xl
        else:
            for _ in range(6):
                rep = M.asyncmap_(pool, x, recv, isend, irecv, comm, nwait=n)
                comm.lsq_update(x, recv, n, (rep == pool.epoch) * 1.0, 0.01)
        torch.cuda.synchronize()
        assert pool.epoch == 6
        assert list(pool.repochs) == [6] * n and not any(pool.active)
        xs.append((x.clone(), recv.clone(), isend.clone()))
        comm.close()
    for a, b in zip(xs[0], xs[1]):
        assert torch.equal(a.view(torch.int32), b.view(torch.int32))
    xs = [xs[0][0], xs[1][0]]
    assert float(torch.linalg.norm(xs[0])) > 0


def test_sampled_timing_counts_one_in_k_launches(M, torch_mod, monkeypatch):
    """mpa_comm_set_timing(comm, k > 1): one in every k task launches and one in every k epoch
    kernels carry the HIP events (bench.py's latency-bound c1 keeps their host cost off the
    critical path); the averages stay per timed launch, and 0 turns timing off."""
    import lsq
    torch = torch_mod
    monkeypatch.setenv("MPA_TAIL", "0")
    monkeypatch.setenv("MPA_AHEAD", "0")
    monkeypatch.setenv("MPA_HEAD", "0")  # every epoch step its own (timed) epoch kernel
    n, rows, cols, seed = 3, 1024, 64, 5
    A = _dev(torch, lsq.gen_matrix(seed, 0, n * rows, cols, "f64"))
    b = _dev(torch, lsq.gen_vector(seed, 0, n * rows, "f64"))
    comm = M.DeviceComm(n)
    for r in range(1, n + 1):
        comm.set_task_lsq(r, A[(r - 1) * rows:r * rows], b[(r - 1) * rows:r * rows])
    pool = M.MPIAsyncPool(n)
    x = torch.zeros(cols, dtype=torch.float64, device="cuda")
    isend = torch.zeros(n * cols, dtype=torch.float64, device="cuda")
    recv = torch.zeros_like(isend)
    irecv = torch.zeros_like(isend)
    counts = {}
    for period in (1, 4):
        comm.timing()
        comm.exchange_timing()
        comm.set_timing(True, period)
        M.lsq_descent(pool, comm, x, recv, isend, irecv, n, 0.01, 8)
        torch.cuda.synchronize()
        t = comm.timing()
        xl = comm.exchange_timing()[0]
        comm.set_timing(False)
        assert t[1] > 0 and t[2] > 0 and t[3] > 0
        counts[period] = (t[0], xl)
    tasks1, epochs1 = counts[1]
    assert epochs1 >= 8 and tasks1 >= 8
    assert counts[4] == ((tasks1 + 3) // 4, (epochs1 + 3) // 4), counts
    with pytest.raises(ValueError):
        comm.set_timing(True, 0)
    comm.close()


@pytest.mark.parametrize("dtype,cols", [("f64", 64), ("f32", 1024)])
def test_fused_head_matches_epoch_kernel(M, torch_mod, monkeypatch, dtype, cols):
    """The epoch step at the head of the task launch (flush, every worker posted: c1's loop)
    gives the same iterates, replies and messages bit for bit as the step in its own epoch
    kernel (MPA_HEAD=0), and it is the one that ran (the transport's counters).  With a
    predicate nwait (not launch-ahead's integer n) the launches are PRE-ARMED (enqueued one
    epoch early, released through the pinned mailbox): bitwise the same again, with
    first_plus(n - 1) = every worker fresh, so every epoch is deterministic.  nwait < n runs
    both, with the pool's bookkeeping intact."""
    import lsq
    torch = torch_mod
    monkeypatch.setenv("MPA_AHEAD", "0")
    monkeypatch.setenv("MPA_WAIT_TIMEOUT_S", "30")
    n, rows, seed, epochs = 3, 4096, 11, 12
    tdt = torch.float64 if dtype == "f64" else torch.float32
    A = _dev(torch, lsq.gen_matrix(seed, 0, n * rows, cols, dtype))
    b = _dev(torch, lsq.gen_vector(seed, 0, n * rows, dtype))
    names = ("head_steps", "epoch_kernels", "prearmed", "prearm_cancelled", "prearm_same")

    def run(nwait, **env):
        for k in ("MPA_HEAD", "MPA_PREARM", "MPA_PRESAME"):
            monkeypatch.setenv(k, env.get(k, "1"))
        comm = M.DeviceComm(n)
        for r in range(1, n + 1):
            comm.set_task_lsq(r, A[(r - 1) * rows:r * rows], b[(r - 1) * rows:r * rows])
        pool = M.MPIAsyncPool(n)
        x = torch.zeros(cols, dtype=tdt, device="cuda")
        isend = torch.zeros(n * cols, dtype=tdt, device="cuda")
        recv = torch.zeros(n * cols, dtype=tdt, device="cuda")
        irecv = torch.zeros_like(recv)
        c0 = [comm.counter(k) for k in names]
        M.lsq_descent(pool, comm, x, recv, isend, irecv, nwait, 1e-3, epochs)
        torch.cuda.synchronize()
        steps = dict(zip(names, [comm.counter(k) - v for k, v in zip(names, c0)]))
        M.waitall_(pool, recv, irecv)
        torch.cuda.synchronize()
        out = (x.clone(), recv.clone(), isend.clone(), pool.epoch, list(pool.repochs))
        comm.close()
        return out, steps

    def same(p, q):
        for a, c in zip(p[:3], q[:3]):
            assert torch.equal(a, c)
        assert p[3:] == q[3:]

    on, s_on = run(n)
    off, s_off = run(n, MPA_HEAD="0")
    assert s_on["head_steps"] >= epochs - 1 and s_off["head_steps"] == 0 and s_off["epoch_kernels"] >= epochs - 1
    same(on, off)
    assert float(torch.linalg.norm(on[0])) > 0
    allf = M.first_plus(n - 1)
    pre, s_pre = run(allf)
    nopre, s_nopre = run(allf, MPA_PREARM="0")
    assert s_pre["prearmed"] >= epochs - 3 and s_nopre["prearmed"] == 0, (s_pre, s_nopre)
    # most pre-armed launches go with the step they predicted (kernel arguments, no mailbox
    # read); with MPA_PRESAME=0 every one reads the mailbox: bitwise the same run
    assert s_pre["prearm_same"] >= 1, s_pre
    presame0, s_ps0 = run(allf, MPA_PRESAME="0")
    assert s_ps0["prearm_same"] == 0 and s_ps0["prearmed"] >= epochs - 3, s_ps0
    same(pre, presame0)
    same(pre, nopre)
    same(pre, on)
    part, s_part = run(n - 1)
    assert s_part["head_steps"] >= 1 and part[3] == epochs and max(part[4]) == epochs
    assert bool(torch.isfinite(part[0]).all()) and float(torch.linalg.norm(part[0])) > 0


@pytest.mark.parametrize("rows4", [1024, 3072, 1 << 18], ids=["equal", "slow3x", "slow256x"])
def test_native_k_of_n_prearmed_with_stragglers(M, torch_mod, monkeypatch, capfd, rows4):
    """The native loop's shipped k-of-n fast path, ungated, at nwait 3 of 4: with equal shards
    the epochs run in pre-armed launches (c1's pattern); with worker 4's shard 256x the
    others' it replies late (a stale harvest inside a later call's wait loop,
    src/MPIAsyncPools.jl:177-184), its re-dispatch is held and joins the next batched launch,
    whose step runs at the head of the launch (3x: in between).  Whatever the timing,
    the loop must compute what the reference's coordinator computes from the repochs it saw
    (examples/iterative_example.jl:41-46): the iterate equals a torch fp64 replay of the
    per-epoch repochs the loop traced (each chunk the gradient of the iterate sent at its
    epoch, fresh chunks weighted 1), and each final chunk is the gradient of the iterate sent
    at its repochs (1e-5, fp32).  The fast path did run: pre-armed launches (equal), held
    re-dispatches and stale copies deferred into a step (256x)."""
    import re
    torch = torch_mod
    monkeypatch.setenv("MPA_DESCENT_TRACE", "1")
    monkeypatch.setenv("MPA_WAIT_TIMEOUT_S", "30")
    n, nwait, cols, epochs, eta = 4, 3, 256, 80, 1e-4
    rows = [1024, 1024, 1024, rows4]
    g = torch.Generator(device="cuda").manual_seed(5)
    A = [torch.randn(r, cols, device="cuda", generator=g) / cols ** 0.5 for r in rows]
    b = [torch.randn(r, device="cuda", generator=g) for r in rows]
    comm = M.DeviceComm(n)
    for r in range(n):
        comm.set_task_lsq(r + 1, A[r], b[r])
    names = ("prearmed", "prearm_same", "held", "stale_deferred", "head_steps")
    c0 = {k: comm.counter(k) for k in names}
    pool = M.MPIAsyncPool(n)
    x = torch.zeros(cols, device="cuda")
    isend = torch.zeros(n * cols, device="cuda")
    recv = torch.zeros(n * cols, device="cuda")
    irecv = torch.zeros_like(recv)
    capfd.readouterr()
    M.lsq_descent(pool, comm, x, recv, isend, irecv, nwait, eta, epochs)
    torch.cuda.synchronize()
    err = capfd.readouterr().err
    got = {k: comm.counter(k) - v for k, v in c0.items()}
    trace = [list(map(int, m.group(1).split())) for m in re.finditer(r"\[mpa descent\] epoch \d+ repochs ([\d ]+) \|", err)]
    assert len(trace) == epochs, (len(trace), err[-500:])
    A64 = [a.double() for a in A]
    b64 = [v.double() for v in b]

    def grad(i, xv):
        return A64[i].T @ (A64[i] @ xv - b64[i])

    xs = [torch.zeros(cols, dtype=torch.float64, device="cuda")]  # xs[e-1]: the iterate sent at epoch e
    for e, rep in enumerate(trace, start=1):
        fresh = [i for i in range(n) if rep[i] == e]
        assert len(fresh) >= nwait, (e, rep)
        upd = sum(grad(i, xs[e - 1]) for i in fresh) * (n / len(fresh))
        xs.append(xs[e - 1] - eta * upd)
    rel = float(torch.linalg.norm(x.double() - xs[-1]) / torch.linalg.norm(xs[-1]))
    assert rel <= 1e-5, rel
    M.waitall_(pool, recv, irecv)
    torch.cuda.synchronize()
    ch = recv.view(n, cols).double()
    for i in range(n):
        r = int(pool.repochs[i])
        ref = grad(i, xs[r - 1])
        assert float(torch.linalg.norm(ch[i] - ref) / torch.linalg.norm(ref)) <= 1e-5, i
    stale = sum(1 for e, rep in enumerate(trace, start=1) if rep[3] not in (0, e))
    print("k-of-n native rows4=%d: %s, epochs with worker 4 stale %d of %d, iterate rel %.2e"
          % (rows4, got, stale, epochs, rel))
    if rows4 == rows[0]:
        assert got["prearmed"] >= 1, got
    if rows4 == 1 << 18:
        assert got["held"] >= 1 and got["stale_deferred"] >= 1, got
    comm.close()


def test_read_bandwidth_probe(M, torch_mod):
    """mpa_read_bandwidth (bench.py's measured read ceiling) reads every byte and reports a
    rate inside what the part can do (below the 8 TB/s spec peak, above a floor)."""
    torch = torch_mod
    buf = torch.ones(1 << 26, dtype=torch.float32, device="cuda")  # 256 MiB
    for grid in (256, 2048):
        gbps = M.read_bandwidth(buf, grid=grid, reps=3)
        assert 500.0 < gbps < 9000.0, (grid, gbps)
    with pytest.raises(M.ArgumentError):
        M.read_bandwidth(buf, grid=0)


def test_host_buffers_refused_by_a_device_comm(M, torch_mod):
    """Pageable host memory handed to a device comm is an ArgumentError naming the buffer
    (a Julia user passing a host Vector), not a kernel reading host addresses; device buffers
    keep working on the same pool afterwards."""
    torch = torch_mod
    comm = M.DeviceComm(2)
    for r in (1, 2):
        comm.set_task(r, "kmap2")
    pool = M.MPIAsyncPool(2)
    host = np.zeros(6)
    with pytest.raises(M.ArgumentError, match="recvbuf is host memory"):
        M.asyncmap_(pool, torch.zeros(1, dtype=torch.float64, device="cuda"), host,
                    torch.zeros(2, dtype=torch.float64, device="cuda"), torch.zeros(6, dtype=torch.float64, device="cuda"),
                    comm, nwait=2)
    assert not pool.active.any()  # refused before any state change
    s = torch.full((1,), 5.0, dtype=torch.float64, device="cuda")
    rb = torch.zeros(6, dtype=torch.float64, device="cuda")
    M.asyncmap_(pool, s, rb, torch.zeros(2, dtype=torch.float64, device="cuda"), torch.zeros_like(rb), comm, nwait=2)
    assert rb.cpu().tolist() == [1, 1, 5, 2, 1, 5]
    comm.close()
