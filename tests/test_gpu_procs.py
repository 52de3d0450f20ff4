"""The multi-process HIP transport on a GPU box: rank 0 coordinates, ranks 1.. (other
processes on the same GPU) serve workers through the shared-memory mailboxes; kmap2.jl
properties across processes and least-squares epochs checked against the fp64 oracle.

(They run after the other GPU tests and before the timing checks, tests/conftest.py.)"""
import multiprocessing as mp

import pytest

import dist_worker

pytestmark = pytest.mark.gpu


def _run(target, world, *args, timeout=180):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = dist_worker.free_port()
    procs = [ctx.Process(target=target, args=(r, world, port) + args + (q,)) for r in range(world)]
    for p in procs:
        p.start()
    try:
        status, payload = q.get(timeout=timeout)
    finally:
        for p in procs:
            p.join(timeout=60)
            if p.is_alive():
                p.kill()
    assert status == "ok", payload
    assert payload == [], payload
    assert all(p.exitcode == 0 for p in procs), [p.exitcode for p in procs]


def test_kmap2_two_processes_hip(built):
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    _run(dist_worker.kmap2_dist, 2, "hip", [0, 1, 1, 1])


def test_lsq_two_processes_hip(built):
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    _run(dist_worker.lsq_dist, 2, [0, 1, 1, 1])


# MPA_ARM_DEPTH=2: two tasks of each armed worker queued behind their doorbells (the default on a GPU
# rank 0 does not use, i.e. the node's; forced here, where every rank shares GPU 0)
@pytest.mark.parametrize("depth", ["1", "2"])
def test_lsq_two_processes_prearmed(built, monkeypatch, depth):
    """Workers 2-4 on rank 1 pre-armed (MPA_ARM=1: every eligible worker, 4 with a delay schedule
    slept in its doorbell wait); two serve sessions around a pause, whose disarm cancels the
    queued tasks rank 0 never rang (one or two per worker) and re-arms them in the next session."""
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    monkeypatch.setenv("MPA_ARM", "1")  # the spawned ranks inherit it
    monkeypatch.setenv("MPA_ARM_DEPTH", depth)
    _run(dist_worker.lsq_dist_armed, 2, [0, 1, 1, 1], [4])


@pytest.mark.parametrize("cols", [256, 2048])
@pytest.mark.parametrize("arm", ["0", "2"])
def test_lsqb_two_processes(built, monkeypatch, arm, cols):
    """The batched variant across processes, host-launched and device-armed (default); at 2048
    columns the FULL form of lsqp4, armed (its doorbell-waiting instantiation) and not."""
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    monkeypatch.setenv("MPA_ARM", arm)
    _run(dist_worker.lsqb_dist, 2, [0, 1], cols, arm == "2")


# ---- the N = 8 placement (one worker per process) on ONE GPU --------------------------------
# On the node each worker process has a GPU of its own; here all eight share GPU 0.  The
# default arms every worker process's next task behind a one-wave doorbell wait
# (door_wait_kernel), so seven waiting tasks hold seven waves, not seven launch grids
# (round 3's in-kernel wait timed out here, profiles/r03_rehearsal_n248.txt).

@pytest.mark.parametrize("depth", ["1", "2"])
def test_lsq_descent_eight_processes_armed(built, depth):
    """BASELINE c2's N = 8 placement (rank 0 coordinates and serves worker 1, ranks 1-7 one
    worker each, device-armed by default, one or two tasks deep): the native loop's iterate,
    replies and messages bitwise equal to the one-process Python loop on the same shards, and
    every server armed its tasks."""
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    _run(dist_worker.lsq_descent_dist, 8, list(range(8)), {"MPA_TEST_EXPECT_ARMED": "1", "MPA_ARM_DEPTH": depth},
         timeout=240)


def test_lsq_descent_eight_processes_host_launched(built):
    """The same with MPA_ARM=0 (the serve loops launch each task when they see its doorbell)."""
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    _run(dist_worker.lsq_descent_dist, 8, list(range(8)), {"MPA_ARM": "0", "MPA_TEST_EXPECT_ARMED": "0"}, timeout=240)


@pytest.mark.parametrize("depth", ["1", "2"])
def test_lsqb_eight_processes_armed(built, monkeypatch, depth):
    """BASELINE c5's N = 8 placement: the batched 64-iterate task at 2048 columns (lsqp4's
    FULL form) in eight processes, every server device-armed (one or two tasks deep), every G
    against the fp64 oracle at 1e-5."""
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    monkeypatch.delenv("MPA_ARM", raising=False)
    monkeypatch.setenv("MPA_ARM_DEPTH", depth)
    _run(dist_worker.lsqb_dist, 8, list(range(8)), 2048, True, timeout=240)


@pytest.mark.parametrize("placement,env", [
    ([0, 1, 1, 1], {}),                                   # rank 1 serves 3 workers (host-launched, one batch)
    ([0, 1, 1, 1], {"MPA_ARM": "1"}),                     # ... each device-armed
    ([0, 1], {}),                                         # one worker per process: device-armed (default)
    ([0, 1], {"MPA_ARM": "0"}),                           # ... host-launched
    ([0, 1, 1], {"MPA_AHEAD": "0"}),                      # fused epoch kernel, no launch-ahead
    ([0, 1], {"MPA_FUSE": "0"}),                          # the unfused loop
    ([0, 1, 1], {"MPA_XGMI": "0"}),                       # payloads through the host mailbox
    ([0, 1], {"MPA_XGMI": "0", "MPA_ARM": "2"}),          # ... never armed (host mailbox)
])  # (MPA_WAIT_VALUE_OPS / MPA_GATHER, A/B switches, exist in the measurement build only)
def test_lsq_descent_two_processes(built, placement, env):
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    _run(dist_worker.lsq_descent_dist, 2, placement, env)


@pytest.mark.parametrize("config,epoch0", [("c3", 0), ("c4", 0), ("c4", 1000)])
def test_sched_eight_processes(built, config, epoch0):
    """BASELINE c3 (nwait 6 of 8, fp32) and c4 (fp64, worker 1 fresh + 5 others, stale results
    at weight 0.5) in the node's placement -- rank 0 plus seven one-worker processes, all on
    GPU 0 here -- on the oracle's golden schedule injected as the workers' delays and gated on
    rank 0: the oracle's repochs / active after every call, every chunk the gradient of the
    iterate sent at its epoch (1e-5 / 1e-12), the iterate equal to the numpy replay
    (dist_worker.lsq_sched_dist; one process: tests/test_gpu_configs.py)."""
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    _run(dist_worker.lsq_sched_dist, 8, list(range(8)), config, epoch0, timeout=240)


@pytest.mark.parametrize("config,epoch0,depth", [("c3", 0, "1"), ("c4", 0, "1"), ("c4", 1000, "1"), ("c5", 0, "1"),
                                                 ("c3", 0, "2"), ("c4", 1000, "2"), ("c5", 0, "2")])
def test_native_kofn_descent_eight_processes(built, monkeypatch, config, epoch0, depth):
    """The native k-of-n coordinator loop across processes -- bench.py's rank 0 at N > 1 for
    c3 (fp32, nwait 6 of 8), c4 (fp64, first_plus(5), stale weight 0.5, epoch0 0 and 1000) and
    c5 (bf16 batched, nwait 7) -- in the node's placement on GPU 0, ungated: the final iterate
    equals a torch fp64 replay of the per-epoch repochs it traced, every final chunk the gradient
    of the iterate sent at its repochs, remote and local stale harvests seen, a stale local
    re-dispatch launched at once on rank 0 of the node's placement and held into the next launch
    where rank 0 serves a second worker (c5)
    (dist_worker.descent_kofn_dist; one process: tests/test_gpu.py
    test_native_k_of_n_prearmed_with_stragglers); armed one or two tasks deep."""
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    monkeypatch.setenv("MPA_ARM_DEPTH", depth)
    world = max(dist_worker.KOFN_CONFIGS[config]["placement"]) + 1
    _run(dist_worker.descent_kofn_dist, world, config, epoch0, timeout=240)


@pytest.mark.parametrize("depth", ["1", "2"])
def test_armed_wait_timeout_cancels_the_task(built, monkeypatch, depth):
    """a device-armed task whose doorbell wait times out is cancelled (the one-wave
    door_wait_kernel stores the task's seq into its go word): no reply, no `done`, the error
    reported by the server's serve(); at depth 2 the task queued behind it is cancelled by the
    disarm."""
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    monkeypatch.setenv("MPA_ARM_DEPTH", depth)
    _run(dist_worker.armed_timeout_dist, 2, timeout=120)
