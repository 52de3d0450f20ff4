"""Per-rank bodies of the multi-process tests (spawned by tests/test_dist_cpu.py and
tests/test_gpu_procs.py).  Rank 0 is the coordinator; the other ranks serve the workers
placed on them.  Mirrors test/kmap2.jl with the workers spread over processes (as the
reference's MPI ranks are) instead of living in the coordinator's process."""
import os
import sys
import traceback
import uuid

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "mpistragglers.jl_amd")):
    if p not in sys.path:
        sys.path.insert(0, p)


def free_port():
    """A TCP port nothing listens on now (the kernel's pick for port 0): the rendezvous's.
    A random pick from a fixed range collided with a socket a previous test had left in use
    (EADDRINUSE, r04gc)."""
    import socket
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _init(rank, world, port):
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    return dist


def kmap2_dist(rank, world, port, transport, placement, result_q):
    """kmap2.jl semantics with workers on ranks `placement`; rank 0 reports failures."""
    import numpy as np
    try:
        dist = _init(rank, world, port)
        if transport == "hip":
            import torch
            torch.cuda.set_device(0)
        import mpiasyncpools as M
        n = len(placement)
        name = [f"/mpa_t{os.getpid()}_{uuid.uuid4().hex[:8]}"] if rank == 0 else [None]
        if rank == 0:
            comm = M.DistComm(n, placement, 0, name[0], 256, transport=transport)
        dist.broadcast_object_list(name, src=0)
        if rank != 0:
            comm = M.DistComm(n, placement, rank, name[0], 256, transport=transport)
        rng = np.random.default_rng(7)
        delays = (np.maximum(rng.random((n, 64)) / 10, 0.005) * 2e7).astype(np.int64)  # 0.1-2 ms
        for w in range(1, n + 1):
            if placement[w - 1] == rank:
                comm.set_task(w, "kmap2")
                comm.set_delays(w, delays[w - 1])
        dist.barrier()
        if rank != 0:
            comm.serve()          # session 1
            dist.barrier()
            comm.serve()          # session 2, until shutdown
            dist.barrier()
            comm.close()
            dist.destroy_process_group()
            return
        if transport == "hip":
            import torch

            def buf(k):
                return torch.zeros(k, dtype=torch.float64, device="cuda")
            host = lambda t: t.cpu().numpy()  # noqa: E731
        else:
            def buf(k):
                return np.zeros(k)
            host = lambda t: t  # noqa: E731
        pool = M.MPIAsyncPool(n)
        sendbuf, isendbuf = buf(1), buf(n)
        recvbuf, irecvbuf = buf(3 * n), buf(3 * n)
        errors = []
        for epoch in range(1, 41):
            sendbuf[0] = epoch
            rep = M.asyncmap_(pool, sendbuf, recvbuf, isendbuf, irecvbuf, comm, nwait=2)
            rb = host(recvbuf).reshape(n, 3)
            fresh = 0
            for i in range(n):
                if rep[i] == 0:
                    continue
                fresh += rep[i] == epoch
                if rb[i, 2] != rep[i] or rb[i, 0] != i + 1:
                    errors.append(("integrity", epoch, i, rb[i].tolist(), int(rep[i])))
            if fresh < 2:
                errors.append(("fresh", epoch, rep.tolist()))
        comm.pause_servers()
        dist.barrier()
        for _ in range(10):
            M.asyncmap_(pool, sendbuf, recvbuf, isendbuf, irecvbuf, comm, nwait=1)
            M.waitall_(pool, recvbuf, irecvbuf)
            if pool.active.any():
                errors.append(("waitall", pool.active.tolist()))
        f = lambda e, r: bool(r[0] == e)  # noqa: E731
        for _ in range(10):
            rep = M.asyncmap_(pool, sendbuf, recvbuf, isendbuf, irecvbuf, comm, nwait=f)
            if rep[0] != pool.epoch:
                errors.append(("predicate", rep.tolist(), pool.epoch))
        M.waitall_(pool, recvbuf, irecvbuf)
        rb = host(recvbuf).reshape(n, 3)
        for i in range(n):
            if rb[i, 1] != comm.tasks_done(i + 1):
                errors.append(("t", i, rb[i].tolist(), comm.tasks_done(i + 1)))
        comm.shutdown()
        dist.barrier()
        comm.close()
        dist.destroy_process_group()
        result_q.put(("ok", errors))
    except Exception:
        result_q.put(("exc", f"rank {rank}: " + traceback.format_exc()))
        raise


def lsq_dist(rank, world, port, placement, result_q):
    """Least-squares workers on several processes: each rank generates the shards of its
    workers on its GPU (Philox layout); rank 0 checks every chunk against the fp64 oracle
    gradient of the iterate sent at epoch repochs[i]."""
    import numpy as np
    try:
        dist = _init(rank, world, port)
        import torch
        torch.cuda.set_device(0)
        sys.path.insert(0, os.path.join(ROOT, "oracle"))
        import mpiasyncpools as M
        n, rows, cols, seed = len(placement), 4096, 1024, 21
        name = [f"/mpa_l{os.getpid()}_{uuid.uuid4().hex[:8]}"] if rank == 0 else [None]
        if rank == 0:
            comm = M.DistComm(n, placement, 0, name[0], cols * 4, transport="hip")
        dist.broadcast_object_list(name, src=0)
        if rank != 0:
            comm = M.DistComm(n, placement, rank, name[0], cols * 4, transport="hip")
        keep = []
        for w in range(1, n + 1):
            if placement[w - 1] == rank:
                A = torch.empty(rows, cols, device="cuda")
                b = torch.empty(rows, device="cuda")
                M.generate(A, seed, 0, (w - 1) * rows * cols, float(np.float32(1 / np.sqrt(cols))))
                M.generate(b, seed, 1, (w - 1) * rows, 1.0)
                keep.append((A, b))
                comm.set_task_lsq(w, A, b)
                comm.set_delays(w, [0, 2_000_000, 0, 0, 5_000_000][w % 5:] + [0])
        torch.cuda.synchronize()
        dist.barrier()
        if rank != 0:
            comm.serve()
            dist.barrier()
            comm.close()
            dist.destroy_process_group()
            return
        import lsq
        A_all = lsq.gen_matrix(seed, 0, n * rows, cols, "f32")
        b_all = lsq.gen_vector(seed, 0, n * rows, "f32")
        pool = M.MPIAsyncPool(n)
        x = torch.zeros(cols, device="cuda")
        isend = torch.zeros(n * cols, device="cuda")
        recv = torch.zeros(n * cols, device="cuda")
        irecv = torch.zeros_like(recv)
        sent, errors = {}, []
        for epoch in range(1, 11):
            sent[epoch] = x.cpu().numpy().copy()
            rep = M.asyncmap_(pool, x, recv, isend, irecv, comm, nwait=3)
            ch = recv.cpu().numpy().reshape(n, cols)
            for i in range(n):
                if rep[i] == 0:
                    continue
                g = lsq.shard_gradient(A_all[i * rows:(i + 1) * rows], b_all[i * rows:(i + 1) * rows], sent[int(rep[i])])
                e = lsq.rel_err(ch[i], g)
                if not e <= 1e-5:
                    errors.append(("grad", epoch, i, int(rep[i]), e))
            w = (rep == epoch).astype(np.float64) * (n / max(1, int((rep == epoch).sum())))
            comm.lsq_update(x, recv, n, w, 0.05)
        M.waitall_(pool, recv, irecv)
        comm.shutdown()
        dist.barrier()
        comm.close()
        dist.destroy_process_group()
        result_q.put(("ok", errors))
    except Exception:
        result_q.put(("exc", f"rank {rank}: " + traceback.format_exc()))
        raise


def lsq_dist_armed(rank, world, port, placement, delayed, result_q):
    """Pre-armed serving (workers without a delay schedule wait on their doorbell inside
    the GPU queue): two serve sessions with a pause between them (armed tasks cancelled and
    re-armed), nwait = n then nwait = 2 with stale results, every chunk checked against the
    fp64 gradient of the iterate of its epoch."""
    import numpy as np
    try:
        dist = _init(rank, world, port)
        import torch
        torch.cuda.set_device(0)
        sys.path.insert(0, os.path.join(ROOT, "oracle"))
        import mpiasyncpools as M
        n, rows, cols, seed = len(placement), 3000, 512, 23
        name = [f"/mpa_a{os.getpid()}_{uuid.uuid4().hex[:8]}"] if rank == 0 else [None]
        if rank == 0:
            comm = M.DistComm(n, placement, 0, name[0], cols * 4, transport="hip")
        dist.broadcast_object_list(name, src=0)
        if rank != 0:
            comm = M.DistComm(n, placement, rank, name[0], cols * 4, transport="hip")
        keep = []
        for w in range(1, n + 1):
            if placement[w - 1] == rank:
                A = torch.empty(rows, cols, device="cuda")
                b = torch.empty(rows, device="cuda")
                M.generate(A, seed, 0, (w - 1) * rows * cols, float(np.float32(1 / np.sqrt(cols))))
                M.generate(b, seed, 1, (w - 1) * rows, 1.0)
                keep.append((A, b))
                comm.set_task_lsq(w, A, b)
                if w in delayed:
                    comm.set_delays(w, [3_000_000, 0, 1_000_000])
        torch.cuda.synchronize()
        dist.barrier()
        if rank != 0:
            for _ in range(2):
                comm.serve()
                dist.barrier()
            comm.close()
            dist.destroy_process_group()
            return
        import lsq
        A_all = lsq.gen_matrix(seed, 0, n * rows, cols, "f32")
        b_all = lsq.gen_vector(seed, 0, n * rows, "f32")
        pool = M.MPIAsyncPool(n)
        x = torch.zeros(cols, device="cuda")
        isend = torch.zeros(n * cols, device="cuda")
        recv = torch.zeros(n * cols, device="cuda")
        irecv = torch.zeros_like(recv)
        sent, errors = {}, []
        for session, nwait in ((1, n), (2, 2)):
            for _ in range(6):
                epoch = pool.epoch + 1
                sent[epoch] = x.cpu().numpy().copy()
                rep = M.asyncmap_(pool, x, recv, isend, irecv, comm, nwait=nwait)
                ch = recv.cpu().numpy().reshape(n, cols)
                if int((rep == epoch).sum()) < nwait:
                    errors.append(("fresh", session, epoch, rep.tolist()))
                for i in range(n):
                    if rep[i] == 0:
                        continue
                    g = lsq.shard_gradient(A_all[i * rows:(i + 1) * rows], b_all[i * rows:(i + 1) * rows],
                                           sent[int(rep[i])])
                    e = lsq.rel_err(ch[i], g)
                    if not e <= 1e-5:
                        errors.append(("grad", session, epoch, i, int(rep[i]), e))
                w = (rep == epoch).astype(np.float64) * (n / max(1, int((rep == epoch).sum())))
                comm.lsq_update(x, recv, n, w, 0.05)
            M.waitall_(pool, recv, irecv)
            if session == 1:
                comm.pause_servers()
                dist.barrier()
        comm.shutdown()
        dist.barrier()
        comm.close()
        dist.destroy_process_group()
        result_q.put(("ok", errors))
    except Exception:
        result_q.put(("exc", f"rank {rank}: " + traceback.format_exc()))
        raise


def lsqb_dist(rank, world, port, placement, cols, expect_armed, result_q):
    """The batched 64-iterate variant across processes (pre-armed on the serving rank); at
    2048 columns and 1024 rows every task takes lsqp4's FULL form, the armed one included."""
    import numpy as np
    try:
        dist = _init(rank, world, port)
        import torch
        torch.cuda.set_device(0)
        sys.path.insert(0, os.path.join(ROOT, "oracle"))
        import mpiasyncpools as M
        import lsq
        n, rows, K, seed = len(placement), (1024 if cols == 2048 else 1000), 64, 29
        name = [f"/mpa_b{os.getpid()}_{uuid.uuid4().hex[:8]}"] if rank == 0 else [None]
        if rank == 0:
            comm = M.DistComm(n, placement, 0, name[0], cols * K * 4, transport="hip")
        dist.broadcast_object_list(name, src=0)
        if rank != 0:
            comm = M.DistComm(n, placement, rank, name[0], cols * K * 4, transport="hip")
        A_all = lsq.gen_matrix(seed, 0, n * rows, cols, "bf16")
        B_all = lsq.gen_matrix(seed, 0, n * rows, K, "bf16", stream=lsq.STREAM_B, scale=np.float32(1.0))

        def bf16(bits):
            return torch.from_numpy(np.ascontiguousarray(bits).view(np.int16)).cuda().view(torch.bfloat16)
        keep = []
        for w in range(1, n + 1):
            if placement[w - 1] == rank:
                A, B = bf16(A_all[(w - 1) * rows:w * rows]), bf16(B_all[(w - 1) * rows:w * rows])
                keep.append((A, B))
                comm.set_task_lsq_batch(w, A, B)
        torch.cuda.synchronize()
        dist.barrier()
        armed = [None] * world
        if rank != 0:
            comm.serve()
            dist.all_gather_object(armed, comm.counter("armed"))
            dist.barrier()
            comm.close()
            dist.destroy_process_group()
            return
        pool = M.MPIAsyncPool(n)
        send = torch.zeros(cols * K, dtype=torch.bfloat16, device="cuda")
        isend = torch.zeros(n * cols * K, dtype=torch.bfloat16, device="cuda")
        recv = torch.zeros(n * cols * K, device="cuda")
        irecv = torch.zeros_like(recv)
        errors = []
        for epoch in range(1, 5):
            X = lsq.gen_matrix(300 + epoch, 0, cols, K, "bf16", stream=lsq.STREAM_X, scale=np.float32(0.5))
            send.copy_(bf16(X).view(-1))
            M.asyncmap_(pool, send, recv, isend, irecv, comm, nwait=n)
            ch = recv.cpu().numpy().reshape(n, cols, K)
            for i in range(n):
                G = lsq.batched_shard_gradient(A_all[i * rows:(i + 1) * rows], B_all[i * rows:(i + 1) * rows], X)
                e = lsq.rel_err(ch[i], G)
                if not e <= 1e-5:  # BASELINE north_star: 1e-5 (fp32 accumulate)
                    errors.append(("G", epoch, i, e))
        comm.shutdown()
        dist.all_gather_object(armed, 0)
        if expect_armed is not None and any((a > 0) != expect_armed for a in armed[1:]):
            errors.append(("armed launches per rank", armed, expect_armed))
        dist.barrier()
        comm.close()
        dist.destroy_process_group()
        result_q.put(("ok", errors))
    except Exception:
        result_q.put(("exc", f"rank {rank}: " + traceback.format_exc()))
        raise


def lsq_descent_dist(rank, world, port, placement, env, result_q):
    """The native descent loop (fused epoch kernel; launch-ahead at nwait = n: the next
    epoch's doorbells queued behind stream waits on the remote completion words) with
    workers on several processes, against the same loop run by Python in one process on
    the same shards: identical iterates, bitwise.  A task's summation grouping follows its
    launch grid (a share of the launch, capped at rows / 16 workgroups), and the two runs
    batch the tasks differently, so the shards are small enough (512 rows: 32 workgroups)
    that every task runs the same grid in both runs."""
    import numpy as np
    try:
        os.environ.update(env)
        dist = _init(rank, world, port)
        import torch
        torch.cuda.set_device(0)
        import mpiasyncpools as M
        # 512 rows (32 workgroups) while a task's share of the one-process launch (192 / n
        # workgroups) is at least that; 384 (24) at n = 8
        n, cols, seed, epochs, eta = len(placement), 1024, 23, 7, 0.02
        rows = min(512, 16 * (192 // n))
        name = [f"/mpa_d{os.getpid()}_{uuid.uuid4().hex[:8]}"] if rank == 0 else [None]
        if rank == 0:
            comm = M.DistComm(n, placement, 0, name[0], cols * 4, transport="hip")
        dist.broadcast_object_list(name, src=0)
        if rank != 0:
            comm = M.DistComm(n, placement, rank, name[0], cols * 4, transport="hip")

        def shard(w):
            A = torch.empty(rows, cols, device="cuda")
            b = torch.empty(rows, device="cuda")
            M.generate(A, seed, 0, (w - 1) * rows * cols, float(np.float32(1 / np.sqrt(cols))))
            M.generate(b, seed, 1, (w - 1) * rows, 1.0)
            return A, b

        keep = []
        for w in range(1, n + 1):
            if placement[w - 1] == rank:
                keep.append(shard(w))
                comm.set_task_lsq(w, *keep[-1])
        torch.cuda.synchronize()
        dist.barrier()
        armed = [None] * world  # device-armed launches per rank (servers), checked by rank 0
        if rank != 0:
            comm.serve()
            dist.all_gather_object(armed, comm.counter("armed"))
            dist.barrier()
            comm.close()
            dist.destroy_process_group()
            return
        pool = M.MPIAsyncPool(n)
        x = torch.zeros(cols, device="cuda")
        isend = torch.zeros(n * cols, device="cuda")
        recv = torch.zeros(n * cols, device="cuda")
        irecv = torch.zeros_like(recv)
        M.lsq_descent(pool, comm, x, recv, isend, irecv, n, eta, epochs)
        torch.cuda.synchronize()
        errors = []
        if pool.epoch != epochs or list(pool.repochs) != [epochs] * n or any(pool.active):
            errors.append(("state", pool.epoch, list(pool.repochs), list(pool.active)))
        want = "host" if env.get("MPA_XGMI") == "0" else "device"
        paths = [comm.payload_path(w) for w in range(1, n + 1) if placement[w - 1] != 0]
        if paths != [want] * len(paths):
            errors.append(("payload path", paths, want))
        # isendbuf holds the message of the last epoch; recvbuf its harvested replies
        got_isend = isend.clone()
        comm.shutdown()
        dist.all_gather_object(armed, 0)
        want_armed = env.get("MPA_TEST_EXPECT_ARMED")
        if want_armed is not None and any((a > 0) != (want_armed == "1") for a in armed[1:]):
            errors.append(("armed launches per rank", armed, want_armed))
        dist.barrier()
        comm.close()
        dist.destroy_process_group()
        # the same loop in one process, Python side (asyncmap_ + lsq_update)
        lc = M.DeviceComm(n)
        shards = [shard(w) for w in range(1, n + 1)]
        for w in range(1, n + 1):
            lc.set_task_lsq(w, *shards[w - 1])
        lp = M.MPIAsyncPool(n)
        x2 = torch.zeros(cols, device="cuda")
        isend2 = torch.zeros(n * cols, device="cuda")
        recv2 = torch.zeros(n * cols, device="cuda")
        irecv2 = torch.zeros_like(recv2)
        for _ in range(epochs):
            rep = M.asyncmap_(lp, x2, recv2, isend2, irecv2, lc, nwait=n)
            lc.lsq_update(x2, recv2, n, (rep == lp.epoch) * 1.0, eta)
        torch.cuda.synchronize()
        if not torch.equal(x.view(torch.int32), x2.view(torch.int32)):
            errors.append(("x", float((x - x2).abs().max())))
        if not torch.equal(recv.view(torch.int32), recv2.view(torch.int32)):
            errors.append(("recvbuf", float((recv - recv2).abs().max())))
        if not torch.equal(got_isend.view(torch.int32), isend2.view(torch.int32)):
            errors.append(("isendbuf",))
        lc.close()
        result_q.put(("ok", errors))
    except Exception:
        result_q.put(("exc", f"rank {rank}: " + traceback.format_exc()))
        raise


SCHED_CONFIGS = {
    # BASELINE configs[2] (c3): fp32, nwait 6 of 8, stale results dropped; configs[3] (c4): fp64,
    # worker 1 fresh + 5 others (mpa_nwait_first_plus), stale results at weight 0.5
    "c3": dict(scenario="gpu_sep_c3", dt="f32", nwait=6, stale=0.0, tol=1e-5, seed=43),
    "c4": dict(scenario="gpu_sep_c4_first_plus_5", dt="f64", nwait="first_plus5", stale=0.5, tol=1e-12, seed=41),
}


def lsq_sched_dist(rank, world, port, placement, config, epoch0, result_q):
    """BASELINE c3 / c4 in the node's placement (rank 0 coordinates and serves worker 1, ranks
    1-7 serve one worker each), on the oracle's golden schedule: every worker process injects
    the schedule's durations as its task delays (so its tasks are host-launched by its serve
    loop's timer, not device-armed), and rank 0 runs the Python-driven coordinator loop under the
    oracle's gate (tests/gated.py), checking what tests/test_gpu_configs.py checks in one
    process: repochs / active after every asyncmap! equal the oracle's, every chunk i equals the
    fp64 gradient of the iterate sent at epoch repochs[i] (1e-5 fp32 / 1e-12 fp64), the iterate
    equals a numpy replay of the update (fresh weight 1, stale `stale`, never heard from 0,
    scaled by n / sum(w))."""
    import numpy as np
    try:
        dist = _init(rank, world, port)
        import torch
        torch.cuda.set_device(0)
        sys.path.insert(0, os.path.join(ROOT, "oracle"))
        import gated
        import lsq
        import mpiasyncpools as M
        cfg = SCHED_CONFIGS[config]
        sc = next(s for s in gated.scenarios() if s["name"] == cfg["scenario"])
        n, rows, cols, eta = sc["n"], 512, 2048, 0.2
        assert n == len(placement)
        es = 8 if cfg["dt"] == "f64" else 4
        tdt = torch.float64 if cfg["dt"] == "f64" else torch.float32
        name = [f"/mpa_s{os.getpid()}_{uuid.uuid4().hex[:8]}"] if rank == 0 else [None]
        if rank == 0:
            comm = M.DistComm(n, placement, 0, name[0], cols * es, transport="hip")
        dist.broadcast_object_list(name, src=0)
        if rank != 0:
            comm = M.DistComm(n, placement, rank, name[0], cols * es, transport="hip")
        dur = np.asarray(sc["durations_ns"], dtype=np.int64).reshape(n, -1)
        keep = []
        for w in range(1, n + 1):
            if placement[w - 1] == rank:
                A = lsq.gen_matrix(cfg["seed"], (w - 1) * rows, rows, cols, cfg["dt"])
                b = lsq.gen_vector(cfg["seed"], (w - 1) * rows, rows, cfg["dt"])
                keep.append((torch.from_numpy(A).cuda(), torch.from_numpy(b).cuda()))
                comm.set_task_lsq(w, *keep[-1])
                comm.set_delays(w, dur[w - 1])
        torch.cuda.synchronize()
        dist.barrier()
        if rank != 0:
            comm.serve()
            dist.barrier()
            comm.close()
            dist.destroy_process_group()
            return
        A_all, b_all = lsq.gen_matrix(cfg["seed"], 0, n * rows, cols, cfg["dt"]), lsq.gen_vector(cfg["seed"], 0, n * rows, cfg["dt"])
        comm.set_gate(*gated.oracle_gate(sc)[1])
        nwait = M.first_plus(5) if cfg["nwait"] == "first_plus5" else cfg["nwait"]
        pool = M.MPIAsyncPool(n, epoch0=epoch0)
        x = torch.zeros(cols, dtype=tdt, device="cuda")
        isend = torch.zeros(n * cols, dtype=tdt, device="cuda")
        recv = torch.zeros(n * cols, dtype=tdt, device="cuda")
        irecv = torch.zeros_like(recv)
        errors, sent, got, reps, ws = [], {}, [], [], []
        steps = [(op, ref) for op, ref in zip(sc["ops"], sc["results"]) if op["op"] == "asyncmap"]
        for k, (op, ref) in enumerate(steps):
            epoch = epoch0 + k + 1
            sent[epoch] = x.clone()
            rep = M.asyncmap_(pool, x, recv, isend, irecv, comm, nwait=nwait).copy()
            ref_rep = [r + epoch0 for r in ref["repochs"]]  # the oracle runs at epoch0 = 0
            if rep.tolist() != ref_rep or pool.active.astype(int).tolist() != ref["active"]:
                errors.append(("trace", k, rep.tolist(), ref_rep, pool.active.astype(int).tolist(), ref["active"]))
            got.append(recv.clone())
            w = np.zeros(n)
            for i in range(n):
                if ref["repochs"][i] != 0:  # never heard from: chunk unfilled, weight 0
                    w[i] = 1.0 if rep[i] == epoch else cfg["stale"]
            w *= n / w.sum() if w.sum() > 0 else 0.0
            comm.lsq_update(x, recv, n, w, eta)
            reps.append(rep)
            ws.append(w)
        M.waitall_(pool, recv, irecv)
        torch.cuda.synchronize()
        paths = [comm.payload_path(w) for w in range(1, n + 1) if placement[w - 1] != 0]
        if paths != ["device"] * len(paths):
            errors.append(("payload path", paths))
        comm.shutdown()
        dist.barrier()
        comm.close()
        dist.destroy_process_group()
        tol = cfg["tol"]
        sent = {e: v.cpu().numpy().astype(np.float64) for e, v in sent.items()}
        x_np = np.zeros(cols)
        for k, (rep, w, r) in enumerate(zip(reps, ws, got)):
            epoch = epoch0 + k + 1
            if not (np.array_equal(sent[epoch], x_np) or lsq.rel_err(sent[epoch], x_np) <= tol):
                errors.append(("iterate", k, lsq.rel_err(sent[epoch], x_np)))
            chunks = r.cpu().numpy().reshape(n, cols).astype(np.float64)
            for i in range(n):
                if rep[i] - epoch0 == 0:
                    continue
                g = lsq.shard_gradient(A_all[i * rows:(i + 1) * rows], b_all[i * rows:(i + 1) * rows], sent[int(rep[i])])
                e = lsq.rel_err(chunks[i], g)
                if not e <= tol:
                    errors.append(("chunk", k, i, int(rep[i]), e))
            x_np = x_np - eta * (w[:, None] * chunks).sum(0)
        if lsq.rel_err(x.cpu().numpy().astype(np.float64), x_np) > tol:
            errors.append(("final iterate", lsq.rel_err(x.cpu().numpy().astype(np.float64), x_np)))
        result_q.put(("ok", errors))
    except Exception:
        result_q.put(("exc", f"rank {rank}: " + traceback.format_exc()))
        raise


# The native k-of-n loop across processes: what bench.py's rank 0 runs at
# N > 1 for c3 / c4 / c5 (make_loop: mpa_lsq_descent / mpa_lsqb_descent on a DistComm).  Worker 1
# lives on rank 0 and is made the straggler -- c3 by an injected 30 ms delay per task, c5 by a shard
# 4096x the others' (an undelayed task: the kind a stale re-dispatch may hold) -- so its stale
# replies and re-dispatches (src/MPIAsyncPools.jl:177-184) happen every few epochs; remote workers
# carry injected delays (`remote`: Exp(mean ms) per task, or "spikes": 20 ms every 4th task of the
# last worker, none for the others), their stale replies harvested from other processes' GPUs.
# eta keeps the slow worker's gradient from converging towards zero over the run (its own L =
# rows / (3 cols) is large): a gradient that cancels down to its rounding has no relative accuracy
# left to check.
KOFN_CONFIGS = {
    # c3: fp32, nwait 6 of 8, stale results dropped; the node's placement (rank 0 serves worker
    # 1 only), so worker 1's stale re-dispatch launches at once (nothing else of rank 0's runs)
    "c3": dict(dt="f32", cols=2048, nwait=6, stale=0.0, tol=1e-5, placement=list(range(8)),
               rows=[256] * 8, local_delay_ms=30.0, remote=0.1, epochs=60, eta=0.05),
    # c4: fp64, worker 1 fresh + 5 others (first_plus), stale results at weight 0.5; worker 1 fast
    "c4": dict(dt="f64", cols=2048, nwait="first_plus5", stale=0.5, tol=1e-12, placement=list(range(8)),
               rows=[256] * 8, local_delay_ms=None, remote=1.0, epochs=40, eta=0.05),
    # c5: the batched 64-iterate variant (bf16 messages, fp32 accumulate), nwait 7 of 8; rank 0
    # serves workers 1 (slow: ~1 ms of lsqp4) and 2 (fast); worker 2's next task queues behind
    # worker 1's running launch on the coordinator stream, so worker 1's stale re-dispatch is
    # HELD and joins worker 2's next launch; the last worker's 20 ms spikes make it the stale one
    # now and then
    "c5": dict(dt="bf16", cols=2048, nwait=7, stale=0.0, tol=1e-5, placement=[0, 0, 1, 2, 3, 4, 5, 6],
               rows=[1 << 20] + [256] * 7, local_delay_ms=None, remote="spikes", epochs=30, eta=2e-5, k=64),
}


def descent_kofn_dist(rank, world, port, config, epoch0, result_q):
    """BASELINE c3 / c4 / c5's coordinator loop in native code (M.lsq_descent / M.lsqb_descent,
    as bench.py runs it at N > 1) on rank 0 of a DistComm (the node's placement, rank 0 serving
    worker 1 and ranks 1-7 one worker each; c5: rank 0 serving workers 1 and 2), ungated, at
    nwait < n.  Whatever the timing, the loop
    must compute what the reference's coordinator computes from the repochs it saw
    (examples/iterative_example.jl:41-46): rank 0 traces the per-epoch repochs
    (MPA_DESCENT_TRACE=1) and replays them in torch fp64 on the device -- each chunk i the
    gradient of the iterate sent at its repochs[i] (c5: the bf16 rounding of that iterate),
    weights fresh 1 / stale `stale` / never heard from 0, scaled by n / sum(w) -- and the final
    iterate must match the replay (1e-5 fp32 and bf16-in/fp32-accumulate, 1e-12 fp64); every
    final chunk is the gradient of the iterate sent at its repochs (after waitall!); the paths
    the node's run depends on did run: remote stale harvests, stale harvests of the slow local
    worker (c3, c5), its re-dispatch launched at once where nothing else of rank 0's runs (c3: no
    hold) and held into worker 2's next launch where it would queue behind it (c5), the
    first_plus predicate on remote completions (c4)."""
    import re
    import tempfile
    import numpy as np
    try:
        dist = _init(rank, world, port)
        import torch
        torch.cuda.set_device(0)
        import mpiasyncpools as M
        cfg = KOFN_CONFIGS[config]
        placement, cols, k = cfg["placement"], cfg["cols"], cfg.get("k", 1)
        n = len(placement)
        assert world == max(placement) + 1, (world, placement)
        tdt = {"f32": torch.float32, "f64": torch.float64, "bf16": torch.bfloat16}[cfg["dt"]]
        es = {"f32": 4, "f64": 8, "bf16": 4}[cfg["dt"]]  # the reply's element size (c5: fp32 G)
        rows = cfg["rows"]
        scale = 1 / np.sqrt(cols) if cfg["dt"] == "f64" else float(np.float32(1 / np.sqrt(cols)))

        def shard(w):
            A = torch.empty(rows[w - 1], cols, dtype=tdt, device="cuda")
            b = torch.empty((rows[w - 1], k) if k > 1 else rows[w - 1], dtype=tdt, device="cuda")
            M.generate(A, 61 + w, 0, 0, scale)
            M.generate(b, 61 + w, 1, 0, 1.0)
            return A, b

        name = [f"/mpa_k{os.getpid()}_{uuid.uuid4().hex[:8]}"] if rank == 0 else [None]
        if rank == 0:
            comm = M.DistComm(n, placement, 0, name[0], cols * k * es, transport="hip")
        dist.broadcast_object_list(name, src=0)
        if rank != 0:
            comm = M.DistComm(n, placement, rank, name[0], cols * k * es, transport="hip")
        keep = []
        for w in (v for v in range(1, n + 1) if placement[v - 1] == rank):
            keep.append(shard(w))
            if k > 1:
                comm.set_task_lsq_batch(w, *keep[-1])
            else:
                comm.set_task_lsq(w, *keep[-1])
            if rank == 0 and cfg["local_delay_ms"]:
                comm.set_delays(w, [int(cfg["local_delay_ms"] * 1e6)])
            elif rank != 0 and cfg["remote"] == "spikes":
                if w == n:
                    comm.set_delays(w, [0, 0, 0, 20_000_000])
            elif rank != 0:
                rng = np.random.default_rng([17, w])
                comm.set_delays(w, rng.exponential(cfg["remote"] * 1e6, size=512).astype(np.int64))
        torch.cuda.synchronize()
        dist.barrier()
        if rank != 0:
            comm.serve()
            dist.barrier()
            comm.close()
            dist.destroy_process_group()
            return
        names = ("held", "held_joined", "stale_deferred", "head_steps", "epoch_kernels", "task_launches")
        c0 = {key: comm.counter(key) for key in names}
        nwait = M.first_plus(5) if cfg["nwait"] == "first_plus5" else cfg["nwait"]
        pool = M.MPIAsyncPool(n, epoch0=epoch0)
        if k > 1:
            x = torch.zeros(cols * k, device="cuda")
            xb = torch.zeros(cols * k, dtype=torch.bfloat16, device="cuda")
            isend = torch.zeros(n * cols * k, dtype=torch.bfloat16, device="cuda")
            recv = torch.zeros(n * cols * k, device="cuda")
        else:
            x = torch.zeros(cols, dtype=tdt, device="cuda")
            isend = torch.zeros(n * cols, dtype=tdt, device="cuda")
            recv = torch.zeros(n * cols, dtype=tdt, device="cuda")
        irecv = torch.zeros_like(recv)
        epochs = cfg["epochs"]
        # the native loop's per-epoch trace goes to fd 2 (C stdio): into a file for the replay
        os.environ["MPA_DESCENT_TRACE"] = "1"
        with tempfile.TemporaryFile(mode="w+") as tf:
            saved = os.dup(2)
            os.dup2(tf.fileno(), 2)
            try:
                if k > 1:
                    M.lsqb_descent(pool, comm, x, xb, recv, isend, irecv, nwait, cfg["eta"], epochs,
                                   stale_weight=cfg["stale"])
                else:
                    M.lsq_descent(pool, comm, x, recv, isend, irecv, nwait, cfg["eta"], epochs,
                                  stale_weight=cfg["stale"])
                torch.cuda.synchronize()
            finally:
                os.dup2(saved, 2)
                os.close(saved)
            tf.seek(0)
            err = tf.read()
        os.environ.pop("MPA_DESCENT_TRACE")
        got = {key: comm.counter(key) - v for key, v in c0.items()}
        x_end = x.clone()
        M.waitall_(pool, recv, irecv)
        torch.cuda.synchronize()
        final_rep = [int(v) for v in pool.repochs]
        final_chunks = recv.clone()
        paths = [comm.payload_path(v) for v in range(1, n + 1) if placement[v - 1] != 0]
        comm.shutdown()
        dist.barrier()
        comm.close()
        dist.destroy_process_group()
        errors = []
        if paths != ["device"] * len(paths):
            errors.append(("payload path", paths))
        trace = [(int(m.group(1)), list(map(int, m.group(2).split())))
                 for m in re.finditer(r"\[mpa descent\] epoch (\d+) repochs ([\d ]+) \|", err)]
        if [e for e, _ in trace] != list(range(epoch0 + 1, epoch0 + epochs + 1)):
            errors.append(("trace epochs", [e for e, _ in trace][:5], len(trace), err[-400:]))
            result_q.put(("ok", errors))
            return
        # the fp64 replay on the device, each worker's gradient memoised per sent epoch
        A64, b64 = [], []
        for v in range(1, n + 1):
            Av, bv = shard(v)
            A64.append(Av.double())
            b64.append(bv.double())
            del Av, bv
        memo = {}

        def msg(xv):  # what the workers receive: the iterate (c5: its bf16 rounding, cols x 64)
            return xv.to(torch.bfloat16).double().view(cols, k) if k > 1 else xv

        def grad(i, e):
            if (i, e) not in memo:
                X = msg(xs[e - epoch0 - 1])
                memo[(i, e)] = (A64[i].T @ (A64[i] @ X - b64[i])).reshape(-1)
            return memo[(i, e)]

        xs = [torch.zeros(cols * k, dtype=torch.float64, device="cuda")]  # xs[e-epoch0-1]: sent at epoch e
        received = [False] * n
        stale_remote = stale_local = 0
        prev = [epoch0] * n
        for e, rep in trace:
            fresh = [i for i in range(n) if rep[i] == e]
            for i in range(n):
                received[i] = received[i] or rep[i] != epoch0
                if rep[i] != prev[i] and rep[i] != e:  # a reply of an earlier epoch harvested in this call
                    if placement[i] == 0:
                        stale_local += 1
                    else:
                        stale_remote += 1
            prev = rep
            if cfg["nwait"] == "first_plus5":
                ok = rep[0] == e and len(fresh) >= 6
            else:
                ok = len(fresh) >= cfg["nwait"]
            if not ok:
                errors.append(("nwait not satisfied", e, rep))
            wts = [1.0 if rep[i] == e else (cfg["stale"] if received[i] else 0.0) for i in range(n)]
            s = n / sum(wts) if sum(wts) > 0 else 0.0
            upd = torch.zeros_like(xs[0])
            for i in range(n):
                if wts[i] != 0.0:
                    upd += (wts[i] * s) * grad(i, rep[i])
            xs.append(xs[-1] - cfg["eta"] * upd)
        tol = cfg["tol"]
        rel = float(torch.linalg.norm(x_end.double() - xs[-1]) / torch.linalg.norm(xs[-1]))
        if not rel <= tol:
            errors.append(("final iterate vs fp64 replay", rel))
        ch = final_chunks.view(n, -1).double()
        for i in range(n):
            r = final_rep[i]
            if r == epoch0:
                continue
            g = grad(i, r)
            e_i = float(torch.linalg.norm(ch[i] - g) / torch.linalg.norm(g))
            if not e_i <= tol:
                errors.append(("final chunk", i, r, e_i))
        # the stale paths the node's run takes (their mix depends on the box's timing: remote
        # workers of eight processes on one loaded GPU range from 0.1 to 10 ms, r06l)
        if config == "c4" and not stale_remote >= 1:
            errors.append(("no remote stale harvest", stale_remote))
        if config == "c3" and not stale_local + stale_remote >= 1:
            errors.append(("no stale harvest", stale_local, stale_remote))
        if config == "c5" and not stale_local >= 1:
            errors.append(("no stale harvest of the slow local worker", stale_local))
        if config == "c3" and got["held"] != 0:
            errors.append(("held a re-dispatch with nothing else of rank 0's in flight", got))
        if config == "c5" and not (got["held"] >= 1 and got["held_joined"] >= 1):
            errors.append(("no held re-dispatch joined a launch", got))
        lat = [list(map(float, m.group(1).split()))
               for m in re.finditer(r"\| latency ms ([\d. ]+)\n", err)]
        med_lat = [round(float(np.median([row[i] for row in lat])), 2) for i in range(n)] if lat else None
        print("descent k-of-n %s epoch0 %d: %s, stale harvests local %d remote %d, iterate rel %.2e, "
              "median latency per worker (ms) %s" % (config, epoch0, got, stale_local, stale_remote, rel, med_lat),
              flush=True)
        if errors:
            errors.append(("median latency per worker (ms)", med_lat))
            errors.append(("first epochs", [ln for ln in err.splitlines() if ln.startswith("[mpa descent]")][:12]))
        result_q.put(("ok", errors))
    except Exception:
        result_q.put(("exc", f"rank {rank}: " + traceback.format_exc()))
        raise


def armed_timeout_dist(rank, world, port, result_q):
    """A device-armed task whose doorbell never comes: rank 1 serves one least-squares
    worker, armed behind a one-wave doorbell wait bounded at MPA_WAIT_TIMEOUT_S = 2 s; rank 0 posts
    it once (the path is decided, the task runs, the server arms the next one) and then never again.
    The wait must time out, cancel the queued task -- which then neither writes its reply nor
    publishes `done` -- and report the device error: rank 1's serve() raises it, and the worker's
    task count stays at 1."""
    import time
    import numpy as np
    try:
        if rank == 1:
            os.environ["MPA_WAIT_TIMEOUT_S"] = "2"
        os.environ.pop("MPA_ARM", None)
        dist = _init(rank, world, port)
        import torch
        torch.cuda.set_device(0)
        import mpiasyncpools as M
        n, rows, cols = 1, 512, 256
        name = [f"/mpa_to{os.getpid()}_{uuid.uuid4().hex[:8]}"] if rank == 0 else [None]
        if rank == 0:
            comm = M.DistComm(n, [1], 0, name[0], cols * 4, transport="hip")
        dist.broadcast_object_list(name, src=0)
        if rank != 0:
            comm = M.DistComm(n, [1], rank, name[0], cols * 4, transport="hip")
            A = torch.empty(rows, cols, device="cuda")
            b = torch.empty(rows, device="cuda")
            M.generate(A, 3, 0, 0, float(np.float32(1 / np.sqrt(cols))))
            M.generate(b, 3, 1, 0, 1.0)
            comm.set_task_lsq(1, A, b)
            torch.cuda.synchronize()
        dist.barrier()
        if rank != 0:
            t0 = time.perf_counter()
            err = None
            try:
                comm.serve()
            except Exception as e:  # the expected outcome
                err = str(e)
            msg = [(err, round(time.perf_counter() - t0, 2), comm.counter("armed"))]
            dist.broadcast_object_list(msg, src=1)
            dist.barrier()
            comm.close()
            dist.destroy_process_group()
            return
        pool = M.MPIAsyncPool(n)
        x = torch.zeros(cols, device="cuda")
        recv = torch.zeros(cols, device="cuda")
        M.asyncmap_(pool, x, recv, torch.zeros(cols, device="cuda"), torch.zeros_like(recv), comm, nwait=1)
        errors = []
        if comm.tasks_done(1) != 1:
            errors.append(("first task", comm.tasks_done(1)))
        msg = [None]
        dist.broadcast_object_list(msg, src=1)  # rank 1's serve() returned (or raised)
        err, waited, armed = msg[0]
        if not err or "in-kernel wait timed out" not in err:
            errors.append(("serve() did not report the timed-out wait", err))
        if not (1.5 <= waited <= 60):
            errors.append(("serve() ended after", waited))
        if armed < 2:
            errors.append(("armed launches", armed))
        time.sleep(0.5)
        if comm.tasks_done(1) != 1:  # the cancelled task published nothing
            errors.append(("the timed-out task published", comm.tasks_done(1)))
        try:
            comm.shutdown()
        except Exception:
            pass  # the shared error word is set: rank 0's own wait may report it too
        dist.barrier()
        comm.close()
        dist.destroy_process_group()
        result_q.put(("ok", errors))
    except Exception:
        result_q.put(("exc", f"rank {rank}: " + traceback.format_exc()))
        raise
