"""Latencies per worker per epoch, native epochs=1 calls, fuse 1 vs 0 (c4 schedule)."""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
for p in (ROOT, os.path.join(ROOT, "mpistragglers.jl_amd"), os.path.join(ROOT, "oracle"), os.path.join(ROOT, "tests")):
    sys.path.insert(0, p)
import numpy as np, torch, time
import mpiasyncpools as M
import test_gpu_configs as T
sc = T.SCEN["gpu_sep_c4_first_plus_5"]
n, rows, cols, stale, eta = sc["n"], 512, 2048, 0.5, 0.2
A, b = T._problem(n, rows, cols, seed=44)
dur = np.asarray(sc["durations_ns"], dtype=np.int64).reshape(n, -1)
for fuse in ("1", "0", "1"):
    os.environ["MPA_FUSE"] = fuse
    comm = T._comm(M, torch, A, b, n, rows, dur)
    pool = M.MPIAsyncPool(n)
    x = torch.zeros(cols, dtype=torch.float64, device="cuda")
    isend = torch.zeros(n * cols, dtype=torch.float64, device="cuda"); recv = torch.zeros_like(isend); irecv = torch.zeros_like(isend)
    t0 = time.perf_counter()
    for k in range(3):
        M.lsq_descent(pool, comm, x, recv, isend, irecv, M.first_plus(5), eta, 1, stale_weight=stale)
        print("fuse", fuse, "epoch", k + 1, "t %.1f ms" % ((time.perf_counter() - t0) * 1e3), pool.repochs.tolist(),
              "sep", pool.sepochs.tolist(), "lat ms", [round(v * 1e3, 1) for v in pool.latency],
              "tasks", [comm.tasks_done(r) for r in range(1, n + 1)], flush=True)
    comm.shutdown()
