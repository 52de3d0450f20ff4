"""Probe: the c5 kernel pair (lsqb pass 1 + pass 2) on 8 workers at several total A sizes,
one label line per size on stderr; run under rocprofv3 --kernel-trace to read per-pass
times.  Small totals stay resident in the 256 MiB Infinity Cache across passes."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "mpistragglers.jl_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402
import mpiasyncpools as M  # noqa: E402

n, cols, K = 8, 2048, 64
torch.cuda.set_device(0)
for rows in [int(r) for r in (sys.argv[1:] or ["2048", "4096", "8192", "65536", "262144"])]:
    A = torch.empty(n * rows, cols, dtype=torch.bfloat16, device="cuda")
    B = torch.empty(n * rows, K, dtype=torch.bfloat16, device="cuda")
    M.generate(A, 3, 0, 0, float(np.float32(1 / np.sqrt(cols))))
    M.generate(B, 3, 1, 0, 1.0)
    comm = M.DeviceComm(n)
    for r in range(1, n + 1):
        comm.set_task_lsq_batch(r, A[(r - 1) * rows:r * rows], B[(r - 1) * rows:r * rows])
    pool = M.MPIAsyncPool(n)
    send = torch.zeros(cols * K, dtype=torch.bfloat16, device="cuda")
    isend = torch.zeros(n * cols * K, dtype=torch.bfloat16, device="cuda")
    recv = torch.zeros(n * cols * K, device="cuda")
    irecv = torch.zeros_like(recv)
    for _ in range(3):
        M.asyncmap_(pool, send, recv, isend, irecv, comm, nwait=n)
    torch.cuda.synchronize()
    comm.set_timing(True)
    t0 = time.perf_counter()
    for _ in range(10):
        M.asyncmap_(pool, send, recv, isend, irecv, comm, nwait=n)
    torch.cuda.synchronize()
    el = (time.perf_counter() - t0) / 10
    kl, kms, kb, busy = comm.timing()
    print("rows/worker %7d  A total %7.1f MiB  pair %.3f ms  %.0f GB/s (one-pass bytes)  epoch %.3f ms" %
          (rows, n * rows * cols * 2 / 2**20, kms / kl, kb / kl / (kms / kl / 1e3) / 1e9, el * 1e3), flush=True)
    comm.close()
    del A, B
    torch.cuda.empty_cache()
