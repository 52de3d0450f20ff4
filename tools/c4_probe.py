"""Probe: fp64 least-squares tasks at the c4 shape (2^20 x 2048 per worker), alone, batched,
and as concurrent single-task launches (delayed workers), one epoch each, timed."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "mpistragglers.jl_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402
import mpiasyncpools as M  # noqa: E402

dt = {"f64": torch.float64, "f32": torch.float32}[sys.argv[1] if len(sys.argv) > 1 else "f64"]
rows, cols, n = int(os.environ.get("ROWS", 1 << 20)), int(os.environ.get("COLS", 2048)), int(os.environ.get("N", 8))
torch.cuda.set_device(0)
A = torch.empty(rows, cols, dtype=dt, device="cuda")
b = torch.empty(rows, dtype=dt, device="cuda")
M.generate(A, 1, 0, 0, 1.0 / np.sqrt(cols))
M.generate(b, 1, 1, 0, 1.0)
torch.cuda.synchronize()
print("generated", flush=True)


def run(label, nw, delays):
    comm = M.DeviceComm(nw)
    for r in range(1, nw + 1):
        comm.set_task_lsq(r, A, b)
        if delays:
            comm.set_delays(r, np.full(16, delays, dtype=np.int64))
    pool = M.MPIAsyncPool(nw)
    x = torch.zeros(cols, dtype=dt, device="cuda")
    isend = torch.zeros(nw * cols, dtype=dt, device="cuda")
    recv = torch.zeros(nw * cols, dtype=dt, device="cuda")
    irecv = torch.zeros_like(recv)
    M.asyncmap_(pool, x, recv, isend, irecv, comm, nwait=nw)
    torch.cuda.synchronize()
    comm.set_timing(True)
    t0 = time.perf_counter()
    for _ in range(3):
        M.asyncmap_(pool, x, recv, isend, irecv, comm, nwait=nw)
    torch.cuda.synchronize()
    el = (time.perf_counter() - t0) / 3
    kl, kms, kb, _ = comm.timing()
    print("%-28s %8.3f ms/epoch  %d launches  %.3f ms/launch  %.1f GB/s/launch  %.1f GB/s epoch" %
          (label, el * 1e3, kl, kms / max(kl, 1), kb / max(kl, 1) / (kms / max(kl, 1)) / 1e6, kb / 3 / el / 1e9), flush=True)
    comm.shutdown()
    comm.close()


run("1 task", 1, 0)
run("%d tasks batched" % n, n, 0)
run("%d tasks delayed 1us" % n, n, 1000)
run("2 tasks delayed 1us", 2, 1000)
