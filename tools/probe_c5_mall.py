"""Probe: c5-shaped batched tasks (8 workers, cols 2048, 64 iterates, bf16) at a reduced
row count per worker, nwait = 8, run back to back by the native loop.  At 16-32 MiB per
worker the whole batch stays in the 256 MiB Infinity Cache between launches, so the
per-launch pass-1 / pass-2 durations (rocprofv3 --kernel-trace --stats) give the rates a
row-chunked schedule (pass 2 right behind pass 1 on the same rows) could reach.

usage: python tools/probe_c5_mall.py ROWS_PER_WORKER [STEPS]
"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "mpistragglers.jl_amd"))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

import mpiasyncpools as M  # noqa: E402
import bench  # noqa: E402


def main():
    per = int(sys.argv[1])
    steps = int(sys.argv[2]) if len(sys.argv) > 2 else 50
    n = 8
    cfg = dict(bench.CONFIGS["c5"])
    cfg.update(rows=per * n, nwait=8, config="c5probe")
    torch.cuda.set_device(0)
    comm = M.DeviceComm(n)
    shards = bench.gen_shards(M, torch, cfg, 7, range(1, n + 1))
    for w, (A, b) in enumerate(shards, start=1):
        comm.set_task_lsq_batch(w, A, b)
    pool = M.MPIAsyncPool(n)
    loop, x = bench.make_loop(M, torch, cfg, pool, comm)
    loop(3)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    loop(steps)
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    abytes = 2.0 * per * n * 2048
    print("rows/worker %d  batch A %.1f MiB  %.3f ms/epoch  %.2f TB/s one-pass"
          % (per, abytes / 2**20, el / steps * 1e3, abytes / (el / steps) / 1e12), flush=True)
    _, recv, _, irecv = loop.bufs
    M.waitall_(pool, recv, irecv)
    comm.shutdown()
    comm.close()


if __name__ == "__main__":
    main()
