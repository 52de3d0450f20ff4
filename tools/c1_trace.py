"""c1's native loop under the task trace (mpa_comm_set_trace): where an epoch's 16 us go,
split on the host's clock into the device round trip of a task (its post -> its harvest) and
the host's turn (a harvest -> the next post).  Run on the GPU box:

    python tools/c1_trace.py [epochs]
"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "mpistragglers.jl_amd"))

import bench  # noqa: E402


def main():
    import torch
    import mpiasyncpools as M
    epochs = int(sys.argv[1]) if len(sys.argv) > 1 else 3000
    cfg = dict(bench.CONFIGS["c1"])
    cfg["config"] = "c1"
    n = cfg["workers"]
    comm = M.DeviceComm(n)
    shards = bench.gen_shards(M, torch, cfg, 1234, range(1, n + 1))
    for w, (A, b) in enumerate(shards, start=1):
        bench.register(comm, cfg, 1234, w, A, b)
    pool = M.MPIAsyncPool(n)
    loop, x = bench.make_loop(M, torch, cfg, pool, comm)
    loop(300)
    torch.cuda.synchronize()
    cap = 4 * epochs
    comm.set_trace(cap)
    import time
    t0 = time.perf_counter()
    loop(epochs)
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    tr = comm.trace(cap)
    F = {k: j for j, k in enumerate(M.DeviceComm.TRACE_FIELDS)}
    post, harv = tr[:, F["post"]], tr[:, F["harvest"]]
    ok = (post > 0) & (harv > 0)
    rt = (harv[ok] - post[ok]) / 1e3
    # the host's turn: every post against the latest harvest before it
    hs = np.sort(harv[harv > 0])
    ps = np.sort(post[post > 0])
    idx = np.searchsorted(hs, ps) - 1
    turn = (ps[idx >= 0] - hs[idx[idx >= 0]]) / 1e3
    pct = lambda a: "p10 %.2f p50 %.2f p90 %.2f us" % tuple(np.percentile(a, [10, 50, 90]))
    print("c1 native loop, %d epochs: %.1f us per epoch (%.0f it/s), %d tasks traced" % (
        epochs, el / epochs * 1e6, epochs / el, int(ok.sum())))
    print("  task round trip (post -> harvest, host clock):", pct(rt))
    print("  host turn (harvest -> next post):", pct(turn))
    out = os.environ.get("C1_TRACE_OUT")
    if out:  # the raw trace (host CLOCK_MONOTONIC ns), to align with a kernel trace of the same run
        np.save(out, tr)
    for k in ("head_steps", "epoch_kernels", "prearmed", "prearm_same"):
        print("  %s %d" % (k, comm.counter(k)))
    comm.close()


if __name__ == "__main__":
    main()
