"""Kernel tuning sweep for the BASELINE c2 shape (one process, interleaved rounds).

    python tools/lsq_tune.py [--rounds 2] [--epochs 20]

For every compiled lsq_grad_kernel variant (mpa_tune "lsq_variant") and workgroups-per-task
setting ("lsq_grid"), runs asyncmap! epochs of 8 fp32 workers over A 2^20 x 1024 and
reports the batched kernel's algorithmic GB/s from HIP events on its own stream, plus a
torch reduction over the same 4 GiB as an achievable-bandwidth reference.  Each variant's
gradient is checked against torch fp64 (rel 1e-5).  Prints one JSON line per measurement.
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "mpistragglers.jl_amd"))

import numpy as np  # noqa: E402
import torch  # noqa: E402

import mpiasyncpools as M  # noqa: E402
from mpiasyncpools._capi import lib  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=2)
    ap.add_argument("--epochs", type=int, default=20)
    ap.add_argument("--grids", default="32,48,64,96,128")
    ap.add_argument("--variants", default="2,4,5,6")
    ap.add_argument("--separate", action="store_true",
                    help="each worker's shard in its own allocation (as bench.py), copied from A")
    a = ap.parse_args()
    n, rows, cols = 8, 1 << 20, 1024
    per = rows // n
    A = torch.empty(rows, cols, device="cuda")
    b = torch.empty(rows, device="cuda")
    M.generate(A, 1234, 0, 0, float(np.float32(1 / np.sqrt(cols))))
    M.generate(b, 1234, 1, 0, 1.0)
    x = torch.empty(cols, device="cuda")
    M.generate(x, 1234, 2, 0, 0.5)
    A0 = A[:per].double()
    g0 = A0.t() @ (A0 @ x.double() - b[:per].double())
    del A0
    # achievable-bandwidth reference: torch reduction over the same 4 GiB
    s0, s1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    for _ in range(3):
        A.sum()
    s0.record()
    for _ in range(10):
        A.sum()
    s1.record()
    torch.cuda.synchronize()
    print(json.dumps({"ref": "torch.sum over A", "GBps": round(A.numel() * 4 * 10 / (s0.elapsed_time(s1) / 1e3) / 1e9, 1)}),
          flush=True)
    for _ in range(3):
        torch.mv(A, x)
    s0.record()
    for _ in range(10):
        torch.mv(A, x)
    s1.record()
    torch.cuda.synchronize()
    print(json.dumps({"ref": "torch.mv(A, x) (vendor GEMV, A read once)",
                      "GBps": round(A.numel() * 4 * 10 / (s0.elapsed_time(s1) / 1e3) / 1e9, 1)}), flush=True)
    nvar = 0
    while lib().mpa_tune(b"lsq_variant", nvar) == 0:
        nvar += 1
    variants = [int(v) for v in a.variants.split(",")] if a.variants else list(range(nvar))
    grids = [int(g) for g in a.grids.split(",")]
    if a.separate:
        shards = [A[(r - 1) * per:r * per].clone() for r in range(1, n + 1)]
        del A
        torch.cuda.empty_cache()
    else:
        shards = [A[(r - 1) * per:r * per] for r in range(1, n + 1)]
    isend = torch.zeros(n * cols, device="cuda")
    recv = torch.zeros(n * cols, device="cuda")
    irecv = torch.zeros_like(recv)
    for rnd in range(a.rounds):
        for v in variants:
            for g in grids:
                assert lib().mpa_tune(b"lsq_variant", v) == 0
                assert lib().mpa_tune(b"lsq_grid", g) == 0
                comm = M.DeviceComm(n)
                for r in range(1, n + 1):
                    comm.set_task_lsq(r, shards[r - 1], b[(r - 1) * per:r * per])
                pool = M.MPIAsyncPool(n)
                for _ in range(3):
                    M.asyncmap_(pool, x, recv, isend, irecv, comm, nwait=n)
                torch.cuda.synchronize()
                err = (torch.linalg.norm(recv[:cols].double() - g0) / torch.linalg.norm(g0)).item()
                comm.set_timing(True)
                t0 = time.perf_counter()
                for _ in range(a.epochs):
                    M.asyncmap_(pool, x, recv, isend, irecv, comm, nwait=n)
                torch.cuda.synchronize()
                el = time.perf_counter() - t0
                launches, ms, by, _ = comm.timing()
                comm.set_timing(False)
                print(json.dumps({"round": rnd, "variant": v,
                                  "grid": g, "kernel_GBps": round(by / (ms / 1e3) / 1e9, 1),
                                  "kernel_ms": round(ms / launches, 4), "epoch_ms": round(el / a.epochs * 1e3, 4),
                                  "rel_err": err}), flush=True)
                comm.close()


if __name__ == "__main__":
    main()
