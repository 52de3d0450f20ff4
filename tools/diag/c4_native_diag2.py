"""Diagnose native lsq_descent (epochs=1 per call) self-consistency on the c4 schedule."""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
for p in (ROOT, os.path.join(ROOT, "mpistragglers.jl_amd"), os.path.join(ROOT, "oracle"), os.path.join(ROOT, "tests")):
    sys.path.insert(0, p)
import numpy as np, torch
import mpiasyncpools as M
import test_gpu_configs as T
import lsq

sc = T.SCEN["gpu_sep_c4_first_plus_5"]
n, rows, cols, stale, eta = sc["n"], 512, 2048, 0.5, 0.2
A, b = T._problem(n, rows, cols, seed=44)
dur = np.asarray(sc["durations_ns"], dtype=np.int64).reshape(n, -1)
steps = [ref for op, ref in zip(sc["ops"], sc["results"]) if op["op"] == "asyncmap"]
for fuse in ("1", "0"):
    os.environ["MPA_FUSE"] = fuse
    comm = T._comm(M, torch, A, b, n, rows, dur)
    pool = M.MPIAsyncPool(n)
    x = torch.zeros(cols, dtype=torch.float64, device="cuda")
    isend = torch.zeros(n * cols, dtype=torch.float64, device="cuda"); recv = torch.zeros_like(isend); irecv = torch.zeros_like(isend)
    sent = {}
    xprev = np.zeros(cols)
    for k in range(len(steps)):
        sent[k + 1] = xprev.copy()
        M.lsq_descent(pool, comm, x, recv, isend, irecv, M.first_plus(5), eta, 1, stale_weight=stale)
        rep = pool.repochs.tolist()
        xk = x.cpu().numpy().copy()
        ch = recv.cpu().numpy().reshape(n, cols)
        errs = []
        w = np.zeros(n)
        for i in range(n):
            if steps[k]["repochs"][i] == 0:
                errs.append(None); continue
            g = lsq.shard_gradient(A[i * rows:(i + 1) * rows], b[i * rows:(i + 1) * rows], sent[rep[i]])
            errs.append("%.1e" % lsq.rel_err(ch[i], g))
            w[i] = 1.0 if rep[i] == k + 1 else stale
        w *= n / w.sum()
        xr = xprev - eta * (w[:, None] * ch).sum(0)
        print("fuse", fuse, k, rep == steps[k]["repochs"], rep, "chunk errs", errs, "update relerr %.1e" % lsq.rel_err(xk, xr),
              "isend slots == x:", [bool(np.array_equal(isend.cpu().numpy().reshape(n, cols)[i], sent[k + 1])) for i in range(n)])
        xprev = xk
    comm.shutdown()
