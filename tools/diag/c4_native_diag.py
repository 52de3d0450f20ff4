"""Diagnose: native lsq_descent vs the Python loop on the c4 golden schedule (fp64)."""
import os, sys, json
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
for p in (ROOT, os.path.join(ROOT, "mpistragglers.jl_amd"), os.path.join(ROOT, "oracle"), os.path.join(ROOT, "tests")):
    sys.path.insert(0, p)
import numpy as np, torch
import mpiasyncpools as M
import test_gpu_configs as T

sc = T.SCEN["gpu_sep_c4_first_plus_5"]
n, rows, cols, stale, eta = sc["n"], 512, 2048, 0.5, 0.2
A, b = T._problem(n, rows, cols, seed=44)
dur = np.asarray(sc["durations_ns"], dtype=np.int64).reshape(n, -1)
steps = [ref for op, ref in zip(sc["ops"], sc["results"]) if op["op"] == "asyncmap"]

def python_loop():
    comm = T._comm(M, torch, A, b, n, rows, dur)
    pool = M.MPIAsyncPool(n)
    x = torch.zeros(cols, dtype=torch.float64, device="cuda")
    isend = torch.zeros(n * cols, dtype=torch.float64, device="cuda"); recv = torch.zeros_like(isend); irecv = torch.zeros_like(isend)
    xs, reps = [], []
    for k in range(len(steps)):
        rep = M.asyncmap_(pool, x, recv, isend, irecv, comm, nwait=M.first_plus(5))
        w = np.array([1.0 if rep[i] == pool.epoch else (stale if steps[k]["repochs"][i] else 0.0) for i in range(n)])
        w *= n / w.sum()
        comm.lsq_update(x, recv, n, w, eta)
        xs.append(x.cpu().numpy().copy()); reps.append(rep.tolist())
    comm.shutdown()
    return xs, reps

def native(mode):
    if mode == "nofuse": os.environ["MPA_FUSE"] = "0"
    else: os.environ.pop("MPA_FUSE", None)
    comm = T._comm(M, torch, A, b, n, rows, dur)
    pool = M.MPIAsyncPool(n)
    x = torch.zeros(cols, dtype=torch.float64, device="cuda")
    isend = torch.zeros(n * cols, dtype=torch.float64, device="cuda"); recv = torch.zeros_like(isend); irecv = torch.zeros_like(isend)
    xs, reps = [], []
    if mode == "single":
        for k in range(len(steps)):
            M.lsq_descent(pool, comm, x, recv, isend, irecv, M.first_plus(5), eta, 1, stale_weight=stale)
            xs.append(x.cpu().numpy().copy()); reps.append(pool.repochs.tolist())
    else:
        M.lsq_descent(pool, comm, x, recv, isend, irecv, M.first_plus(5), eta, len(steps), stale_weight=stale)
        xs.append(x.cpu().numpy().copy()); reps.append(pool.repochs.tolist())
    comm.shutdown()
    os.environ.pop("MPA_FUSE", None)
    return xs, reps

px, pr = python_loop()
print("oracle reps ok:", all(pr[k] == steps[k]["repochs"] for k in range(len(steps))))
for mode in ("single", "nofuse", "fused"):
    nx, nr = native(mode)
    if mode == "single":
        for k in range(len(steps)):
            print(mode, k, nr[k] == steps[k]["repochs"], nr[k], steps[k]["repochs"], "x eq", np.array_equal(nx[k], px[k]),
                  "relerr %.2e" % (np.linalg.norm(nx[k] - px[k]) / np.linalg.norm(px[k])))
    else:
        print(mode, nr[-1], "x eq", np.array_equal(nx[-1], px[-1]), "relerr %.2e" % (np.linalg.norm(nx[-1] - px[-1]) / np.linalg.norm(px[-1])))
