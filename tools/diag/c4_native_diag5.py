import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
for p in (ROOT, os.path.join(ROOT, "mpistragglers.jl_amd"), os.path.join(ROOT, "oracle"), os.path.join(ROOT, "tests")):
    sys.path.insert(0, p)
import numpy as np, torch
import mpiasyncpools as M
import test_gpu_configs as T
sc = T.SCEN["gpu_sep_c4_first_plus_5"]
n, rows, cols, stale, eta = sc["n"], 512, 2048, 0.5, 0.2
A, b = T._problem(n, rows, cols, seed=44)
for ref in sc["results"][:4]:
    print("oracle", ref["repochs"], "lat", [v / 1e6 for v in ref["latency_ns"]], flush=True)
for fuse in ("1", "0"):
    os.environ["MPA_FUSE"] = fuse
    os.environ["MPA_DESCENT_TRACE"] = "1"
    comm, pool, x = T._native(M, torch, sc, A, b, rows, cols, M.first_plus(5), eta, stale, 0)
    os.environ["MPA_DESCENT_TRACE"] = "0"
    print("fuse", fuse, "final", pool.repochs.tolist(), flush=True)
    comm.shutdown()
