"""The PRODUCT pool over a real MPI communicator with GPU worker ranks (SURVEY.md §8f row 3
on the GPU box): tests/mpi/lsq_mpi_gpu.c runs examples/iterative_example.jl's program shape
(coordinator rank 0, worker ranks 1..n, data + control tags) as BASELINE configs[0] (3
workers, fp64, A 3*2^12 x 64, nwait 2, 10 epochs): the coordinator drives mpa_asyncmap /
mpa_waitall through libmpiasyncpools_mpi.so on host buffers, and every worker rank computes
its shard gradient on the GPU through libmpiasyncpools.so (a one-worker HIP communicator,
lsq_grad_kernel fp64), behind an injected host delay (the example's `sleep(rand())`, :71).

Checked against the oracle: every epoch has >= nwait fresh workers, and the final iterate
equals an fp64 numpy replay of x -= eta * sum(fresh g_i(x)) driven by the printed repochs,
with g_i from oracle/lsq.py (relative 1e-12, BASELINE's fp64 tolerance).  The delay schedule
makes worker 3 the straggler on odd tasks, so stale replies are exercised.  The driver is
prebuilt by __graft_entry__.build() (MPICH of this image, /opt/conda)."""
import os
import subprocess

import numpy as np
import pytest

from test_mpi_replay import MPI_DIR, MPIEXEC

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
DRIVER = os.path.join(ROOT, "mpistragglers.jl_amd", "_build", "lsq_mpi_gpu")

pytestmark = [pytest.mark.gpu,
              pytest.mark.skipif(not (os.path.exists(os.path.join(MPI_DIR, "include", "mpi.h")) and
                                      os.path.exists(MPIEXEC)), reason="MPICH not present")]


def test_iterative_example_over_mpi_with_gpu_workers(built):
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU visible")
    assert os.path.exists(DRIVER), "build() builds tests/mpi/lsq_mpi_gpu"
    import lsq
    n, rows, cols, epochs, nwait, seed = 3, 4096, 64, 10, 2, 7
    eta = 0.5 / (rows * n / (3 * cols) * (1 + np.sqrt(cols / (rows * n))) ** 2)
    delays = "1,2:3,4:30,2"  # ms per task, cycled: worker 3 straggles on its odd tasks
    env = dict(os.environ, HYDRA_LAUNCHER="fork")
    out = subprocess.run([MPIEXEC, "-n", str(n + 1), DRIVER, str(epochs), str(nwait), str(rows), str(cols),
                          str(seed), "%.17g" % eta, delays], capture_output=True, text=True, timeout=120, env=env)
    assert out.returncode == 0, (out.stdout[-2000:], out.stderr[-2000:])
    lines = out.stdout.splitlines()
    reps = [[int(v) for v in ln.split("|")[1].split()] for ln in lines if ln.startswith("E ")]
    xs = [ln for ln in lines if ln.startswith("X ")]
    assert len(reps) == epochs and len(xs) == 1
    x_dev = np.array([float(v) for v in xs[0].split()[1:]])
    shards = [(lsq.gen_matrix(seed, (w - 1) * rows, rows, cols, "f64"),
               lsq.gen_vector(seed, (w - 1) * rows, rows, "f64")) for w in range(1, n + 1)]
    x = np.zeros(cols)
    stale = 0
    for e, rep in enumerate(reps, start=1):
        fresh = [i for i in range(n) if rep[i] == e]
        assert len(fresh) >= nwait, (e, rep)
        stale += sum(1 for i in range(n) if 0 < rep[i] < e)
        s = np.zeros(cols)
        for i in fresh:
            s += lsq.shard_gradient(*shards[i], x, "f64")
        x = x - eta * s
    err = np.linalg.norm(x_dev - x) / np.linalg.norm(x)
    print("mpi + gpu workers: repochs %s; stale replies %d; final x rel err %.3e" % (reps, stale, err))
    assert stale > 0, "the schedule must leave a straggler behind"
    assert err <= 1e-12
