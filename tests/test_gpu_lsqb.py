"""GPU parity of the batched 64-iterate variant (BASELINE configs[4], "c5"):
G_i = A_i^T (A_i X - B_i), bf16 A/B/X, fp32 accumulate (lsqb_kernel.hip), through the
C ABI (mpa_comm_set_task_lsq_batch + mpa_asyncmap), against the fp64 oracle
(oracle/lsq.py batched_shard_gradient) on the same bf16-rounded inputs.

Tolerance: normwise relative 1e-5, set from evidence.  Every kernel carries the residual
as bf16 hi + lo (~2^-17 relative per element) and accumulates in fp32 over up to 2^20 rows;
over every case of this file and every kernel the worst measured error is 2.42e-6
(profiles/r02_c5_tolerance.txt: the default lsqp4, the eight-wave lsqp, the two passes,
lsqf), so 1e-5 is about 4x the worst case and equals BASELINE's fp32 tolerance.
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu
K = 64
TOL = 1e-5


@pytest.fixture(scope="module")
def M(built):
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU visible")
    import mpiasyncpools
    return mpiasyncpools


def _bf16(torch, bits):
    return torch.from_numpy(np.ascontiguousarray(bits).view(np.int16)).cuda().view(torch.bfloat16)


def _problem(rows, cols, seed):
    import lsq
    A = lsq.gen_matrix(seed, 0, rows, cols, "bf16")
    B = lsq.gen_matrix(seed, 0, rows, K, "bf16", stream=lsq.STREAM_B, scale=np.float32(1.0))
    X = lsq.gen_matrix(seed, 0, cols, K, "bf16", stream=lsq.STREAM_X, scale=np.float32(0.5))
    return A, B, X


class _Bufs:
    """sendbuf / recvbuf / isendbuf / irecvbuf, allocated once: the reference requires the
    same isendbuf / irecvbuf on every call (in-flight requests point at them,
    src/MPIAsyncPools.jl:63-66)."""

    def __init__(self, torch, n, cols):
        self.send = torch.zeros(cols * K, dtype=torch.bfloat16, device="cuda")
        self.isend = torch.zeros(n * cols * K, dtype=torch.bfloat16, device="cuda")
        self.recv = torch.zeros(n * cols * K, dtype=torch.float32, device="cuda")
        self.irecv = torch.zeros_like(self.recv)


def _run(M, torch, shards, cols, X, nwait=None, comm=None, pool=None, delays=None, bufs=None):
    n = len(shards)
    if comm is None:
        comm = M.DeviceComm(n)
        for r, (A, B) in enumerate(shards, start=1):
            comm.set_task_lsq_batch(r, _bf16(torch, A), _bf16(torch, B))
            if delays is not None:
                comm.set_delays(r, delays[r - 1])
        pool = M.MPIAsyncPool(n)
    if bufs is None:
        bufs = comm._bufs = _Bufs(torch, n, cols)
    bufs.send.copy_(_bf16(torch, X).view(-1))
    rep = M.asyncmap_(pool, bufs.send, bufs.recv, bufs.isend, bufs.irecv, comm, nwait=n if nwait is None else nwait)
    return bufs.recv.cpu().numpy().reshape(n, cols, K), rep, comm, pool


@pytest.mark.parametrize("rows,cols", [(1, 32), (100, 64), (1000, 256), (4113, 544), (3000, 2048), (257, 4096),
                                       (20000, 1024)])
def test_lsqb_vs_oracle(M, rows, cols):
    import lsq
    import torch
    A, B, X = _problem(rows, cols, seed=rows + cols)
    out, rep, comm, _ = _run(M, torch, [(A, B)], cols, X)
    assert list(rep) == [1]
    ref = lsq.batched_shard_gradient(A, B, X, "bf16")
    err = lsq.rel_err(out[0], ref)
    print(f"lsqb rows={rows} cols={cols} rel err {err:.3e}")
    assert err <= TOL, err
    comm.close()


def test_lsqb_batched_launch_counters_and_determinism(M):
    """3 workers (different shards, ragged rows) in one batched launch pair, 4 epochs:
    counters advance per launch, results bitwise identical for the same X."""
    import lsq
    import torch
    cols = 512
    shards, refs = [], []
    A, B, X = _problem(3 * 1500, cols, seed=7)
    for i, rr in enumerate((1500, 1400, 1100)):
        Ai, Bi = A[i * 1500:i * 1500 + rr], B[i * 1500:i * 1500 + rr]
        shards.append((Ai, Bi))
        refs.append(lsq.batched_shard_gradient(Ai, Bi, X, "bf16"))
    out, rep, comm, pool = _run(M, torch, shards, cols, X)
    for i in range(3):
        assert lsq.rel_err(out[i], refs[i]) <= TOL, i
    for _ in range(3):
        again, rep, _, _ = _run(M, torch, shards, cols, X, comm=comm, pool=pool, bufs=comm._bufs)
        assert np.array_equal(again.view(np.uint32), out.view(np.uint32))
    comm.close()


def test_lsqb_stragglers_chunks_match_their_epochs(M):
    """Delayed workers run the single-task path; every chunk equals G of the X of epoch
    repochs[i] (test/kmap2.jl:50's integrity invariant, numerically)."""
    import lsq
    import torch
    n, rows, cols = 3, 700, 256
    A, B, _ = _problem(n * rows, cols, seed=9)
    shards = [(A[i * rows:(i + 1) * rows], B[i * rows:(i + 1) * rows]) for i in range(n)]
    rng = np.random.default_rng(1)
    delays = [rng.integers(0, 5, size=8) * 2_000_000 for _ in range(n)]
    comm = pool = None
    sent = {}
    for epoch in range(1, 9):
        X = lsq.gen_matrix(100 + epoch, 0, cols, K, "bf16", stream=lsq.STREAM_X, scale=np.float32(0.5))
        sent[epoch] = X
        out, rep, comm, pool = _run(M, torch, shards, cols, X, nwait=1, comm=comm, pool=pool,
                                    delays=delays if comm is None else None,
                                    bufs=None if comm is None else comm._bufs)
        assert (rep == epoch).sum() >= 1
        for i in range(n):
            if rep[i] == 0:
                continue
            ref = lsq.batched_shard_gradient(shards[i][0], shards[i][1], sent[int(rep[i])], "bf16")
            assert lsq.rel_err(out[i], ref) <= TOL, (epoch, i)
    comm.shutdown()
    comm.close()


def test_lsqb_full_c5_shard_against_torch_fp64(M):
    """One full c5 shard (A_i 2^20 x 2048 bf16, generated on the device) against torch
    fp64 on the same device data, and a second worker in the same launch."""
    import torch
    rows, cols, seed, n = 1 << 20, 2048, 55, 2
    A = torch.empty(n * rows, cols, dtype=torch.bfloat16, device="cuda")
    B = torch.empty(n * rows, K, dtype=torch.bfloat16, device="cuda")
    X = torch.empty(cols, K, dtype=torch.bfloat16, device="cuda")
    M.generate(A, seed, 0, 0, float(np.float32(1 / np.sqrt(cols))))
    M.generate(B, seed, 1, 0, 1.0)
    M.generate(X, seed, 2, 0, 0.5)
    comm = M.DeviceComm(n)
    for r in range(1, n + 1):
        comm.set_task_lsq_batch(r, A[(r - 1) * rows:r * rows], B[(r - 1) * rows:r * rows])
    pool = M.MPIAsyncPool(n)
    isend = torch.zeros(n * cols * K, dtype=torch.bfloat16, device="cuda")
    recv = torch.zeros(n * cols * K, dtype=torch.float32, device="cuda")
    irecv = torch.zeros_like(recv)
    M.asyncmap_(pool, X, recv, isend, irecv, comm, nwait=n)
    got = recv.view(n, cols, K).double()
    X64 = X.double()
    for i in range(n):
        Ai = A[i * rows:(i + 1) * rows].double()
        G = Ai.t() @ (Ai @ X64 - B[i * rows:(i + 1) * rows].double())
        err = (torch.linalg.norm(got[i] - G) / torch.linalg.norm(G)).item()
        print(f"c5 shard {i}: rel err {err:.3e}")
        assert err <= TOL, (i, err)
        del Ai, G
    comm.close()


@pytest.mark.parametrize("env", [{}, {"MPA_AHEAD": "0"}, {"MPA_FUSE": "0"}])
def test_lsqb_descent_native_loop_matches_python_loop(M, monkeypatch, env):
    """mpa_lsqb_descent (fused epoch kernel: harvests, fp32 update, bf16 mirror, dispatch
    of the mirror; launch-ahead at nwait = n) against the Python loop (asyncmap_ +
    lsqb_update): identical fp32 iterates, bf16 messages and replies, bitwise."""
    import torch
    for k, v in env.items():
        monkeypatch.setenv(k, v)
    n, rows, cols, epochs, eta = 3, 600, 256, 5, 0.01
    A, B, _ = _problem(n * rows, cols, seed=13)
    outs = []
    for native in (False, True):
        comm = M.DeviceComm(n)
        for r in range(1, n + 1):
            comm.set_task_lsq_batch(r, _bf16(torch, A[(r - 1) * rows:r * rows]), _bf16(torch, B[(r - 1) * rows:r * rows]))
        pool = M.MPIAsyncPool(n)
        bufs = _Bufs(torch, n, cols)
        x32 = torch.zeros(cols * K, device="cuda")
        if native:
            M.lsqb_descent(pool, comm, x32, bufs.send, bufs.recv, bufs.isend, bufs.irecv, n, eta, epochs)
        else:
            for _ in range(epochs):
                rep = M.asyncmap_(pool, bufs.send, bufs.recv, bufs.isend, bufs.irecv, comm, nwait=n)
                comm.lsqb_update(x32, bufs.send, bufs.recv, n, (rep == pool.epoch) * 1.0, eta)
        torch.cuda.synchronize()
        assert pool.epoch == epochs and list(pool.repochs) == [epochs] * n
        outs.append((x32.clone(), bufs.send.clone().view(torch.int16), bufs.recv.clone(), bufs.isend.clone().view(torch.int16)))
        comm.close()
    for a, b in zip(outs[0], outs[1]):
        assert torch.equal(a.view(torch.int16) if a.dtype != torch.int16 else a, b.view(torch.int16) if b.dtype != torch.int16 else b)
    assert float(torch.linalg.norm(outs[0][0])) > 0


@pytest.mark.parametrize("env", [{}, {"MPA_LSQP": "c"}, {"MPA_LSQP": "8"}, {"MPA_LSQP": "0"}, {"MPA_LSQF": "1"},
                                 {"MPA_LSQF": "1", "MPA_LSQF_DBG": "7"}, {"MPA_LSQQ": "1"}],
                         ids=["lsqp4_pairs_default", "lsqc_column_pairs", "lsqp_eight_waves", "two_pass",
                              "lsqf_xcd_local_groups", "lsqf_cross_xcd_groups", "lsqq_quads"])
@pytest.mark.parametrize("rows,cols,n", [(1, 32, 1), (4113, 544, 1), (3000, 2048, 3), (20000, 1024, 2),
                                         (2500, 1312, 2)])
def test_single_pass_vs_oracle(M, monkeypatch, env, rows, cols, n):
    """Every c5 kernel against the oracle: the default single pass by iterate halves
    (lsqp4_kernel.hip: pairs of workgroups of one wave per SIMD, no exchange), column pairs
    (lsqc_kernel.hip, MPA_LSQP=c: members split the columns and exchange per-block partial
    products as tagged granules; one workgroup per row group at <= 1024 columns), the same
    scheme cut into eight waves (lsqp_kernel.hip, MPA_LSQP=8), the two passes (MPA_LSQP=0), and
    the opt-in single pass lsqf_kernel.hip (MPA_LSQF=1),
    groups of P = ceil(cols / 512) workgroups exchanging partial residuals inside an XCD
    (plain stores through the shared L2) or, with MPA_LSQF_DBG=7, every group treated as
    spread over XCDs (write-through stores); and lsqq_kernel.hip (MPA_LSQQ=1), quads of
    workgroups owning 16 iterates each.  Ragged rows and several tasks per launch;
    repeated launches are bitwise identical (fixed summation orders)."""
    import lsq
    import torch
    if env not in ({}, {"MPA_LSQP": "0"}) and b"measurement build" not in M.lib().mpa_build_info():
        pytest.skip("a c5 variant of the measurement build (make MEASURE=1, MPA_LIB=...): not in the product")
    for k, v in env.items():
        monkeypatch.setenv(k, v)
    A, B, X = _problem(n * rows, cols, seed=rows + cols + n)
    shards = [(A[i * rows:(i + 1) * rows - (i * 7 % max(rows, 1) if rows > 7 else 0)],
               B[i * rows:(i + 1) * rows - (i * 7 % max(rows, 1) if rows > 7 else 0)]) for i in range(n)]
    out, rep, comm, pool = _run(M, torch, shards, cols, X)
    assert list(rep) == [1] * n
    for i, (Ai, Bi) in enumerate(shards):
        err = lsq.rel_err(out[i], lsq.batched_shard_gradient(Ai, Bi, X, "bf16"))
        print(f"lsqf rows={Ai.shape[0]} cols={cols} worker {i + 1} rel err {err:.3e}")
        assert err <= TOL, (i, err)
    again, _, _, _ = _run(M, torch, shards, cols, X, comm=comm, pool=pool, bufs=comm._bufs)
    assert np.array_equal(again.view(np.uint32), out.view(np.uint32))
    comm.close()


def test_lsqp4_full_form_matches_general_form_bitwise(M):
    """lsqp4_kernel's FULL form (every task of the batch has cols = 2048 and rows % 16 = 0:
    immediate-offset strip DMAs, no clamps or masks, -B folded into one MFMA per tile) against
    the oracle and bit for bit against the general form: the same two 4800-row shards run once
    in a batch of their own (FULL) and once beside a third, ragged shard (general form); the
    row groups per task are equal in both batches, so the G trees sum in the same order."""
    import lsq
    import torch
    rows, cols = 4800, 2048
    A, B, X = _problem(3 * rows, cols, seed=77)
    full = [(A[i * rows:(i + 1) * rows], B[i * rows:(i + 1) * rows]) for i in range(2)]
    # a third shard makes the batch general: 4799 rows (ragged); 3 tasks in both batches
    shards_f = full + [(A[2 * rows:3 * rows], B[2 * rows:3 * rows])]
    shards_g = full + [(A[2 * rows:3 * rows - 1], B[2 * rows:3 * rows - 1])]
    out_f, rep, comm, _ = _run(M, torch, shards_f, cols, X)
    comm.close()
    out_g, rep, comm, _ = _run(M, torch, shards_g, cols, X)
    comm.close()
    for i in range(2):
        err = lsq.rel_err(out_f[i], lsq.batched_shard_gradient(full[i][0], full[i][1], X, "bf16"))
        print(f"lsqp4 FULL worker {i + 1} rel err {err:.3e}")
        assert err <= TOL, (i, err)
        assert np.array_equal(out_f[i].view(np.uint32), out_g[i].view(np.uint32)), i
    err = lsq.rel_err(out_g[2], lsq.batched_shard_gradient(shards_g[2][0], shards_g[2][1], X, "bf16"))
    assert err <= TOL, err


_VARIANT_CHILD = r"""
import os, sys
import numpy as np
sys.path[:0] = [os.path.join(sys.argv[1], p) for p in ("tests", "mpistragglers.jl_amd", "oracle")]
import torch
import mpiasyncpools as M
import test_gpu_lsqb as T
outs = []
for rows, cols, n, seed in T._VARIANT_CASES:
    A, B, X = T._problem(n * rows, cols, seed)
    shards = [(A[i * rows:(i + 1) * rows - (i if rows % 16 else 0)], B[i * rows:(i + 1) * rows - (i if rows % 16 else 0)])
              for i in range(n)]
    out, rep, comm, _ = T._run(M, torch, shards, cols, X)
    comm.close()
    outs.append(out)
np.savez(sys.argv[2], *outs)
"""
# lone tasks (the second launch's case) of 128, 128, 63 and 17 row groups (trees of 4, 3 and 3 levels,
# short last groups at several levels), ragged rows, 1312 and 512 columns (waves with part of a slice
# or none); and a batch of two tasks, which keeps the in-kernel tree either way
_VARIANT_CASES = [(4800, 2048, 1, 95), (3001, 1312, 1, 96), (1000, 2048, 1, 97), (272, 512, 1, 98),
                  (2500, 2048, 2, 99)]


def _variant_outputs(tmp_path, tag, env_extra):
    import os
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    out = str(tmp_path / f"{tag}.npz")
    env = dict(os.environ, **env_extra)
    r = subprocess.run([sys.executable, "-c", _VARIANT_CHILD, root, out], env=env, capture_output=True, text=True,
                       timeout=240)
    assert r.returncode == 0, r.stderr[-3000:]
    z = np.load(out)
    return [z[f"arr_{k}"] for k in range(len(_VARIANT_CASES))]


def test_lsqp4_second_launch_reduce_matches_tree_bitwise(M, tmp_path):
    """A lone task's G over the row groups in a second launch (lsqp4_reduce_kernel, the default)
    against the in-kernel tree (MPA_LSQP4_XRED=0), each in a process of its own: bit for bit on
    every case -- the reduction keeps the tree's summation order -- and every G within 1e-5 of the
    fp64 oracle."""
    import lsq
    new = _variant_outputs(tmp_path, "xred", {"MPA_LSQP4_XRED": "1"})
    old = _variant_outputs(tmp_path, "tree", {"MPA_LSQP4_XRED": "0"})
    for (rows, cols, n, seed), a, b in zip(_VARIANT_CASES, new, old):
        assert np.array_equal(a.view(np.uint32), b.view(np.uint32)), (rows, cols, n)
        A, B, X = _problem(n * rows, cols, seed)
        for i in range(n):
            lo, hi = i * rows, (i + 1) * rows - (i if rows % 16 else 0)
            err = lsq.rel_err(a[i], lsq.batched_shard_gradient(A[lo:hi], B[lo:hi], X, "bf16"))
            assert err <= TOL, (rows, cols, n, i, err)
