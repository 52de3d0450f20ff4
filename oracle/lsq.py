"""ORACLE — TEST INFRASTRUCTURE ONLY.

numpy restatement of (1) the build's synthetic least-squares data layout (Philox4x32-10,
see philox.h) and (2) the worker compute the BASELINE workload puts in the reference's
compute slot (examples/iterative_example.jl:74, `sleep(rand())` there):
    g_i = A_i^T (A_i x - b_i)
in float64 on the exact (rounded) inputs.  The reference has no numeric workload, so
gradient parity is pinned by these restatements only ("parity unpinned" w.r.t. the
reference itself; tolerance from BASELINE.json north_star: 1e-5 fp32, 1e-12 fp64).
Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg import this.
"""
import numpy as np

M0, M1 = np.uint64(0xD2511F53), np.uint64(0xCD9E8D57)
W0, W1 = np.uint32(0x9E3779B9), np.uint32(0xBB67AE85)
MASK32 = np.uint64(0xFFFFFFFF)

STREAM_A, STREAM_B, STREAM_X = 0, 1, 2


def philox4x32_10(c0, c1, c2, c3, k0, k1):
    """Vectorised Philox4x32-10 over uint32 arrays (Salmon et al. SC'11)."""
    c0, c1, c2, c3 = (np.asarray(v, dtype=np.uint32) for v in (c0, c1, c2, c3))
    k0 = np.uint32(k0)
    k1 = np.uint32(k1)
    with np.errstate(over="ignore"):
        for r in range(10):
            if r > 0:
                k0 = np.uint32(k0 + W0)
                k1 = np.uint32(k1 + W1)
            p0 = M0 * c0.astype(np.uint64)
            p1 = M1 * c2.astype(np.uint64)
            hi0 = (p0 >> np.uint64(32)).astype(np.uint32)
            lo0 = (p0 & MASK32).astype(np.uint32)
            hi1 = (p1 >> np.uint64(32)).astype(np.uint32)
            lo1 = (p1 & MASK32).astype(np.uint32)
            c0, c1, c2, c3 = hi1 ^ c1 ^ k0, lo1, hi0 ^ c3 ^ k1, lo0
    return c0, c1, c2, c3


def philox_words(seed, stream, e):
    """32-bit word for linear element indices e (uint64 array) of a stream."""
    e = np.asarray(e, dtype=np.uint64)
    q = e >> np.uint64(2)
    lo = (q & MASK32).astype(np.uint32)
    hi = (q >> np.uint64(32)).astype(np.uint32)
    s = np.full(e.shape, stream, dtype=np.uint32)
    z = np.zeros(e.shape, dtype=np.uint32)
    o = philox4x32_10(lo, hi, s, z, seed & 0xFFFFFFFF, (seed >> 32) & 0xFFFFFFFF)
    j = (e & np.uint64(3)).astype(np.int64)
    return np.choose(j, o)


def unit_f32(w):
    """uniform on [-1, 1), 2^-23 grid (exact in fp32/fp64)."""
    return ((w >> np.uint32(8)).astype(np.int32) - 8388608).astype(np.float32) * np.float32(1.0 / 8388608.0)


def f32_to_bf16_bits(a):
    """round-to-nearest-even fp32 -> bf16 bit pattern (uint16); inputs here are finite."""
    u = np.asarray(a, dtype=np.float32).view(np.uint32).astype(np.uint64)
    r = (u + np.uint64(0x7FFF) + ((u >> np.uint64(16)) & np.uint64(1))) >> np.uint64(16)
    return r.astype(np.uint16)


def bf16_bits_to_f32(h):
    return (np.asarray(h, dtype=np.uint16).astype(np.uint32) << np.uint32(16)).view(np.float32)


def scale_for(cols, dtype):
    s = 1.0 / np.sqrt(float(cols))
    return np.float64(s) if dtype == "f64" else np.float32(s)


def gen_matrix(seed, row0, rows, cols, dtype="f32", stream=STREAM_A, scale=None):
    """Rows [row0, row0+rows) of the global synthetic A (row-major, element e = r*cols+c).

    dtype "f32" -> float32, "f64" -> float64, "bf16" -> uint16 bf16 bit patterns."""
    if scale is None:
        scale = scale_for(cols, dtype)
    e = (np.arange(row0, row0 + rows, dtype=np.uint64)[:, None] * np.uint64(cols)
         + np.arange(cols, dtype=np.uint64)[None, :])
    u = unit_f32(philox_words(seed, stream, e))
    if dtype == "f64":
        return u.astype(np.float64) * np.float64(scale)
    v = u * np.float32(scale)
    if dtype == "bf16":
        return f32_to_bf16_bits(v)
    return v


def gen_vector(seed, i0, n, dtype="f32", stream=STREAM_B, scale=1.0):
    e = np.arange(i0, i0 + n, dtype=np.uint64)
    u = unit_f32(philox_words(seed, stream, e))
    if dtype == "f64":
        return u.astype(np.float64) * np.float64(scale)
    v = u * np.float32(scale)
    if dtype == "bf16":
        return f32_to_bf16_bits(v)
    return v


def as_f64(a, dtype):
    if dtype == "bf16":
        return bf16_bits_to_f32(a).astype(np.float64)
    return np.asarray(a, dtype=np.float64)


def shard_gradient(A, b, x, dtype="f32"):
    """g = A^T (A x - b) in float64 on the rounded inputs (the worker compute)."""
    A64 = as_f64(A, dtype)
    r = A64 @ as_f64(x, dtype) - as_f64(b, dtype)
    return A64.T @ r


def batched_shard_gradient(A, B, X, dtype="bf16"):
    """G = A^T (A X - B) for the 64-iterate variant; X is cols x k, B is rows x k."""
    A64 = as_f64(A, dtype)
    R = A64 @ as_f64(X, dtype) - as_f64(B, dtype)
    return A64.T @ R


def rel_err(got, ref):
    ref = np.asarray(ref, dtype=np.float64)
    den = np.linalg.norm(ref)
    return float(np.linalg.norm(np.asarray(got, dtype=np.float64) - ref) / (den if den > 0 else 1.0))
