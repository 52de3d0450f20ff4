"""Host-side mirror of the MPIAsyncPools.jl API over the C ABI.

    pool = MPIAsyncPool(n)                       # src/MPIAsyncPools.jl:46
    pool = MPIAsyncPool([1, 4, 5], epoch0=0, nwait=2)   # :35
    repochs = asyncmap_(pool, sendbuf, recvbuf, isendbuf, irecvbuf, comm,
                        nwait=..., epoch=..., tag=0)    # Base.asyncmap!, :68
    repochs = waitall_(pool, recvbuf, irecvbuf)          # waitall!, :195

`!` is not a Python identifier character, so the bang functions are `asyncmap_` /
`waitall_`.  Pool fields (`ranks, sepochs, repochs, active, stimestamps, latency`) are
numpy views of the library's state: `repochs` returned by `asyncmap_` is the same aliased
vector the reference returns (`return pool.repochs`, :187).

Errors are the reference's: ArgumentError, DimensionMismatch, ErrorException, with the
reference's message text.
"""
import ctypes as C

import numpy as np

from . import _capi
from ._capi import lib


class ArgumentError(ValueError):
    """Julia ArgumentError (src/MPIAsyncPools.jl:71,73,74,197)."""


class DimensionMismatch(ValueError):
    """Julia DimensionMismatch (src/MPIAsyncPools.jl:75-77,198,199)."""


class ErrorException(RuntimeError):
    """Julia error(...) (src/MPIAsyncPools.jl:157)."""


class DeviceError(RuntimeError):
    """A HIP call or a device-side check failed."""


_EXC = {
    _capi.MPA_ARGUMENT_ERROR: ArgumentError,
    _capi.MPA_DIMENSION_MISMATCH: DimensionMismatch,
    _capi.MPA_ERROR: ErrorException,
    _capi.MPA_DEVICE_ERROR: DeviceError,
    _capi.MPA_CALLBACK_ERROR: ErrorException,
}


def check(rc):
    if rc != _capi.MPA_OK:
        raise _EXC.get(rc, ErrorException)(_capi.last_error())


_torch = None


def _torch_mod():
    global _torch
    if _torch is None:
        try:
            import torch
            _torch = torch
        except ImportError:  # pragma: no cover
            _torch = False
    return _torch


def buffer_info(a):
    """(pointer, bytes, length, eltype, isbits, is_device) of a numpy array or torch tensor; the
    eltype is the dtype object (str() names it).  Runs four times per asyncmap! call, so it
    reads attributes only (the numpy ctypes view and str(dtype) cost a SIM call a third of its
    time)."""
    if isinstance(a, np.ndarray):
        if not a.flags.c_contiguous:
            raise ArgumentError("buffers must be contiguous")
        return a.__array_interface__["data"][0], a.nbytes, a.size, a.dtype, not a.dtype.hasobject, False
    torch = _torch_mod()
    if torch and isinstance(a, torch.Tensor):
        if not a.is_contiguous():
            raise ArgumentError("buffers must be contiguous")
        return a.data_ptr(), a.nbytes, a.numel(), a.dtype, True, a.is_cuda
    raise ArgumentError(f"unsupported buffer type {type(a).__name__}")


class MPIAsyncPool:
    """MPIAsyncPool (src/MPIAsyncPools.jl:24-46), state owned by libmpiasyncpools."""

    def __init__(self, n_or_ranks, epoch0=0, nwait=None):
        if np.isscalar(n_or_ranks):
            ranks = np.arange(1, int(n_or_ranks) + 1, dtype=np.int64)
        else:
            ranks = np.ascontiguousarray(n_or_ranks, dtype=np.int64)
        n = len(ranks)
        h = C.c_void_p()
        check(lib().mpa_pool_create(n, ranks.ctypes.data, int(epoch0), n if nwait is None else int(nwait),
                                    C.byref(h)))
        self._h = h
        self.n = n
        L = lib()

        def view(ptr, dt):
            if n == 0:
                return np.zeros(0, dtype=dt)
            return np.ctypeslib.as_array(ptr, shape=(n,)).view(dt)

        self.ranks = view(L.mpa_pool_ranks(h), np.int64)
        self.sepochs = view(L.mpa_pool_sepochs(h), np.int64)
        self.repochs = view(L.mpa_pool_repochs(h), np.int64)
        self.active = view(L.mpa_pool_active(h), np.bool_)
        self.stimestamps = view(L.mpa_pool_stimestamps(h), np.int64)
        self.latency = view(L.mpa_pool_latency(h), np.float64)
        self._nwait = L.mpa_pool_nwait(h)
        self._epoch = L.mpa_pool_epoch(h)

    @property
    def nwait(self):
        return int(self._nwait[0])

    @nwait.setter
    def nwait(self, v):
        self._nwait[0] = int(v)

    @property
    def epoch(self):
        return int(self._epoch[0])

    @epoch.setter
    def epoch(self, v):
        self._epoch[0] = int(v)

    def __len__(self):
        return self.n

    def __del__(self):
        h = getattr(self, "_h", None)
        if h is not None and h.value:
            try:
                lib().mpa_pool_destroy(h)
            except Exception:
                pass
            self._h = None


def _isbits_check(name_shown, a):
    ptr, nb, ln, elt, isbits, dev = buffer_info(a)
    if not isbits:  # src/MPIAsyncPools.jl:73-74 (message text as in the reference)
        raise ArgumentError(f"The eltype of {name_shown} must be isbits, but is {elt}")
    return ptr, nb, ln, dev


def asyncmap_(pool, sendbuf, recvbuf, isendbuf, irecvbuf, comm, nwait=None, epoch=None, tag=0):
    """Base.asyncmap! (src/MPIAsyncPools.jl:68-188)."""
    if nwait is None:
        nwait = pool.nwait
    if epoch is None:
        epoch = pool.epoch + 1
    s_ptr, s_nb, _, s_dev = _isbits_check("sendbuf", sendbuf)
    r_ptr, r_nb, r_len, r_dev = _isbits_check("sendbuf", recvbuf)  # sic, :74
    is_ptr, is_nb, _, _ = buffer_info(isendbuf)[:4]
    ir_ptr, ir_nb, _, _ = buffer_info(irecvbuf)[:4]
    comm._before_call(sendbuf)
    err = []
    cb = None
    fn_ptr, ctx, keep = None, None, None
    if _is_first_plus(nwait):  # the native predicate (mpa_nwait_first_plus)
        kind, k, fn_ptr, ctx, keep = _native_nwait(nwait)
    elif isinstance(nwait, (bool, np.bool_)):
        kind, k = _capi.MPA_NWAIT_OTHER, 0
    elif isinstance(nwait, (int, np.integer)):
        kind, k = _capi.MPA_NWAIT_INT, int(nwait)
    elif callable(nwait):
        kind, k = _capi.MPA_NWAIT_FN, 0

        def _f(ctx, ep, rep, n):
            try:
                r = nwait(ep, pool.repochs)
                if not isinstance(r, (bool, np.bool_)):  # `nwait(...)::Bool`, :153
                    raise TypeError(f"TypeError: in typeassert, expected Bool, got a value of type {type(r).__name__}")
                return 1 if r else 0
            except BaseException as e:
                err.append(e)
                return -1
        cb = _capi.NWAIT_FN(_f)
    else:
        kind, k = _capi.MPA_NWAIT_OTHER, 0
    out = C.POINTER(C.c_int64)()
    if cb:
        fn_ptr = C.cast(cb, C.c_void_p)
    rc = lib().mpa_asyncmap(pool._h, s_ptr, s_nb, r_ptr, r_nb, r_len, is_ptr, is_nb, ir_ptr, ir_nb,
                            comm._h, kind, k, fn_ptr, ctx, type(nwait).__name__.encode(), int(epoch), int(tag),
                            C.byref(out))
    del keep
    if err:
        raise err[0]
    check(rc)
    return pool.repochs


def waitall_(pool, recvbuf, irecvbuf):
    """waitall! (src/MPIAsyncPools.jl:195-224)."""
    r_ptr, r_nb, r_len, _ = _isbits_check("sendbuf", recvbuf)  # sic, :197
    ir_ptr, ir_nb, _, _ = buffer_info(irecvbuf)[:4]
    out = C.POINTER(C.c_int64)()
    check(lib().mpa_waitall(pool._h, r_ptr, r_nb, r_len, ir_ptr, ir_nb, C.byref(out)))
    return pool.repochs


def _device_buffer(name, t, dtype, numel):
    """A contiguous CUDA tensor of `numel` elements of `dtype`: the native loops hand raw
    pointers to device kernels, so an undersized or mistyped buffer is refused here (and its
    byte size is checked again in the library, src/MPIAsyncPools.jl:75-77)."""
    import torch
    if not isinstance(t, torch.Tensor) or not t.is_cuda:
        raise ArgumentError(f"{name} must be a CUDA tensor")
    if t.dtype != dtype:
        raise ArgumentError(f"{name} must be {dtype}, but is {t.dtype}")
    if not t.is_contiguous():
        raise ArgumentError(f"{name} must be contiguous")
    if t.numel() != numel:
        raise DimensionMismatch(f"{name} has {t.numel()} elements, but {numel} are needed")
    return C.c_void_p(t.data_ptr()), t.numel() * t.element_size()


def lsq_descent(pool, comm, x, recvbuf, isendbuf, irecvbuf, nwait, eta, epochs, stale_weight=0.0):
    """`epochs` iterations of the least-squares coordinator loop in native code
    (mpa_lsq_descent): asyncmap_(...; nwait) then x -= eta * n/sum(w) * sum_i w_i g_i with
    w_i = 1 for fresh chunks, stale_weight for older ones, 0 for workers never heard from."""
    from .comm import dtype_code
    n = pool.n
    xp, _ = _device_buffer("x", x, x.dtype, x.numel())
    r = _device_buffer("recvbuf", recvbuf, x.dtype, n * x.numel())
    s = _device_buffer("isendbuf", isendbuf, x.dtype, n * x.numel())
    ir = _device_buffer("irecvbuf", irecvbuf, x.dtype, n * x.numel())
    kind, k, fn, ctx, keep = _native_nwait(nwait)
    comm._before_call(x)
    check(lib().mpa_lsq_descent(pool._h, comm._h, dtype_code(x), xp, int(x.numel()), r[0], r[1], s[0], s[1],
                                ir[0], ir[1], kind, k, fn, ctx, float(eta), float(stale_weight), int(epochs)))
    del keep  # the predicate's context lives until the native loop has returned
    return pool.repochs


def first_plus(k):
    """nwait: worker 1 fresh and >= k of the others fresh (mpa_nwait_first_plus, native; the
    predicate of test/kmap2.jl:65 widened to k-of-n).  Accepted by asyncmap_ and the native
    loops alike."""
    return ("first_plus", int(k))


def _is_first_plus(nwait):
    return isinstance(nwait, tuple) and len(nwait) == 2 and nwait[0] == "first_plus"


def _native_nwait(nwait):
    """(kind, int nwait, fn pointer, ctx pointer, keep-alive) for the native descent loops;
    the caller holds `keep` for the duration of its call."""
    if _is_first_plus(nwait):
        ctx = C.c_int64(nwait[1])
        fn = C.cast(lib().mpa_nwait_first_plus, C.c_void_p)
        return _capi.MPA_NWAIT_FN, 0, fn, C.cast(C.byref(ctx), C.c_void_p), ctx
    if not isinstance(nwait, (int, np.integer)) or isinstance(nwait, bool):
        raise ArgumentError("the native loops take an integer nwait or first_plus(k)")
    return _capi.MPA_NWAIT_INT, int(nwait), None, None, None


def lsqb_descent(pool, comm, x32, xb16, recvbuf, isendbuf, irecvbuf, nwait, eta, epochs, stale_weight=0.0):
    """mpa_lsqb_descent: the coordinator loop of the batched 64-iterate variant.  x32 is the
    fp32 master iterate (cols x 64), xb16 its bf16 rounding = the message."""
    import torch
    n, e = pool.n, x32.numel()
    x32p, _ = _device_buffer("x32", x32, torch.float32, e)
    xbp, _ = _device_buffer("xb16", xb16, torch.bfloat16, e)
    r = _device_buffer("recvbuf", recvbuf, torch.float32, n * e)
    s = _device_buffer("isendbuf", isendbuf, torch.bfloat16, n * e)
    ir = _device_buffer("irecvbuf", irecvbuf, torch.float32, n * e)
    kind, k, fn, ctx, keep = _native_nwait(nwait)
    comm._before_call(x32)
    check(lib().mpa_lsqb_descent(pool._h, comm._h, x32p, xbp, int(e), r[0], r[1], s[0], s[1], ir[0], ir[1],
                                 kind, k, fn, ctx, float(eta), float(stale_weight), int(epochs)))
    del keep
    return pool.repochs


asyncmap = asyncmap_
waitall = waitall_
