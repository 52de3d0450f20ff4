"""Communicators: the `comm::MPI.Comm` argument of asyncmap! plus the worker programs.

In the reference, rank 0 of MPI.COMM_WORLD is the coordinator and ranks 1..n run a
worker program (examples/iterative_example.jl:55-82, test/kmap1.jl:23-33,
test/kmap2.jl:76-99).  Here a communicator owns n device workers with ranks 1..n; each
worker runs a registered task kernel on its own HIP stream:

    comm = DeviceComm(n)                      # HIP transport, current GPU
    comm.set_task(rank, "kmap2")              # the reference's test worker programs
    comm.set_task_lsq(rank, A_i, b_i)         # g_i = A_i^T (A_i x - b_i)
    comm.set_task_lsq_batch(rank, A_i, B_i)   # G_i = A_i^T (A_i X - B_i), 64 iterates (bf16)
    comm.set_delays(rank, delays_ns)          # straggler emulation

`SimComm` is a deterministic virtual-clock host transport used only to test the pool
state machine without a GPU; it is never chosen implicitly.
"""
import ctypes as C

import numpy as np

from . import _capi
from ._capi import lib
from .pool import ArgumentError, buffer_info, check

_TASKS = {"echo": _capi.MPA_TASK_ECHO, "kmap1": _capi.MPA_TASK_KMAP1, "kmap2": _capi.MPA_TASK_KMAP2}
_DTYPES = {"float32": _capi.MPA_F32, "float64": _capi.MPA_F64, "torch.float32": _capi.MPA_F32,
           "torch.float64": _capi.MPA_F64, "bfloat16": _capi.MPA_BF16, "torch.bfloat16": _capi.MPA_BF16}


def dtype_code(a):
    return _DTYPES[str(a.dtype)]


def _row_major(A, b, cols, lda):
    """(rows, cols, lda) of a row-major A whose rows may be padded (a row-range or
    column-slice view is fine: the leading dimension is A's row stride); b must be
    contiguous.  A transposed view would silently give wrong gradients, so it is refused."""
    if A.shape[0] > 1 and A.stride(1) != 1:
        raise ArgumentError("A must be row-major with unit column stride (got strides %s)" % (tuple(A.stride()),))
    if not b.is_contiguous():
        raise ArgumentError("b / B must be contiguous")
    rows = int(A.shape[0])
    ld = int(A.stride(0)) if rows > 1 else int(A.shape[1])
    cols = int(A.shape[1]) if cols is None else int(cols)
    lda = ld if lda is None else int(lda)
    if cols > lda or (rows > 1 and lda != ld):
        raise ArgumentError(f"cols ({cols}) / lda ({lda}) do not match A's row stride ({ld})")
    return rows, cols, lda


class _Comm:
    transport = None

    def __init__(self, nworkers, devices=None, _handle=None):
        h = C.c_void_p()
        if _handle is not None:
            h = _handle
        else:
            dev = None
            if devices is not None:
                dev = (C.c_int * nworkers)(*devices)
            check(lib().mpa_comm_create(self.transport, int(nworkers), dev, C.byref(h)))
        self._h = h
        self.nworkers = int(nworkers)
        self._keep = {}

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    def size(self):
        """MPI.Comm_size: workers + the coordinator."""
        return int(lib().mpa_comm_size(self._h))

    def set_task(self, rank, task):
        check(lib().mpa_comm_set_task_kmap(self._h, int(rank), _TASKS[task]))

    def set_delays(self, rank, delays_ns):
        d = np.ascontiguousarray(delays_ns, dtype=np.int64)
        check(lib().mpa_comm_set_delays(self._h, int(rank), d.ctypes.data if d.size else None, d.size))

    def tasks_done(self, rank):
        return int(lib().mpa_comm_tasks_done(self._h, int(rank)))

    def shutdown(self):
        """Control channel (examples/iterative_example.jl:49-52): drain, then stop."""
        check(lib().mpa_comm_shutdown(self._h))

    def counter(self, name):
        """An event counter of the transport (mpa_comm_counter, include/mpiasyncpools.h):
        "held", "held_joined", "held_alone", "gate_steps", "head_steps", "epoch_kernels",
        "prearmed", "prearm_cancelled", "prearm_same", "stale_deferred", "task_launches",
        "armed", "sleeps", "clock_samples", "timer_late", "queues", "queues_past_cap",
        "shared_worker_streams", "reserved_cus"; -1 if the transport does not count it."""
        return int(lib().mpa_comm_counter(self._h, name.encode()))

    def set_gate(self, kinds, offsets, ranks):
        """Gated replay (mpa_comm_set_gate, a test mode): at the k-th observation point of
        the state machine (kinds[k]: MPA_GATE_CALL / _WAIT / _WAITALL) one more completion of
        each rank in ranks[offsets[k]:offsets[k+1]] becomes visible, and only released
        completions are.  The schedule comes from the oracle (OracleSim.gate_schedule);
        kinds == [] switches the gate off."""
        k = np.ascontiguousarray(kinds, dtype=np.int32)
        o = np.ascontiguousarray(offsets, dtype=np.int64)
        r = np.ascontiguousarray(ranks, dtype=np.int64)
        if k.size and o.size != k.size + 1:
            raise ArgumentError("gate schedule: offsets needs one entry more than kinds")
        self._keep["gate"] = (k, o, r)
        check(lib().mpa_comm_set_gate(self._h, int(k.size), k.ctypes.data if k.size else None,
                                      o.ctypes.data if o.size else None, r.ctypes.data if r.size else None))

    def _before_call(self, sendbuf):
        pass

    def close(self):
        h = getattr(self, "_h", None)
        if h is not None and h.value:
            lib().mpa_comm_destroy(h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class DeviceComm(_Comm):
    """HIP transport: workers are task kernels on per-worker streams of the current GPU.

    Buffers passed to asyncmap_/waitall_ with this comm are torch CUDA tensors on the
    coordinator's GPU; the pool's copies are ordered on torch's current stream."""

    transport = _capi.MPA_TRANSPORT_HIP

    def __init__(self, nworkers, devices=None):
        import torch
        if not torch.cuda.is_available():
            raise RuntimeError("DeviceComm needs a GPU (HIP); no device is visible")
        torch.cuda.init()
        super().__init__(nworkers, devices)

    _stream = None  # the stream last handed to the library

    def _before_call(self, sendbuf):
        # torch's current stream (the raw handle: a Stream object costs microseconds per call),
        # passed on only when it changed
        import torch
        raw = getattr(torch._C, "_cuda_getCurrentRawStream", None)
        s = raw(torch.cuda.current_device()) if raw else torch.cuda.current_stream().cuda_stream
        if s != self._stream:
            check(lib().mpa_comm_set_stream(self._h, C.c_void_p(s)))
            self._stream = s

    def set_task_lsq(self, rank, A, b, cols=None, lda=None):
        """g = A^T (A x - b) with A (rows x cols, row-major, leading dim lda) and b on the GPU."""
        if A.dim() != 2 or b.dim() != 1 or A.shape[0] != b.shape[0]:
            raise ArgumentError("A must be rows x lda and b must have rows elements")
        if A.dtype != b.dtype:
            raise ArgumentError("A and b must have the same dtype")
        rows, cols, lda = _row_major(A, b, cols, lda)
        check(lib().mpa_comm_set_task_lsq(self._h, int(rank), dtype_code(A), int(rows), cols,
                                          C.c_void_p(A.data_ptr()), lda, C.c_void_p(b.data_ptr())))
        self._keep[int(rank)] = (A, b)

    def set_task_lsq_batch(self, rank, A, B, cols=None, lda=None):
        """G = A^T (A X - B): the batched 64-iterate variant (bf16 in, fp32 G).

        A (rows x lda, bf16, row-major), B (rows x 64, bf16) on the GPU; the message X is
        cols x 64 bf16 and the reply G is cols x 64 fp32 (both row-major)."""
        import torch
        if A.dim() != 2 or B.dim() != 2 or A.shape[0] != B.shape[0]:
            raise ArgumentError("A must be rows x lda and B rows x k")
        if A.dtype != torch.bfloat16 or B.dtype != torch.bfloat16:
            raise ArgumentError("the batched variant takes bf16 A and B")
        rows, cols, lda = _row_major(A, B, cols, lda)
        check(lib().mpa_comm_set_task_lsq_batch(self._h, int(rank), int(rows), cols, int(B.shape[1]),
                                                C.c_void_p(A.data_ptr()), lda, C.c_void_p(B.data_ptr())))
        self._keep[int(rank)] = (A, B)

    def set_timing(self, enable, period=1):
        """Time least-squares launches with HIP events on their own stream: every launch, or
        one in every `period` launches (and epoch kernels)."""
        if int(period) < 1:
            raise ValueError("period must be >= 1")
        check(lib().mpa_comm_set_timing(self._h, int(period) if enable else 0))

    def timing(self):
        """(launches, kernel_ms, algorithmic_bytes, busy_ms) since the previous call;
        busy_ms = the union of the launch intervals (concurrent launches overlap)."""
        out = (C.c_double * 4)()
        check(lib().mpa_comm_timing(self._h, out))
        return int(out[0]), float(out[1]), float(out[2]), float(out[3])

    def exchange_timing(self):
        """(epoch_kernel_launches, ms, remote_payload_bytes) of the coordinator's timed epoch
        kernels since the previous call (mpa_comm_exchange_timing)."""
        out = (C.c_double * 3)()
        check(lib().mpa_comm_exchange_timing(self._h, out))
        return int(out[0]), float(out[1]), float(out[2])

    TRACE_FIELDS = ("rank", "seq", "post", "due", "call", "ret", "start", "pub", "gate", "seen", "harvest")

    def set_trace(self, capacity):
        """Trace the next `capacity` posted tasks (mpa_comm_set_trace; 0 = off)."""
        check(lib().mpa_comm_set_trace(self._h, int(capacity)))

    def trace(self, capacity=1 << 16):
        """The task trace as an int64 array (tasks x 11, columns TRACE_FIELDS, host ns)."""
        out = np.zeros((int(capacity), len(self.TRACE_FIELDS)), dtype=np.int64)
        n = C.c_int64(0)
        check(lib().mpa_comm_trace(self._h, out.ctypes.data_as(C.POINTER(C.c_int64)), int(capacity), C.byref(n)))
        return out[:n.value]

    def aggregate(self, recvbuf, nchunks, weights, out):
        """out = sum_i weights[i] * chunk_i of recvbuf (device kernel, fixed order)."""
        w = np.ascontiguousarray(weights, dtype=np.float64)
        chunk = recvbuf.numel() // nchunks
        self._before_call(out)
        check(lib().mpa_aggregate(self._h, dtype_code(recvbuf), C.c_void_p(recvbuf.data_ptr()), int(nchunks),
                                  int(chunk), w.ctypes.data, C.c_void_p(out.data_ptr())))

    def lsq_update(self, x, recvbuf, nchunks, weights, eta):
        """x -= eta * sum_i weights[i] * g_i (device kernel, fixed order)."""
        w = np.ascontiguousarray(weights, dtype=np.float64)
        self._before_call(x)
        check(lib().mpa_lsq_update(self._h, dtype_code(x), C.c_void_p(x.data_ptr()),
                                   C.c_void_p(recvbuf.data_ptr()), int(nchunks), int(x.numel()),
                                   w.ctypes.data, float(eta)))

    def lsqb_update(self, x32, xb16, recvbuf, nchunks, weights, eta):
        """Batched variant: x32 -= eta * sum_i weights[i] * G_i ; xb16 = bf16(x32) (one kernel)."""
        w = np.ascontiguousarray(weights, dtype=np.float64)
        self._before_call(x32)
        check(lib().mpa_lsqb_update(self._h, C.c_void_p(x32.data_ptr()), C.c_void_p(xb16.data_ptr()),
                                    C.c_void_p(recvbuf.data_ptr()), int(nchunks), int(x32.numel()),
                                    w.ctypes.data, float(eta)))


class DistComm(DeviceComm):
    """One process per GPU.

    Every rank constructs it with the same `placement` (placement[w-1] = the process rank
    serving worker w) and `shm_name`; rank 0 must construct it first (it creates the
    shared-memory mailboxes).  Rank 0 is the coordinator and calls asyncmap_/waitall_;
    every other rank registers the tasks of its workers and calls serve(), which returns
    when rank 0 calls pause_servers() or shutdown().  transport="host" runs the same
    protocol with host-executed test workers (echo/kmap1/kmap2) and no GPU."""

    def __init__(self, nworkers, placement, rank, shm_name, max_msg_bytes, transport="hip"):
        code = {"hip": _capi.MPA_TRANSPORT_HIP, "host": _capi.MPA_TRANSPORT_HOST}[transport]
        if code == _capi.MPA_TRANSPORT_HIP:
            import torch
            if not torch.cuda.is_available():
                raise RuntimeError("DistComm(transport='hip') needs a GPU (HIP); no device is visible")
            torch.cuda.init()
        pl = (C.c_int * nworkers)(*[int(p) for p in placement])
        h = C.c_void_p()
        check(lib().mpa_comm_create_dist(code, int(nworkers), pl, int(rank), shm_name.encode(), int(max_msg_bytes),
                                         C.byref(h)))
        self.transport = code
        self.rank = int(rank)
        self.placement = list(placement)
        _Comm.__init__(self, nworkers, _handle=h)

    def _before_call(self, sendbuf):
        if self.transport == _capi.MPA_TRANSPORT_HIP:
            DeviceComm._before_call(self, sendbuf)

    def serve(self):
        """Worker processes: serve this rank's workers until rank 0 pauses or shuts down."""
        check(lib().mpa_comm_serve(self._h))

    def pause_servers(self):
        check(lib().mpa_comm_pause_servers(self._h))

    def payload_path(self, rank):
        """Rank 0: 'device' (xGMI, HIP IPC), 'host' (shared-memory mailbox) or None
        (undecided / served here) for worker `rank`."""
        return {1: "host", 2: "device"}.get(int(lib().mpa_comm_payload_path(self._h, int(rank))))


class SimComm(_Comm):
    """Virtual-clock host transport (tests of the state machine only); numpy buffers."""

    transport = _capi.MPA_TRANSPORT_SIM

    def set_compute(self, ns):
        check(lib().mpa_comm_sim_set_compute(self._h, int(ns)))

    def advance(self, dt_ns):
        check(lib().mpa_comm_sim_advance(self._h, int(dt_ns)))

    @property
    def now(self):
        return int(lib().mpa_comm_sim_now(self._h))


def generate(out, seed, stream, e0, scale=1.0):
    """Fill a CUDA tensor with the Philox4x32-10 synthetic layout."""
    import torch
    check(lib().mpa_generate(C.c_void_p(out.data_ptr()), dtype_code(out), int(seed), int(stream), int(e0),
                             int(out.numel()), float(scale), C.c_void_p(torch.cuda.current_stream().cuda_stream)))


def read_bandwidth(buf, grid=2048, reps=10):
    """Measured HBM read rate (GB/s) of a plain streaming read over a CUDA tensor's bytes
    (mpa_read_bandwidth): the ceiling bench.py reads the shard kernels' rate against."""
    import torch
    out = C.c_double()
    nbytes = buf.numel() * buf.element_size() // 16 * 16
    check(lib().mpa_read_bandwidth(C.c_void_p(buf.data_ptr()), nbytes, int(grid), int(reps),
                                   C.c_void_p(torch.cuda.current_stream().cuda_stream), C.byref(out)))
    return out.value
