"""ORACLE — TEST INFRASTRUCTURE ONLY.

ctypes binding of the C restatement of MPIAsyncPools.jl (asyncpool_oracle.c) and of its
virtual-clock worker transport.  Mirrors the reference API so tests read like
test/kmap1.jl and test/kmap2.jl:

    pool = OraclePool(n)                                   # src/MPIAsyncPools.jl:46
    repochs = asyncmap(pool, sim, sendbuf, recvbuf, isendbuf, irecvbuf,
                       nwait=..., epoch=..., tag=...)      # :68
    repochs = waitall(pool, sim, recvbuf, irecvbuf)        # :195

`repochs` aliases the pool's state vector (the reference returns `pool.repochs` itself,
:187), so later calls mutate arrays returned earlier.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import this.
"""
import ctypes as C
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
BUILD = os.path.join(HERE, "_build")
LIB_PATH = os.path.join(BUILD, "liboracle.so")

ORC_WORKER_ECHO, ORC_WORKER_KMAP1, ORC_WORKER_KMAP2, ORC_WORKER_TAG = 0, 1, 2, 3


class ArgumentError(ValueError):
    """Julia ArgumentError."""


class DimensionMismatch(ValueError):
    """Julia DimensionMismatch."""


class ErrorException(RuntimeError):
    """Julia error(...)."""


_ERRS = {1: ArgumentError, 2: DimensionMismatch, 3: ErrorException}


def build():
    """Compile the oracle (gcc) into oracle/_build/."""
    subprocess.check_call(["make", "-s", "-C", HERE, "all"])


_lib = None


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            build()
        L = C.CDLL(LIB_PATH)
        L.orc_pool_create.restype = C.c_void_p
        L.orc_pool_create.argtypes = [C.c_int64, C.c_void_p, C.c_int64, C.c_int64]
        L.orc_pool_destroy.argtypes = [C.c_void_p]
        L.orc_asyncmap.restype = C.c_int
        L.orc_asyncmap.argtypes = [C.c_void_p, C.c_void_p,
                                   C.c_void_p, C.c_size_t,
                                   C.c_void_p, C.c_size_t, C.c_size_t,
                                   C.c_void_p, C.c_size_t,
                                   C.c_void_p, C.c_size_t,
                                   C.c_int, C.c_int64, C.c_void_p, C.c_void_p,
                                   C.c_char_p, C.c_int64, C.c_int64]
        L.orc_waitall.restype = C.c_int
        L.orc_waitall.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, C.c_size_t, C.c_size_t,
                                  C.c_void_p, C.c_size_t]
        L.orc_sim_create.restype = C.c_void_p
        L.orc_sim_create.argtypes = [C.c_int64, C.c_int, C.c_void_p, C.c_int64, C.c_int64]
        L.orc_sim_destroy.argtypes = [C.c_void_p]
        L.orc_sim_transport.argtypes = [C.c_void_p, C.c_void_p]
        L.orc_sim_advance.argtypes = [C.c_void_p, C.c_int64]
        L.orc_sim_now.restype = C.c_int64
        L.orc_sim_now.argtypes = [C.c_void_p]
        L.orc_sim_tasks.restype = C.c_int64
        L.orc_sim_tasks.argtypes = [C.c_void_p, C.c_int64]
        L.orc_sim_events.restype = C.c_int64
        L.orc_sim_events.argtypes = [C.c_void_p, C.c_void_p, C.c_int64]
        L.orc_sim_obs.restype = C.c_int64
        L.orc_sim_obs.argtypes = [C.c_void_p, C.c_void_p, C.c_int64]
        _lib = L
    return _lib


class _Transport(C.Structure):
    _fields_ = [("ctx", C.c_void_p), ("isend_irecv", C.c_void_p), ("test", C.c_void_p),
                ("waitany", C.c_void_p), ("waitall", C.c_void_p), ("time_ns", C.c_void_p),
                ("observe", C.c_void_p)]


class _PoolStruct(C.Structure):
    _fields_ = [("n", C.c_int64),
                ("ranks", C.POINTER(C.c_int64)), ("sepochs", C.POINTER(C.c_int64)),
                ("repochs", C.POINTER(C.c_int64)), ("active", C.POINTER(C.c_uint8)),
                ("stimestamps", C.POINTER(C.c_int64)), ("latency", C.POINTER(C.c_double)),
                ("rreq_live", C.POINTER(C.c_uint8)),
                ("nwait", C.c_int64), ("epoch", C.c_int64), ("errmsg", C.c_char * 512)]


class _Obs(C.Structure):
    _fields_ = [("kind", C.c_int64), ("worker", C.c_int64), ("t", C.c_int64), ("done_ns", C.c_int64),
                ("now", C.c_int64)]


# observation kinds of the sim's log (asyncpool_oracle.h ORC_OBS_*; the first three are the
# step kinds of a gated replay, include/mpiasyncpools.h MPA_GATE_*)
OBS_CALL, OBS_WAIT, OBS_WAITALL, OBS_POST = 0, 1, 2, 3


class _Event(C.Structure):
    _fields_ = [("worker", C.c_int64), ("t", C.c_int64), ("post_ns", C.c_int64),
                ("done_ns", C.c_int64), ("seen_ns", C.c_int64)]


NWAIT_FN = C.CFUNCTYPE(C.c_int, C.c_void_p, C.c_int64, C.POINTER(C.c_int64), C.c_int64)


class OraclePool:
    """MPIAsyncPool (src/MPIAsyncPools.jl:24-46) restated in C."""

    def __init__(self, n_or_ranks, epoch0=0, nwait=None):
        if np.isscalar(n_or_ranks):
            ranks = np.arange(1, int(n_or_ranks) + 1, dtype=np.int64)
        else:
            ranks = np.asarray(n_or_ranks, dtype=np.int64)
        n = len(ranks)
        self._h = lib().orc_pool_create(n, ranks.ctypes.data, int(epoch0), n if nwait is None else int(nwait))
        self._s = _PoolStruct.from_address(self._h)
        self.n = n

        def arr(ptr, dt):
            return np.ctypeslib.as_array(ptr, shape=(max(n, 1),))[:n].view(dt)

        self.ranks = arr(self._s.ranks, np.int64)
        self.sepochs = arr(self._s.sepochs, np.int64)
        self.repochs = arr(self._s.repochs, np.int64)
        self.active = arr(self._s.active, np.bool_)
        self.stimestamps = arr(self._s.stimestamps, np.int64)
        self.latency = arr(self._s.latency, np.float64)

    @property
    def epoch(self):
        return self._s.epoch

    @property
    def nwait(self):
        return self._s.nwait

    def __del__(self):
        try:
            lib().orc_pool_destroy(self._h)
        except Exception:
            pass


class OracleSim:
    """Virtual-clock workers: task t of worker w lasts durations[w, (t-1) % ncols] + compute_ns."""

    def __init__(self, nworkers, kind=ORC_WORKER_TAG, durations_ns=None, compute_ns=0):
        d = np.zeros((nworkers, 1), dtype=np.int64) if durations_ns is None else \
            np.ascontiguousarray(durations_ns, dtype=np.int64).reshape(nworkers, -1)
        self._d = d
        self._h = lib().orc_sim_create(nworkers, kind, d.ctypes.data, d.shape[1], int(compute_ns))
        self._tp = _Transport()
        lib().orc_sim_transport(self._h, C.byref(self._tp))
        self.nworkers = nworkers

    def advance(self, dt_ns):
        lib().orc_sim_advance(self._h, int(dt_ns))

    @property
    def now(self):
        return lib().orc_sim_now(self._h)

    def tasks(self, w):
        return lib().orc_sim_tasks(self._h, w)

    def events(self):
        n = lib().orc_sim_events(self._h, None, 0)
        buf = (_Event * max(n, 1))()
        lib().orc_sim_events(self._h, buf, n)
        return [(e.worker, e.t, e.post_ns, e.done_ns, e.seen_ns) for e in buf[:n]]

    def observations(self):
        """The sim's observation log: (kind, worker, t, done_ns, now) in program order."""
        n = lib().orc_sim_obs(self._h, None, 0)
        buf = (_Obs * max(n, 1))()
        lib().orc_sim_obs(self._h, buf, n)
        return [(o.kind, o.worker, o.t, o.done_ns, o.now) for o in buf[:n]]

    def gate_schedule(self, ranks=None):
        """The gated-replay schedule of everything run on this sim so far (the arguments
        of mpa_comm_set_gate): at every observation point, the tasks whose virtual
        completion time has passed and that no earlier point released -- exactly the
        completions the oracle's Test!/Waitany!/Waitall! could see there.  `ranks` maps
        the sim's worker positions (pool positions) to comm ranks (default 1..n).

        Returns (kinds, offsets, ranks) as int32 / int64 / int64 arrays."""
        ranks = np.arange(1, self.nworkers + 1) if ranks is None else np.asarray(ranks)
        pending, kinds, offs, rel = [], [], [0], []
        for kind, w, t, done, now in self.observations():
            if kind == OBS_POST:
                pending.append((done, int(ranks[w])))
                continue
            rel.extend(sorted(r for d, r in pending if d <= now))
            pending = [p for p in pending if p[0] > now]
            kinds.append(kind)
            offs.append(len(rel))
        return (np.asarray(kinds, dtype=np.int32), np.asarray(offs, dtype=np.int64),
                np.asarray(rel, dtype=np.int64))

    def __del__(self):
        try:
            lib().orc_sim_destroy(self._h)
        except Exception:
            pass


def _buf(a):
    a = np.asarray(a)
    assert a.flags.c_contiguous
    return a.ctypes.data, a.nbytes, a.size


def _raise(pool, rc):
    if rc != 0:
        raise _ERRS.get(rc, ErrorException)(pool._s.errmsg.decode())


def asyncmap(pool, sim, sendbuf, recvbuf, isendbuf, irecvbuf, nwait=None, epoch=None, tag=0):
    """Base.asyncmap! (src/MPIAsyncPools.jl:68-188) over the simulated transport."""
    if nwait is None:
        nwait = pool.nwait
    if epoch is None:
        epoch = pool.epoch + 1
    for name, a in (("sendbuf", sendbuf), ("recvbuf", recvbuf)):  # :73-74
        if np.asarray(a).dtype == object:
            raise ArgumentError(f"The eltype of sendbuf must be isbits, but is {np.asarray(a).dtype}")
    s, sb, _ = _buf(sendbuf)
    r, rb, rn = _buf(recvbuf)
    i_s, isb, _ = _buf(isendbuf)
    i_r, irb, _ = _buf(irecvbuf)
    cb = None
    err = []
    if isinstance(nwait, (int, np.integer)) and not isinstance(nwait, bool):
        kind, k = 0, int(nwait)
    elif callable(nwait):
        kind, k = 1, 0

        def _f(ctx, ep, rep, n):
            try:
                return 1 if bool(nwait(ep, pool.repochs)) else 0
            except Exception as e:  # propagate after the C frame unwinds
                err.append(e)
                return -1
        cb = NWAIT_FN(_f)
    else:
        kind, k = 2, 0
    rc = lib().orc_asyncmap(pool._h, C.byref(sim._tp), s, sb, r, rb, rn, i_s, isb, i_r, irb,
                            kind, k, C.cast(cb, C.c_void_p) if cb else None, None,
                            type(nwait).__name__.encode(), int(epoch), int(tag))
    if err:
        raise err[0]
    _raise(pool, rc)
    return pool.repochs


def waitall(pool, sim, recvbuf, irecvbuf):
    """waitall! (src/MPIAsyncPools.jl:195-224) over the simulated transport."""
    if np.asarray(recvbuf).dtype == object:  # :197
        raise ArgumentError(f"The eltype of sendbuf must be isbits, but is {np.asarray(recvbuf).dtype}")
    r, rb, rn = _buf(recvbuf)
    i_r, irb, _ = _buf(irecvbuf)
    rc = lib().orc_waitall(pool._h, C.byref(sim._tp), r, rb, rn, i_r, irb)
    _raise(pool, rc)
    return pool.repochs
