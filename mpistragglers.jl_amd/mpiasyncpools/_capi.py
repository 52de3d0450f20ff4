"""ctypes binding of the C ABI (include/mpiasyncpools.h) of libmpiasyncpools.so.

The library is built in-tree (`make -C mpistragglers.jl_amd`, or __graft_entry__.build()).
There is no fallback: if the library is missing, importing the package fails loudly.
"""
import ctypes as C
import os

PKG_ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
# MPA_LIB: another build of the same library (A/B measurements of kernel variants)
LIB_PATH = os.environ.get("MPA_LIB") or os.path.join(PKG_ROOT, "_build", "libmpiasyncpools.so")

MPA_OK, MPA_ARGUMENT_ERROR, MPA_DIMENSION_MISMATCH, MPA_ERROR, MPA_DEVICE_ERROR, MPA_CALLBACK_ERROR = range(6)
MPA_F32, MPA_F64, MPA_BF16 = 0, 1, 2
MPA_TRANSPORT_HIP, MPA_TRANSPORT_SIM, MPA_TRANSPORT_HOST = 0, 1, 2
MPA_NWAIT_INT, MPA_NWAIT_FN, MPA_NWAIT_OTHER = 0, 1, 2
(MPA_TASK_NONE, MPA_TASK_ECHO, MPA_TASK_KMAP1, MPA_TASK_KMAP2, MPA_TASK_LSQ,
 MPA_TASK_LSQ_BATCH) = range(6)

NWAIT_FN = C.CFUNCTYPE(C.c_int, C.c_void_p, C.c_int64, C.POINTER(C.c_int64), C.c_int64)

_i64p = C.POINTER(C.c_int64)
_vp = C.c_void_p
_sz = C.c_size_t

# (name, restype, argtypes) for every symbol declared in include/mpiasyncpools.h
SIGNATURES = [
    ("mpa_abi_version", C.c_int, []),
    ("mpa_last_error", C.c_char_p, []),
    ("mpa_build_info", C.c_char_p, []),
    ("mpa_tune", C.c_int, [C.c_char_p, C.c_int64]),
    ("mpa_pool_create", C.c_int, [C.c_int64, _vp, C.c_int64, C.c_int64, C.POINTER(_vp)]),
    ("mpa_pool_destroy", None, [_vp]),
    ("mpa_pool_size", C.c_int64, [_vp]),
    ("mpa_pool_ranks", _i64p, [_vp]),
    ("mpa_pool_sepochs", _i64p, [_vp]),
    ("mpa_pool_repochs", _i64p, [_vp]),
    ("mpa_pool_active", C.POINTER(C.c_uint8), [_vp]),
    ("mpa_pool_stimestamps", _i64p, [_vp]),
    ("mpa_pool_latency", C.POINTER(C.c_double), [_vp]),
    ("mpa_pool_nwait", _i64p, [_vp]),
    ("mpa_pool_epoch", _i64p, [_vp]),
    ("mpa_asyncmap", C.c_int, [_vp, _vp, _sz, _vp, _sz, _sz, _vp, _sz, _vp, _sz, _vp,
                               C.c_int, C.c_int64, _vp, _vp, C.c_char_p, C.c_int64, C.c_int64,
                               C.POINTER(_i64p)]),
    ("mpa_waitall", C.c_int, [_vp, _vp, _sz, _sz, _vp, _sz, C.POINTER(_i64p)]),
    ("mpa_comm_create", C.c_int, [C.c_int, C.c_int64, _vp, C.POINTER(_vp)]),
    ("mpa_comm_destroy", None, [_vp]),
    ("mpa_comm_size", C.c_int64, [_vp]),
    ("mpa_comm_set_stream", C.c_int, [_vp, _vp]),
    ("mpa_comm_set_task_kmap", C.c_int, [_vp, C.c_int64, C.c_int]),
    ("mpa_comm_set_task_lsq", C.c_int, [_vp, C.c_int64, C.c_int, C.c_int64, C.c_int64, _vp, C.c_int64, _vp]),
    ("mpa_comm_set_task_lsq_batch", C.c_int, [_vp, C.c_int64, C.c_int64, C.c_int64, C.c_int64, _vp, C.c_int64, _vp]),
    ("mpa_comm_set_delays", C.c_int, [_vp, C.c_int64, _vp, C.c_int64]),
    ("mpa_comm_tasks_done", C.c_int64, [_vp, C.c_int64]),
    ("mpa_comm_shutdown", C.c_int, [_vp]),
    ("mpa_comm_create_dist", C.c_int, [C.c_int, C.c_int64, _vp, C.c_int, C.c_char_p, _sz, C.POINTER(_vp)]),
    ("mpa_comm_serve", C.c_int, [_vp]),
    ("mpa_comm_pause_servers", C.c_int, [_vp]),
    ("mpa_comm_payload_path", C.c_int, [_vp, C.c_int64]),
    ("mpa_comm_set_timing", C.c_int, [_vp, C.c_int]),
    ("mpa_comm_timing", C.c_int, [_vp, C.POINTER(C.c_double)]),
    ("mpa_comm_exchange_timing", C.c_int, [_vp, C.POINTER(C.c_double)]),
    ("mpa_comm_sim_set_compute", C.c_int, [_vp, C.c_int64]),
    ("mpa_comm_sim_advance", C.c_int, [_vp, C.c_int64]),
    ("mpa_comm_sim_now", C.c_int64, [_vp]),
    ("mpa_aggregate", C.c_int, [_vp, C.c_int, _vp, C.c_int64, C.c_int64, _vp, _vp]),
    ("mpa_lsq_update", C.c_int, [_vp, C.c_int, _vp, _vp, C.c_int64, C.c_int64, _vp, C.c_double]),
    ("mpa_lsq_descent", C.c_int, [_vp, _vp, C.c_int, _vp, C.c_int64, _vp, _vp, _vp, C.c_int, C.c_int64, _vp, _vp,
                                  C.c_double, C.c_double, C.c_int64]),
    ("mpa_nwait_first_plus", C.c_int, [_vp, C.c_int64, _vp, C.c_int64]),
    ("mpa_lsqb_update", C.c_int, [_vp, _vp, _vp, _vp, C.c_int64, C.c_int64, _vp, C.c_double]),
    ("mpa_lsqb_descent", C.c_int, [_vp, _vp, _vp, _vp, C.c_int64, _vp, _vp, _vp, C.c_int, C.c_int64, _vp, _vp,
                                   C.c_double, C.c_double, C.c_int64]),
    ("mpa_generate", C.c_int, [_vp, C.c_int, C.c_uint64, C.c_uint32, C.c_uint64, C.c_int64, C.c_double, _vp]),
    ("mpa_read_bandwidth", C.c_int, [_vp, C.c_size_t, C.c_int, C.c_int, _vp, C.POINTER(C.c_double)]),
]

_lib = None


def lib():
    """Load libmpiasyncpools.so (raises if it has not been built)."""
    global _lib
    if _lib is None:
        # One HIP runtime per process: torch bundles its own libamdhip64 (soname
        # libamdhip64.so.7, NEEDED unversioned by torch), so load torch first and let
        # libmpiasyncpools bind to the runtime already mapped; loading ours first would map
        # /opt/rocm's copy and torch would then map a second, disjoint runtime.
        try:
            import torch  # noqa: F401
        except ImportError:
            pass
        if not os.path.exists(LIB_PATH):
            raise ImportError(
                f"{LIB_PATH} is missing: build the HIP library first "
                "(`make -C mpistragglers.jl_amd` or `python -c 'import __graft_entry__ as g; g.build()'`)")
        L = C.CDLL(LIB_PATH)
        for name, res, args in SIGNATURES:
            f = getattr(L, name)
            f.restype = res
            f.argtypes = args
        if L.mpa_abi_version() != 1:
            raise ImportError("libmpiasyncpools ABI version mismatch")
        _lib = L
    return _lib


def last_error():
    return lib().mpa_last_error().decode(errors="replace")
