"""ctypes binding of the C ABI (include/mpiasyncpools.h) of libmpiasyncpools.so.

The library is built in-tree (`make -C mpistragglers.jl_amd`, or __graft_entry__.build()).
There is no fallback: if the library is missing, importing the package fails loudly.
"""
import ctypes as C
import os

from . import abi

PKG_ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
# MPA_LIB: another build of the same library (A/B measurements of kernel variants)
LIB_PATH = os.environ.get("MPA_LIB") or os.path.join(PKG_ROOT, "_build", "libmpiasyncpools.so")

MPA_OK, MPA_ARGUMENT_ERROR, MPA_DIMENSION_MISMATCH, MPA_ERROR, MPA_DEVICE_ERROR, MPA_CALLBACK_ERROR = range(6)
MPA_F32, MPA_F64, MPA_BF16 = 0, 1, 2
MPA_TRANSPORT_HIP, MPA_TRANSPORT_SIM, MPA_TRANSPORT_HOST = 0, 1, 2
MPA_NWAIT_INT, MPA_NWAIT_FN, MPA_NWAIT_OTHER = 0, 1, 2
MPA_GATE_CALL, MPA_GATE_WAIT, MPA_GATE_WAITALL = 0, 1, 2
(MPA_TASK_NONE, MPA_TASK_ECHO, MPA_TASK_KMAP1, MPA_TASK_KMAP2, MPA_TASK_LSQ,
 MPA_TASK_LSQ_BATCH) = range(6)

NWAIT_FN = C.CFUNCTYPE(C.c_int, C.c_void_p, C.c_int64, C.POINTER(C.c_int64), C.c_int64)

# (name, restype, argtypes) for every symbol declared in include/mpiasyncpools.h, generated
# from the one signature table (abi.py) the Julia binding is generated from as well
SIGNATURES = abi.ctypes_signatures()

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
        if L.mpa_abi_version() != abi.ABI_VERSION:
            raise ImportError("libmpiasyncpools ABI version mismatch")
        _lib = L
    return _lib


def last_error():
    return lib().mpa_last_error().decode(errors="replace")
