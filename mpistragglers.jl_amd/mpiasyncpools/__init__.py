"""MI355X-native MPIAsyncPools: the `asyncmap!` hot path of MPIAsyncPools.jl
(severinson/MPIStragglers.jl) over HIP streams, device task kernels and host-visible
completion words.  See DESIGN.md at the repository root.
"""
from ._capi import MPA_GATE_CALL, MPA_GATE_WAIT, MPA_GATE_WAITALL, lib  # noqa: F401  (fails loudly if the HIP library is not built)
from .comm import DeviceComm, DistComm, SimComm, generate, read_bandwidth  # noqa: F401
from .pool import (ArgumentError, DeviceError, DimensionMismatch, ErrorException,  # noqa: F401
                   MPIAsyncPool, asyncmap, asyncmap_, first_plus, lsq_descent, lsqb_descent, waitall, waitall_)

lib()

__all__ = ["MPIAsyncPool", "asyncmap_", "waitall_", "asyncmap", "waitall", "lsq_descent", "lsqb_descent", "first_plus", "DeviceComm", "DistComm",
           "SimComm", "generate", "read_bandwidth", "MPA_GATE_CALL", "MPA_GATE_WAIT", "MPA_GATE_WAITALL", "ArgumentError", "DimensionMismatch", "ErrorException", "DeviceError"]
