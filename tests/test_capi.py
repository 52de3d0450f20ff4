"""The C-ABI library loads and exports every symbol include/*.h declares (no GPU needed,
no compute calls), and the Python binding declares a signature for each of them."""
import ctypes
import glob
import os
import re


ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


# headers of the device library; include/mpiasyncpools_mpi.h belongs to the optional MPI
# transport library (tests/test_mpi_transport.py checks its export)
MPI_HEADER = "mpiasyncpools_mpi.h"


def declared(headers=None):
    names = []
    for h in headers or [h for h in glob.glob(os.path.join(ROOT, "include", "*.h")) if not h.endswith(MPI_HEADER)]:
        src = open(h).read()
        src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
        src = re.sub(r"//[^\n]*", "", src)
        for m in re.finditer(r"\b(mpa_[a-z0-9_]+)\s*\(", src):
            if not src[:m.start()].rstrip().endswith("(*"):  # skip function-pointer typedefs
                names.append(m.group(1))
    return sorted(set(names) - {"mpa_nwait_fn"})


def test_header_declares_entry_points():
    names = declared()
    for must in ("mpa_pool_create", "mpa_asyncmap", "mpa_waitall", "mpa_comm_create", "mpa_comm_create_dist",
                 "mpa_comm_serve", "mpa_comm_set_task_lsq", "mpa_lsq_update", "mpa_generate"):
        assert must in names


def test_library_exports_every_declared_symbol(built):
    from mpiasyncpools import _capi
    lib = ctypes.CDLL(_capi.LIB_PATH)
    missing = [n for n in declared() if not hasattr(lib, n)]
    assert missing == []
    bound = {s[0] for s in _capi.SIGNATURES}
    assert sorted(set(declared()) - bound) == []


def test_abi_version_and_build_info(built):
    from mpiasyncpools._capi import lib
    assert lib().mpa_abi_version() == 3
    assert b"gfx950" in lib().mpa_build_info()


def test_errors_without_device(built):
    """Argument errors come back as status codes with the message, no GPU involved."""
    from mpiasyncpools._capi import lib, MPA_ARGUMENT_ERROR
    h = ctypes.c_void_p()
    assert lib().mpa_comm_create(7, 1, None, ctypes.byref(h)) == MPA_ARGUMENT_ERROR
    assert b"unknown transport" in lib().mpa_last_error()
    assert lib().mpa_tune(b"nope", 1) == MPA_ARGUMENT_ERROR
    assert b"unknown tuning key" in lib().mpa_last_error()
    out = ctypes.c_double()
    assert lib().mpa_read_bandwidth(None, 1 << 20, 1024, 1, None, ctypes.byref(out)) == MPA_ARGUMENT_ERROR
    assert b"read_bandwidth: bad arguments" in lib().mpa_last_error()


def test_kernel_object_is_gfx950_only(built):
    """The fat binary carries gfx950 code objects and no other target."""
    so = open(os.path.join(ROOT, "mpistragglers.jl_amd", "_build", "libmpiasyncpools.so"), "rb").read()
    targets = set(re.findall(rb"amdgcn-amd-amdhsa--(gfx[0-9a-z]+)", so))
    assert targets == {b"gfx950"}, targets
