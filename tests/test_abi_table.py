"""Header, Python and Julia bindings come from ONE signature table:

  * include/mpiasyncpools.h declares exactly the prototypes of mpiasyncpools/abi.py;
  * the ctypes argtypes the Python binding loads are generated from that table;
  * julia/MPIAsyncPools/src/capi.jl is what julia/gen_capi.py writes from it;
  * every mpa_* call of the Julia module names a table entry with the right arity.
"""
import os
import re
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
JL = os.path.join(ROOT, "julia", "MPIAsyncPools", "src")


def test_header_matches_table():
    from mpiasyncpools import abi
    header = abi.parse(open(os.path.join(ROOT, "include", "mpiasyncpools.h")).read())
    assert header == abi.table()
    assert "#define MPA_ABI_VERSION %d" % abi.ABI_VERSION in open(os.path.join(ROOT, "include", "mpiasyncpools.h")).read()


def test_python_signatures_come_from_table():
    from mpiasyncpools import _capi, abi
    assert _capi.SIGNATURES == abi.ctypes_signatures()
    assert [s[0] for s in _capi.SIGNATURES] == [t[0] for t in abi.table()]


def test_julia_capi_is_generated_from_table():
    p = subprocess.run([sys.executable, os.path.join(ROOT, "julia", "gen_capi.py"), "--check"],
                       capture_output=True, text=True)
    assert p.returncode == 0, p.stdout + p.stderr


def _calls(src, name):
    """Argument lists (top-level comma split) of every call `name(...)` in src."""
    out = []
    for m in re.finditer(r"\b%s\(" % re.escape(name), src):
        depth, i, start, args = 1, m.end(), m.end(), []
        while depth:
            c = src[i]
            if c in "([{":
                depth += 1
            elif c in ")]}":
                depth -= 1
            elif c == "," and depth == 1:
                args.append(src[start:i])
                start = i + 1
            i += 1
        last = src[start:i - 1]
        if last.strip() or args:
            args.append(last)
        out.append(args)
    return out


def test_julia_module_calls_exist_with_arity():
    from mpiasyncpools import abi
    arity = {name: len(params) for name, _, params in abi.table()}
    src = open(os.path.join(JL, "MPIAsyncPools.jl")).read()
    used = set(re.findall(r"\b(mpa_[a-z0-9_]+)\(", src))
    assert used and used <= set(arity), used - set(arity)
    for name in used:
        for args in _calls(src, name):
            assert len(args) == arity[name], (name, args)


def test_julia_capi_types_match_arity():
    from mpiasyncpools import abi
    src = open(os.path.join(JL, "capi.jl")).read()
    for name, _, params in abi.table():
        m = re.search(r"ccall\(\(:%s, libmpiasyncpools\), [^,]+, \(([^)]*)\)" % name, src)
        assert m, name
        types = [t for t in m.group(1).split(", ") if t.strip(",")]
        assert len(types) == len(params), (name, types)


def test_julia_mpi_extension_matches_its_header():
    """The package extension for MPI.Comm ccalls mpa_comm_create_mpi as
    include/mpiasyncpools_mpi.h declares it (int64_t Fortran handle, mpa_comm** out)."""
    from mpiasyncpools import abi
    decl = {n: (r, p) for n, r, p in abi.parse(open(os.path.join(ROOT, "include", "mpiasyncpools_mpi.h")).read())}
    assert "mpa_comm_create_mpi" in decl
    ret, params = decl["mpa_comm_create_mpi"]
    src = open(os.path.join(ROOT, "julia", "MPIAsyncPools", "ext", "MPIAsyncPoolsMPIExt.jl")).read()
    m = re.search(r"ccall\(\(:mpa_comm_create_mpi, libmpi_t\), (\w+), \(([^)]*)\)", src)
    assert m, "the extension ccalls mpa_comm_create_mpi"
    assert m.group(1) == abi.julia_type(ret)
    assert [t.strip() for t in m.group(2).split(",")] == [abi.julia_type(t) for t, _ in params]
    proj = open(os.path.join(ROOT, "julia", "MPIAsyncPools", "Project.toml")).read()
    assert 'MPIAsyncPoolsMPIExt = "MPI"' in proj


def test_julia_byte_counts_are_data_bytes():
    """Buffer byte counts handed to the ABI are length * element size (`_nbytes`), never
    `sizeof(buffer)`, which for a wrapper array type is the wrapper's size."""
    src = open(os.path.join(JL, "MPIAsyncPools.jl")).read()
    for name in ("mpa_asyncmap", "mpa_waitall", "mpa_lsq_descent", "mpa_lsqb_descent"):
        for args in _calls(src, name):
            assert not any(re.search(r"\bsizeof\(", a) for a in args), (name, args)
    assert "DistComm" in src and "serve!" in src and "set_task_lsq_batch!" in src and "lsqb_descent!" in src
