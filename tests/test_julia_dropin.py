"""The Julia drop-in answers to the reference programs' `using MPIAsyncPools`.

Julia is not installed in this image, so this is a static check of the committed package
(`julia/MPIAsyncPools/`) against what the reference's own programs use:

  * package identity: name and uuid of the reference's `Project.toml:1-2`, so `Pkg.develop`
    of this directory replaces the reference in an environment that depends on it;
  * every program (`test/kmap1.jl:2`, `test/kmap2.jl:2`, `test/runtests.jl:2`,
    `examples/iterative_example.jl:5`) loads `MPIAsyncPools`, and the module of that name
    exports the reference's export list (`src/MPIAsyncPools.jl:9`) and extends
    `Base.asyncmap!` (`:68`) for a real `MPI.Comm` (the package extension, loaded with MPI.jl);
  * every `pool.<field>` the programs read is a field or property of our `MPIAsyncPool`
    (`src/MPIAsyncPools.jl:24-34`), every keyword they pass to `asyncmap!` is accepted, and
    no name the programs define at top level collides with one we export.

Reads /root/reference (CPU suite only; skipped where it is absent, e.g. the GPU box).
"""
import os
import re

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "julia", "MPIAsyncPools")
REF = "/root/reference"
PROGRAMS = ["test/kmap1.jl", "test/kmap2.jl", "test/runtests.jl", "examples/iterative_example.jl"]

needs_ref = pytest.mark.skipif(not os.path.isdir(REF), reason="reference tree absent")


def _read(*p):
    with open(os.path.join(*p)) as f:
        return f.read()


def _toml_field(text, key):
    m = re.search(r'^%s\s*=\s*"([^"]*)"' % key, text, re.M)
    return m.group(1) if m else None


def _strip_comments(src):
    src = re.sub(r"#=.*?=#", "", src, flags=re.S)
    return "\n".join(line.split("#", 1)[0] for line in src.splitlines())


def _exports(src):
    """Names of every `export` statement (continued while a line ends in a comma)."""
    names, cont = [], False
    for line in _strip_comments(src).splitlines():
        s = line.strip()
        if s.startswith("export ") or cont:
            s = s[len("export "):] if s.startswith("export ") else s
            names += [n.strip() for n in s.split(",") if n.strip()]
            cont = s.endswith(",")
    return names


def _module_src():
    return _read(PKG, "src", "MPIAsyncPools.jl")


def _ext_src():
    return _read(PKG, "ext", "MPIAsyncPoolsMPIExt.jl")


def test_package_layout_and_extension():
    proj = _read(PKG, "Project.toml")
    assert _toml_field(proj, "name") == "MPIAsyncPools"
    assert re.search(r"^module MPIAsyncPools$", _module_src(), re.M)
    # the MPI.Comm methods live in a weak-dependency extension that loads with MPI.jl
    assert re.search(r'^MPIAsyncPoolsMPIExt\s*=\s*"MPI"', proj, re.M)
    ext = _ext_src()
    assert re.search(r"^module MPIAsyncPoolsMPIExt$", ext, re.M)
    assert "using MPIAsyncPools" in ext
    assert re.search(r"Base\.asyncmap!\(pool::MPIAsyncPool,[^)]*comm::MPI\.Comm;\s*kwargs\.\.\.\)", ext)
    assert re.search(r"waitall!|asyncmap!", ext)


@needs_ref
def test_package_identity_is_the_reference():
    ref, ours = _read(REF, "Project.toml"), _read(PKG, "Project.toml")
    assert _toml_field(ours, "name") == _toml_field(ref, "name") == "MPIAsyncPools"
    assert _toml_field(ours, "uuid") == _toml_field(ref, "uuid")
    # the reference's compat bounds a dependent may hold ("0.1"): same minor series
    assert _toml_field(ours, "version").split(".")[:2] == _toml_field(ref, "version").split(".")[:2]


@needs_ref
def test_reference_programs_load_this_package():
    for p in PROGRAMS:
        src = _read(REF, p)
        assert re.search(r"^using (MPI, )?MPIAsyncPools$", src, re.M), p


@needs_ref
def test_exports_cover_the_reference():
    ours = set(_exports(_module_src()))
    ref = set(_exports(_read(REF, "src", "MPIAsyncPools.jl")))
    assert ref and ref <= ours, ref - ours
    # asyncmap! is Base's, extended (src/MPIAsyncPools.jl:68), not exported
    assert "Base.asyncmap!" in _read(REF, "src", "MPIAsyncPools.jl")
    assert re.search(r"^function Base\.asyncmap!\(pool::MPIAsyncPool,", _module_src(), re.M)


def _pool_properties(src):
    """Fields of `mutable struct MPIAsyncPool` plus the properties its getproperty adds."""
    m = re.search(r"mutable struct MPIAsyncPool\n(.*?)\nend", src, re.S)
    fields = set(re.findall(r"^\s*(\w+)::", m.group(1), re.M))
    gp = re.search(r"function Base\.getproperty\(p::MPIAsyncPool.*?\nend", src, re.S)
    fields |= set(re.findall(r"s === :(\w+)", gp.group(0)))
    return fields


def _asyncmap_keywords(src):
    m = re.search(r"function Base\.asyncmap!\(pool::MPIAsyncPool,[^;]*;(.*?)\)\n", src, re.S)
    return set(re.findall(r"(\w+)(?:::(?:[^=,{}]|\{[^}]*\})+)?=", m.group(1)))


@needs_ref
def test_fields_and_keywords_the_programs_use():
    props = _pool_properties(_module_src())
    kws = _asyncmap_keywords(_module_src())
    assert {"nwait", "epoch", "tag"} <= kws
    used_fields, used_kws = set(), set()
    for p in PROGRAMS:
        src = _strip_comments(_read(REF, p))
        used_fields |= set(re.findall(r"\bpool\.(\w+)", src))
        for call in re.findall(r"asyncmap!\([^;()]*;([^)]*)\)", src):
            for kw in call.split(","):
                used_kws.add(kw.split("=")[0].strip())
    assert used_fields >= {"ranks", "active", "latency", "epoch"}, used_fields
    assert used_fields <= props, used_fields - props
    assert used_kws and used_kws <= kws, used_kws - kws


@needs_ref
def test_no_export_collides_with_program_globals():
    ours = set(_exports(_module_src()))
    for p in PROGRAMS:
        src = _strip_comments(_read(REF, p))
        defined = set(re.findall(r"^const (\w+)", src, re.M))
        defined |= set(re.findall(r"^function (\w+!?)\(", src, re.M))
        defined |= set(re.findall(r"^(\w+!?)\([^)]*\)\s*=", src, re.M))
        assert not (defined & ours), (p, defined & ours)
