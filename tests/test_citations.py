"""Every `file:line` citation of the reference in the product, the oracle, the tests and the
docs points at a line that exists in the reference tree (VERDICT r01 "What's weak" #8: the
test/kmap2.jl citations were offset by +34).  Skipped where /root/reference is absent (the
GPU box); the reference is read as text only.
"""
import os
import re

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
REF = "/root/reference"

# basename (as cited) -> path in the reference tree
REF_FILES = {
    "MPIAsyncPools.jl": "src/MPIAsyncPools.jl",
    "kmap1.jl": "test/kmap1.jl",
    "kmap2.jl": "test/kmap2.jl",
    "runtests.jl": "test/runtests.jl",
    "iterative_example.jl": "examples/iterative_example.jl",
}
CITE = re.compile(r"(?<![\w/])(?:src/|test/|examples/)?(MPIAsyncPools\.jl|kmap1\.jl|kmap2\.jl|runtests\.jl|"
                  r"iterative_example\.jl):(\d+(?:-\d+)?(?:,\d+(?:-\d+)?)*)")
SCAN_DIRS = ["include", "oracle", "tests", "julia", os.path.join("mpistragglers.jl_amd", "csrc"),
             os.path.join("mpistragglers.jl_amd", "mpiasyncpools")]
SCAN_FILES = ["DESIGN.md", "INTEGRATION.md", "bench.py", "__graft_entry__.py", "README.md"]
EXTS = (".py", ".c", ".h", ".cpp", ".hpp", ".hip", ".md", ".jl", ".toml")


def _sources():
    for d in SCAN_DIRS:
        top = os.path.join(ROOT, d)
        for dirpath, dirnames, files in os.walk(top):
            dirnames[:] = [x for x in dirnames if not x.startswith(("_", "."))]
            for f in files:
                if f.endswith(EXTS) and f != os.path.basename(__file__):
                    yield os.path.join(dirpath, f)
    for f in SCAN_FILES:
        p = os.path.join(ROOT, f)
        if os.path.exists(p):
            yield p


def _citations():
    out = []
    for path in _sources():
        with open(path, errors="replace") as fh:
            for ln, text in enumerate(fh, 1):
                for m in CITE.finditer(text):
                    for part in m.group(2).split(","):
                        a, _, b = part.partition("-")
                        out.append((os.path.relpath(path, ROOT), ln, m.group(1), int(a), int(b) if b else int(a)))
    return out


def test_citation_scanner_finds_citations():
    cites = _citations()
    assert len(cites) > 50
    assert any(c[2] == "kmap2.jl" for c in cites)


@pytest.mark.skipif(not os.path.isdir(REF), reason="reference tree not mounted")
def test_every_cited_reference_line_exists():
    lengths = {}
    for base, rel in REF_FILES.items():
        with open(os.path.join(REF, rel), errors="replace") as fh:
            lengths[base] = sum(1 for _ in fh)
    bad = [c for c in _citations() if not (1 <= c[3] <= c[4] <= lengths[c[2]])]
    assert not bad, "citations past the end of the reference file: %s" % bad[:20]


@pytest.mark.skipif(not os.path.isdir(REF), reason="reference tree not mounted")
def test_kmap2_anchor_lines():
    """The kmap2.jl lines the code leans on hold what the citations say they hold."""
    with open(os.path.join(REF, "test/kmap2.jl")) as fh:
        lines = fh.read().splitlines()
    anchors = {14: "function shutdown", 22: "pool.ranks == collect", 50: "wepoch == repochs[i]",
               53: "from_this_epoch >= nwait", 60: "pool.active", 65: "repochs[1] == epoch",
               70: "repochs[1] == pool.epoch", 71: "pool.latency[1]", 76: "function worker_main",
               95: "sleep(max(rand()/10, 0.005))"}
    for ln, text in anchors.items():
        assert text in lines[ln - 1], (ln, lines[ln - 1])


@pytest.mark.skipif(not os.path.isdir(REF), reason="reference tree not mounted")
@pytest.mark.parametrize("rel,anchors", [
    ("src/MPIAsyncPools.jl", {68: "function Base.asyncmap!", 71: "nwait must be in the range", 87: "pool.epoch = epoch",
                              99: "MPI.Test!", 105: "pool.latency[i]", 130: "isendbufs[i] .=", 137: "MPI.Isend",
                              138: "MPI.Irecv!", 153: "nwait(pool.epoch, pool.repochs)", 161: "MPI.Waitany!",
                              174: "pool.repochs[i] == pool.epoch", 187: "return pool.repochs",
                              212: "MPI.Waitall!"}),
    ("examples/iterative_example.jl", {37: "for epoch in 1:10", 40: "asyncmap!", 42: "repochs[i] == epoch",
                                       51: "control_tag", 55: "function worker_main", 74: "sleep(rand())"}),
])
def test_core_anchor_lines(rel, anchors):
    with open(os.path.join(REF, rel)) as fh:
        lines = fh.read().splitlines()
    for ln, text in anchors.items():
        assert text in lines[ln - 1], (rel, ln, lines[ln - 1])
