"""The oracle's state machine over a REAL MPI (MPICH) against its own virtual-clock traces.

oracle/mpi_replay.c runs orc_asyncmap / orc_waitall (the restatement of
src/MPIAsyncPools.jl:35-224) on rank 0 of an MPICH job whose ranks 1..n run test/kmap2.jl's
worker program, sleeping each task's scheduled duration.  On the golden schedules whose
completions are >= 4 ms apart (tests/golden/traces.json, `min_gap_ns`) the trace
(repochs, active, recvbuf after every call) must equal the virtual-clock trace: this pins the
oracle's transport model (Isend/Irecv!/Test!/Waitany!/Waitall!) against the MPI library
MPI.jl binds.  MPICH is outside the repository (this image's /opt/conda); the test is
skipped where it is absent (the GPU box)."""
import json
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ORACLE = os.path.join(ROOT, "oracle")
MPI_DIR = os.environ.get("MPI_DIR", "/opt/conda")
MPIEXEC = os.path.join(MPI_DIR, "bin", "mpiexec")
GOLD = json.load(open(os.path.join(ROOT, "tests", "golden", "traces.json")))["scenarios"]
SEPARATED = [s["name"] for s in GOLD if s.get("min_gap_ns", 0) >= 4_000_000]

pytestmark = pytest.mark.skipif(not (os.path.exists(os.path.join(MPI_DIR, "include", "mpi.h")) and
                                     os.path.exists(MPIEXEC)), reason="MPICH not present")


@pytest.fixture(scope="module")
def replay_bin():
    subprocess.check_call(["make", "-s", "-C", ORACLE, "mpi", f"MPI_DIR={MPI_DIR}"])
    return os.path.join(ORACLE, "_build", "mpi_replay")


def scenario_text(sc):
    n = sc["n"]
    dur = sc["durations_ns"]
    nc = len(dur) // n
    lines = [f"{n} {nc} {len(sc['ops'])}"]
    lines += [" ".join(str(x) for x in dur[w * nc:(w + 1) * nc]) for w in range(n)]
    for op in sc["ops"]:
        if op["op"] == "waitall":
            lines.append("W")
            continue
        assert "epoch" not in op and "advance_ns" not in op
        nw = op["nwait"]
        if isinstance(nw, str):
            k = int(nw.rsplit("_", 1)[1])
            lines.append(("F" if nw.startswith("first_plus_") else "C") + f" {k} {op['send']}")
        else:
            lines.append(f"A {nw} {op['send']}")
    return "\n".join(lines) + "\n"


def _replay(replay_bin, path, sc):
    """(mismatches, stderr) of one MPICH run of the scenario against its virtual-clock trace."""
    env = dict(os.environ, HYDRA_LAUNCHER="fork")
    # durations x10: the same trace (order depends only on sums of durations), gaps >= 40 ms;
    # x16 when the job has more ranks than the host has CPUs (MPICH ranks busy-poll, so an
    # oversubscribed rank can miss its wake-up by a scheduler time slice)
    scale = "16" if sc["n"] + 1 > (os.cpu_count() or 1) else "10"
    out = subprocess.run([MPIEXEC, "-n", str(sc["n"] + 1), replay_bin, str(path), scale], capture_output=True, text=True,
                         timeout=240, env=env)
    assert out.returncode == 0, out.stderr[-2000:]
    lines = [ln for ln in out.stdout.splitlines() if "|" in ln]
    bad = [] if len(lines) == len(sc["results"]) else [("records", len(lines), len(sc["results"]))]
    for k, (ln, ref) in enumerate(zip(lines, sc["results"])):
        rep, act, rec = ln.split("|")
        if ([int(v) for v in rep.split()] != ref["repochs"] or [int(v) for v in act.split()] != ref["active"]
                or [float(v) for v in rec.split()] != ref["recv"]):
            bad.append((k, ln))
    return bad


@pytest.mark.parametrize("name", SEPARATED)
def test_mpi_replay_matches_virtual_clock_trace(replay_bin, tmp_path, name):
    """A run whose physical completions crossed (a rank descheduled past a >= 40 ms gap on an
    oversubscribed host) is repeated once; the trace must match in that run."""
    sc = next(s for s in GOLD if s["name"] == name)
    f = tmp_path / "scenario.txt"
    f.write_text(scenario_text(sc))
    bad = _replay(replay_bin, f, sc)
    if bad:
        print("%s: run 1 diverged at %s; repeating" % (name, bad[:2]))
        bad = _replay(replay_bin, f, sc)
    assert bad == [], (name, bad[:3])
