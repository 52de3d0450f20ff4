"""Diagnose the ~20 ms latency outliers of the gated kmap2_n9 replay.

Runs the golden scenario kmap2_n9 under the gate several times in ONE process, first with
only the streams it needs, then after a 16-worker comm has grown the process-wide stream
pool (more HSA queues alive), and prints per run: the process's KFD queue count (when
/sys exposes it), the latency deviation from the oracle (median / max / count > 1 ms), the
timer thread's worst lateness against a due time and its worst launch-call duration.
Usage (GPU box): python tools/diag_gated_stall.py [reps] [scenario ...]
  --grow=N  (named scenarios) a N-worker comm fills the process's stream pool first
  --stream  run the replays under a non-blocking torch stream (the coordinator's copies and the
            harness's tensor ops off the legacy NULL stream, which orders against every blocking
            worker stream)
A watchdog process (same cgroup) sleeps 0.5 ms at a time and reports its worst oversleep per run:
a host-wide stall (CPU throttling, descheduling) shows there as well as in the latencies.
"""
import multiprocessing as mp
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (os.path.join(ROOT, "mpistragglers.jl_amd"), os.path.join(ROOT, "tests"), os.path.join(ROOT, "oracle")):
    sys.path.insert(0, p)

import torch  # noqa: E402

import gated  # noqa: E402
import mpiasyncpools as M  # noqa: E402


def kfd_queues():
    d = "/sys/class/kfd/kfd/proc/%d/queues" % os.getpid()
    try:
        return len(os.listdir(d))
    except OSError:
        return -1


def watchdog(conn):
    """Sleep 0.5 ms at a time; on each request reply (worst oversleep ms, count > 2 ms) since the last."""
    worst, over = 0.0, 0
    while True:
        if conn.poll():
            if conn.recv() is None:
                return
            conn.send((worst, over))
            worst, over = 0.0, 0
        t0 = time.perf_counter()
        time.sleep(0.0005)
        d = (time.perf_counter() - t0 - 0.0005) * 1e3
        worst = max(worst, d)
        over += d > 2.0


WD = None


def run(sc):
    if WD is not None:
        WD.send(1)
        WD.recv()
    _, sched = gated.oracle_gate(sc)
    n = sc["n"]
    dur = np.asarray(sc["durations_ns"], dtype=np.int64).reshape(n, -1)
    comm = M.DeviceComm(n)
    for r in range(1, n + 1):
        comm.set_task(r, "kmap2")
        comm.set_delays(r, dur[r - 1])
    comm.set_gate(*sched)

    def buf(k):
        return torch.zeros(k, dtype=torch.float64, device="cuda")
    t0 = time.time()
    if STREAM:
        with torch.cuda.stream(torch.cuda.Stream()):
            got, pool = gated.replay(M, sc, comm, buf, lambda t: t.cpu().numpy(), gated.make_golden().predicate,
                                     snap=lambda t: t.clone())
            torch.cuda.current_stream().synchronize()
    else:
        got, pool = gated.replay(M, sc, comm, buf, lambda t: t.cpu().numpy(), gated.make_golden().predicate,
                                 snap=lambda t: t.clone())
    wall = time.time() - t0
    wd = (-1.0, -1)
    if WD is not None:
        WD.send(1)
        wd = WD.recv()
    q = kfd_queues()
    c = {k: comm.counter(k) for k in ("sleeps", "timer_late", "queues", "shared_worker_streams")}
    comm.shutdown()
    comm.close()
    bad = gated.mismatches(sc["name"], got, sc["results"])
    tol = gated.latency_tolerance(sc)
    dev, where = [], []
    for k, (g, r) in enumerate(zip(got, sc["results"])):
        for i, (v, lat) in enumerate(zip(g["latency_s"], r["latency_ns"])):
            if lat > 0:
                dev.append(abs(v - lat / 1e9))
                where.append((k, i))
    dev = np.asarray(dev)
    big = [(where[j], round(1e3 * dev[j], 2)) for j in np.argsort(dev)[::-1][:4] if dev[j] > 0.5e-3]
    over = [(where[j], round(1e3 * dev[j], 2), round(1e3 * tol[where[j]], 2)) for j in range(len(dev)) if dev[j] > tol[where[j]]]
    print("    beyond tolerance: %d %s" % (len(over), over[:5]))
    for j in np.argsort(dev)[::-1][:3]:
        k, i = where[j]
        print("    op %d %s worker %d: oracle %.3f ms device %.3f ms" % (
            k, sc["ops"][k], i, sc["results"][k]["latency_ns"][i] / 1e6, 1e3 * got[k]["latency_s"][i]))
    print("  kfd_queues %d  mismatches %d  wall %.1f s  latency dev median %.3f ms max %.3f ms  >1ms %d  worst %s  %s"
          "  watchdog worst oversleep %.2f ms, %d > 2 ms%s"
          % (q, len(bad), wall, 1e3 * np.median(dev), 1e3 * dev.max(), int((dev > 1e-3).sum()), big, c, wd[0], wd[1],
             "  [non-blocking stream]" if STREAM else ""), flush=True)


STREAM = False


def main():
    global STREAM, WD
    args = [a for a in sys.argv[1:] if not a.startswith("--")]
    STREAM = "--stream" in sys.argv
    parent, child = mp.Pipe()
    proc = mp.get_context("spawn").Process(target=watchdog, args=(child,), daemon=True)
    proc.start()
    WD = parent
    reps = int(args[0]) if args else 4
    grow = next((int(a.split("=")[1]) for a in sys.argv[1:] if a.startswith("--grow=")), 0)
    if len(args) > 1:  # named scenarios only, fresh process (--grow=N: a N-worker comm fills the pool first)
        torch.zeros(1, device="cuda")
        if grow:
            big = M.DeviceComm(grow)
            for r in range(1, grow + 1):
                big.set_task(r, "kmap2")
            big.close()
        for name in args[1:]:
            sc = next(s for s in gated.scenarios() if s["name"] == name)
            print("== %s" % name, flush=True)
            for _ in range(reps):
                run(sc)
        return
    torch.cuda.init()
    torch.zeros(1, device="cuda")
    sc = next(s for s in gated.scenarios() if s["name"] == "kmap2_n9")
    print("== kmap2_n9, fresh process (queues %d)" % kfd_queues(), flush=True)
    for _ in range(reps):
        run(sc)
    for grow in (16, 24):
        big = M.DeviceComm(grow)
        for r in range(1, grow + 1):
            big.set_task(r, "kmap2")
        big.close()
        print("== after a %d-worker comm grew the stream pool (queues %d)" % (grow, kfd_queues()), flush=True)
        for _ in range(reps):
            run(sc)


if __name__ == "__main__":
    main()
