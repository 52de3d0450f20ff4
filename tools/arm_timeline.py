"""Merged host / kernel timeline of a two-process run (measurement build, round 6): the host event
stamps (MPA_HOST_STAMP=<dir>, hip_transport.hpp) and the rocprofv3 kernel traces of the same run,
both on CLOCK_MONOTONIC.

    python tools/arm_timeline.py <stamp dir> <trace dir> <bench JSON line file> [--last N]

Host events: D armed task's completion seen by its server (rank, seq); W / L its next door_wait /
task enqueued by arm(); B a doorbell seen by the serve loop (host-launched path); T that task
launched; R rank 0's wait returned for (rank, seq); A rank 0's launch-ahead enqueued.
Prints the last N events, then per-event-pair median gaps of the server's armed cycle."""
import argparse
import csv
import glob
import json
import os
import statistics as st


def main():
    p = argparse.ArgumentParser()
    p.add_argument("stamps")
    p.add_argument("traces")
    p.add_argument("bench_json")
    p.add_argument("--last", type=int, default=80)
    a = p.parse_args()
    pids = json.load(open(a.bench_json))["rank_pids"]
    ev = []
    for r, pid in enumerate(pids):
        f = os.path.join(a.stamps, "%d.txt" % pid)
        if os.path.exists(f):
            for line in open(f):
                k, x, y, t = line.split()
                ev.append((int(t), r, "host %s %s %s" % (k, x, y), k))
    for f in glob.glob(os.path.join(a.traces, "**", "*kernel_trace.csv"), recursive=True):
        pid = int(os.path.basename(f).split("_")[0])
        if pid not in pids:
            continue
        r = pids.index(pid)
        for row in csv.DictReader(open(f)):
            name = row["Kernel_Name"].replace("void mpa::(anonymous namespace)::", "").replace("mpa::", "")[:18]
            ev.append((int(row["Start_Timestamp"]), r, "start " + name, "s" + name[:3]))
            ev.append((int(row["End_Timestamp"]), r, "end   " + name, "e" + name[:3]))
    ev.sort()
    tail = ev[-a.last - 40:-40]
    t0 = tail[0][0]
    prev = t0
    for t, r, what, _ in tail:
        print("%9.2f %+8.2f  r%d %s" % ((t - t0) / 1e3, (t - prev) / 1e3, r, what))
        prev = t
    # rank 1's armed cycle: D (done seen) -> W -> L, door_wait start / end, lsq start / end
    seq = [(t, k) for t, r, _, k in ev if r == 1]
    pairs = {}
    for (t1, k1), (t2, k2) in zip(seq, seq[1:]):
        pairs.setdefault(k1 + "->" + k2, []).append(t2 - t1)
    print("rank 1 consecutive event gaps (us): median, count")
    for k, v in sorted(pairs.items(), key=lambda kv: -len(kv[1]))[:14]:
        print("  %-16s %8.2f %6d" % (k, st.median(v) / 1e3, len(v)))
    seq = [(t, k) for t, r, _, k in ev if r == 0]
    pairs = {}
    for (t1, k1), (t2, k2) in zip(seq, seq[1:]):
        pairs.setdefault(k1 + "->" + k2, []).append(t2 - t1)
    print("rank 0 consecutive event gaps (us): median, count")
    for k, v in sorted(pairs.items(), key=lambda kv: -len(kv[1]))[:14]:
        print("  %-16s %8.2f %6d" % (k, st.median(v) / 1e3, len(v)))


if __name__ == "__main__":
    main()
