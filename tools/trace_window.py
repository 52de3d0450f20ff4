"""Average duration of a kernel over the timed region of a bench run traced by
`rocprofv3 --kernel-trace --stats`: the last N launches of the kernel in the trace, N = the
`roofline.launches` of the bench line that run printed, before the `launches_after_timed`
ones that follow the timed region (the c5 bench's waitall releases a held 1-task re-dispatch
after it); the warm-up launches before the timed region are dropped, and the c5 bench mixes
8-, 7- and 1-task launches, so an all-launch average of the --stats summary is not comparable
with the timed-region figure.

    python tools/trace_window.py --trace DIR/c5_kernel_trace.csv --bench-log DIR/../c5_trace.log \
        --kernel lsqp4_kernel --out profiles/r02_c5_rocprof_window.json
"""
import argparse
import csv
import json
import time


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--trace", required=True)
    p.add_argument("--bench-log", required=True, help="stdout of the traced bench run (its JSON line)")
    p.add_argument("--kernel", required=True)
    p.add_argument("--out", required=True)
    p.add_argument("--tail", type=int, default=None,
                   help="launches after the timed region, for bench lines older than launches_after_timed")
    a = p.parse_args()
    line = [ln for ln in open(a.bench_log) if ln.startswith("{")][-1]
    bench = json.loads(line)
    # every launch of the timed region (launches_total), not only the ones the bench timed
    n = int(bench["roofline"].get("launches_total") or bench["roofline"]["launches"])
    rows = [r for r in csv.DictReader(open(a.trace)) if a.kernel in r["Kernel_Name"]]
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    tail = a.tail if a.tail is not None else int(bench.get("launches_after_timed", 0))
    ms = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6 for r in rows]
    ms = ms[len(ms) - tail - n:len(ms) - tail]
    out = {
        "kernel": a.kernel,
        "launches": len(ms),
        "avg_ms": sum(ms) / len(ms),
        "sum_ms": sum(ms),
        "bench_avg_launch_ms_same_run": bench["roofline"]["avg_launch_ms"],
        "bench_steps": bench["steps"],
        "launches_after_timed": tail,
        "source": "rocprofv3 --kernel-trace of bench.py (the `launches` dispatches before the last "
                  "`launches_after_timed` = the timed region)",
        "date": time.strftime("%Y-%m-%d"),
    }
    with open(a.out, "w") as fh:
        json.dump(out, fh, indent=1)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
