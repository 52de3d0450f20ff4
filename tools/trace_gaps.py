"""Per-epoch timeline of the coordinator loop from a rocprofv3 --kernel-trace CSV.

    python tools/trace_gaps.py <dir with *_kernel_trace.csv> [--anchor lsq_grad_kernel]

For every anchor-kernel dispatch (one per epoch) it reports the gaps on the GPU timeline
between the end of one epoch's anchor kernel and the start of the next, broken down by the
kernels that ran in between (aggregate / exchange), as medians over the trace.  This is
where the non-kernel part of ms_per_step goes.
"""
import argparse
import csv
import glob
import json
import os
import statistics as st


def load(d):
    rows = []
    for f in glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True):
        with open(f) as fh:
            for r in csv.DictReader(fh):
                rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"],
                             r.get("Queue_Id", "")))
    rows.sort()
    return rows


def short(name):
    for k in ("lsqb_resid_kernel", "lsqb_grad_kernel", "lsq_grad_kernel", "exchange_kernel", "aggregate_kernel",
              "kmap_task_kernel", "generate_kernel"):
        if k in name:
            return k
    return name[:40]


def main():
    p = argparse.ArgumentParser()
    p.add_argument("dir")
    p.add_argument("--anchor", default="lsq_grad_kernel")
    p.add_argument("--skip", type=int, default=50, help="epochs to skip (warmup)")
    a = p.parse_args()
    rows = [(s, e, short(n), q) for s, e, n, q in load(a.dir)]
    anchors = [i for i, r in enumerate(rows) if r[2] == a.anchor][a.skip:]
    gaps, kdur, between = [], [], {}
    for x, y in zip(anchors, anchors[1:]):
        s0, e0 = rows[x][0], rows[x][1]
        s1 = rows[y][0]
        kdur.append(e0 - s0)
        gaps.append(s1 - e0)
        for s, e, n, q in rows[x + 1:y]:
            between.setdefault(n, []).append((s - e0, e - s))
    out = {"epochs": len(gaps), "anchor": a.anchor,
           "anchor_us_median": st.median(kdur) / 1e3 if kdur else None,
           "gap_us_median": st.median(gaps) / 1e3 if gaps else None,
           "between": {n: {"count_per_epoch": len(v) / max(1, len(gaps)),
                           "start_after_anchor_end_us_median": st.median(t for t, _ in v) / 1e3,
                           "duration_us_median": st.median(d for _, d in v) / 1e3} for n, v in between.items()}}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
