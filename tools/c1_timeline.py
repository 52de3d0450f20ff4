"""c1 epoch timeline from a rocprofv3 --kernel-trace CSV: per epoch the coordinator's
epoch_kernel and the workers' lsq_grad_kernel; medians of their durations and of the gaps
between them (epoch end -> task start: launch latency; task end -> next epoch start: the
host noticing the replies and launching the next epoch)."""
import csv
import statistics as st
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
n = int(sys.argv[2]) if len(sys.argv) > 2 else 3000
ks = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), "epoch" if "epoch_kernel" in r["Kernel_Name"] else "lsq")
            for r in rows if "epoch_kernel" in r["Kernel_Name"] or "lsq_grad_kernel" in r["Kernel_Name"])
ks = ks[-2 * n:]
dur, gap = {}, {}
for i, k in enumerate(ks):
    dur.setdefault(k[2], []).append((k[1] - k[0]) / 1e3)
    if i:
        gap.setdefault(ks[i - 1][2] + "->" + k[2], []).append((k[0] - ks[i - 1][1]) / 1e3)
for k, v in sorted(dur.items()):
    print("%-6s duration  n %5d median %7.2f us mean %7.2f us" % (k, len(v), st.median(v), st.mean(v)))
for k, v in sorted(gap.items()):
    print("%-12s gap n %5d median %7.2f us mean %7.2f us" % (k, len(v), st.median(v), st.mean(v)))
print("epoch period %.2f us (last %d epochs)" % ((ks[-1][0] - ks[0][0]) / 1e3 / (len(ks) / 2), len(ks) // 2))
