"""Median per-pass lsqb kernel times per probe size from a rocprofv3 kernel trace."""
import csv
import glob
import statistics as st
import sys

d, sizes = sys.argv[1], [int(s) for s in sys.argv[2:]]
f = glob.glob(d + "/**/*kernel_trace.csv", recursive=True)[0]
k = [(r["Kernel_Name"], int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) for r in csv.DictReader(open(f))
     if "lsqb" in r["Kernel_Name"]]
for i, rows in enumerate(sizes):
    ch = k[i * 26:(i + 1) * 26][6:]
    gb = 8 * rows * 2048 * 2
    r1 = st.median([x for n, x in ch if "resid" in n])
    r2 = st.median([x for n, x in ch if "grad" in n])
    print("rows/worker %7d A %7.0f MiB  pass1 %8.1f us %5.0f GB/s  pass2 %8.1f us %5.0f GB/s" %
          (rows, gb / 2**20, r1 / 1e3, gb / r1, r2 / 1e3, gb / r2))
