"""Print the kernel timeline (duration, gap to the previous kernel) of the
k-th occurrence of a phase in a rocprofv3 kernel-trace CSV.

usage: python tools/lab/timeline.py TRACE.csv START_KERNEL END_KERNEL [OCCURRENCE]
"""
import csv, sys

path, start, end = sys.argv[1:4]
occ = int(sys.argv[4]) if len(sys.argv) > 4 else 1
rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
idx = [i for i, r in enumerate(rows) if r["Kernel_Name"].startswith(start)]
i0 = idx[occ]
t0 = int(rows[i0]["Start_Timestamp"])
prev = None
busy = 0.0
for r in rows[i0:]:
    if r is not rows[i0] and r["Kernel_Name"].startswith(end):
        print("phase wall %.1f us, kernels busy %.1f us" % ((int(r["Start_Timestamp"]) - t0) / 1e3, busy))
        break
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    busy += (e - s) / 1e3
    print("%8.1f us  dur %7.1f  gap %7.1f  %s" % ((s - t0) / 1e3, (e - s) / 1e3,
                                               (s - prev) / 1e3 if prev else 0.0, r["Kernel_Name"][:60]))
    prev = e
