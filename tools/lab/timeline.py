"""Lab: a window of a rocprofv3 kernel trace in time order (start, duration, gap
to the previous kernel's end, queue, name, grid) -- tools/lab/timeline.py
TRACE.csv[.gz] ERR.log TAG [first-line last-line]"""
import csv
import gzip
import sys

path, err, tag = sys.argv[1:4]
op = gzip.open if path.endswith(".gz") else open
rows = list(csv.DictReader(op(path, "rt")))
w = [ln.split() for ln in open(err) if ln.startswith("[window] %s " % tag)][0]
a, b = int(w[2]), int(w[3])
ks = sorted((r for r in rows if int(r["Start_Timestamp"]) >= a and int(r["End_Timestamp"]) <= b),
            key=lambda r: int(r["Start_Timestamp"]))
t0 = int(ks[0]["Start_Timestamp"])
prev = t0
lo, hi = (int(sys.argv[4]), int(sys.argv[5])) if len(sys.argv) > 5 else (0, len(ks))
for i, r in enumerate(ks):
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    if lo <= i < hi:
        print("%4d %8.1f %6.1f gap%7.1f q%s %-40s grid %s" % (i, (s - t0) / 1e3, (e - s) / 1e3, (s - prev) / 1e3,
                                                          r["Queue_Id"], r["Kernel_Name"][:40], r["Grid_Size_X"]))
    prev = max(prev, e)
