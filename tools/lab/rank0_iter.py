"""Lab: from a kernel trace of bench.configs4_rank0_of_8 (XFK_LAB_WINDOW=1 prints
the timed replay's window), the last timed solve: its setup kernels (time,
gaps) and one PCG iteration in launch order (between two k_cg_axpy)."""
import csv
import re
import sys
from collections import defaultdict

rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
win = None
for ln in open(sys.argv[2]):
    m = re.search(r"\[window\] rank0 replay (\d+) (\d+)", ln)
    if m:
        win = (int(m.group(1)), int(m.group(2)))
seg = [r for r in rows if win is None or win[0] <= int(r["Start_Timestamp"]) <= win[1]]
starts = [i for i, r in enumerate(seg) if r["Kernel_Name"].startswith("k_n2e_tile")][::2]
a = starts[-1]
seg = seg[a:]
t0 = int(seg[0]["Start_Timestamp"])
axpy = [i for i, r in enumerate(seg) if r["Kernel_Name"].startswith("k_cg_axpy")]
print("last timed solve: %d kernels, span %.1f us, PCG starts at %.1f us, %d iterations" % (
    len(seg), (int(seg[-1]["End_Timestamp"]) - t0) / 1e3, (int(seg[axpy[0]]["Start_Timestamp"]) - t0) / 1e3, len(axpy)))
by = defaultdict(lambda: [0, 0.0, 0.0])
pe = t0
for r in seg[:axpy[0]]:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    k = r["Kernel_Name"].split("(")[0][:50]
    by[k][0] += 1
    by[k][1] += (e - s) / 1e3
    by[k][2] += max(0, s - pe) / 1e3
    pe = max(pe, e)
print("setup + symbolic + assembly by kernel (calls, busy us, gaps before us):")
for k, v in sorted(by.items(), key=lambda kv: -(kv[1][1] + kv[1][2]))[:30]:
    print("  %-50s %4d %9.1f %9.1f" % (k, v[0], v[1], v[2]))
i0, i1 = axpy[len(axpy) // 2], axpy[len(axpy) // 2 + 1]
print("one PCG iteration (%d kernels, %.1f us):" % (i1 - i0, (int(seg[i1]["Start_Timestamp"]) - int(seg[i0]["Start_Timestamp"])) / 1e3))
pe = int(seg[i0]["Start_Timestamp"])
for r in seg[i0:i1]:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    print("  %7.1f %6.1f gap %5.1f  %s grid %s" % ((s - int(seg[i0]["Start_Timestamp"])) / 1e3, (e - s) / 1e3,
                                                max(0, s - pe) / 1e3, r["Kernel_Name"].split("(")[0][:48],
                                                r.get("Grid_Size_X", r.get("Grid_Size", ""))))
    pe = max(pe, e)
