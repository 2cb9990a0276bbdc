"""Per (kernel, grid size) breakdown of a rocprofv3 results .db or kernel_trace.csv."""
import collections
import csv
import glob
import sqlite3
import sys

src = sys.argv[1]
top = int(sys.argv[2]) if len(sys.argv) > 2 else 40
rows = []
if src.endswith(".csv"):
    for r in csv.DictReader(open(src)):
        rows.append((r["Kernel_Name"], int(r["Grid_Size_X"]), (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3))
else:
    db = src if src.endswith(".db") else glob.glob(src + "/**/*.db", recursive=True)[0]
    c = sqlite3.connect(db)
    rows = [(n, g, (e - s) / 1e3) for n, g, s, e in c.execute("select name, grid_x, start, end from kernels")]
agg = collections.defaultdict(lambda: [0, 0.0])
for nm, g, d in rows:
    short = nm.replace("void ", "").replace("(anonymous namespace)::", "").replace("xfk::", "")
    short = short.split("(")[0]
    agg[(short[:60], g)][0] += 1
    agg[(short[:60], g)][1] += d
tot = sum(v[1] for v in agg.values())
for (k, g), (n, t) in sorted(agg.items(), key=lambda kv: -kv[1][1])[:top]:
    print("%-60s grid %9d calls %5d avg %8.2f us total %9.1f (%4.1f%%)" % (k, g, n, t / n, t, 100 * t / tot))
print("total %.1f us" % tot)
