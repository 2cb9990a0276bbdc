"""Summarise a rocprofv3 results .db (kernel name, calls, total/avg us)."""
import glob
import sqlite3
import sys

db = sys.argv[1]
if not db.endswith(".db"):
    db = glob.glob(db + "/**/*.db", recursive=True)[0]
c = sqlite3.connect(db)
cols = [r[1] for r in c.execute("pragma table_info(kernels)")]
name = "kernel_name" if "kernel_name" in cols else ("name" if "name" in cols else None)
rows = c.execute("select %s, count(*), sum(end-start), avg(end-start) from kernels group by %s order by 3 desc"
                 % (name, name)).fetchall()
tot = sum(r[2] for r in rows)
print("%-70s %8s %10s %9s %6s" % ("kernel", "calls", "total_us", "avg_us", "%"))
for r in rows[: int(sys.argv[2]) if len(sys.argv) > 2 else 40]:
    print("%-70s %8d %10.1f %9.2f %6.1f" % (r[0][:70], r[1], r[2] / 1e3, r[3] / 1e3, 100.0 * r[2] / tot))
print("total kernel time %.1f us" % (tot / 1e3))
