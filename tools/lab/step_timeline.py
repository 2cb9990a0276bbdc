"""One bench step from a rocprofv3 kernel trace: the solves are cut at the
symbolic phase's first kernel (k_n2e_tile); for the last timed step, the
kernels in order with start offset, duration and the gap before each
(idle device time between dependent launches), plus totals per phase
(setup = before the first k_cg_axpy, iterations after)."""
import csv
import sys
from collections import defaultdict

rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
starts = [i for i, r in enumerate(rows) if r["Kernel_Name"].startswith("k_n2e_tile")]
# k_n2e_tile runs twice per symbolic phase (count, fill): a solve starts at every other one
solve_starts = starts[::2]
which = int(sys.argv[2]) if len(sys.argv) > 2 else 3
a = solve_starts[which]
b = solve_starts[which + 1] if which + 1 < len(solve_starts) else len(rows)
seg = rows[a:b]
t0 = int(seg[0]["Start_Timestamp"])
prev_end = t0
busy = gap = 0
by = defaultdict(lambda: [0, 0.0, 0.0])
first_axpy = next((i for i, r in enumerate(seg) if r["Kernel_Name"].startswith("k_cg_axpy")), len(seg))
phase_busy = [0.0, 0.0]
phase_gap = [0.0, 0.0]
for i, r in enumerate(seg):
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    g = max(0, s - prev_end)
    d = e - s
    ph = 0 if i < first_axpy else 1
    phase_busy[ph] += d
    phase_gap[ph] += g
    busy += d
    gap += g
    k = r["Kernel_Name"].split("(")[0][:40]
    by[k][0] += 1
    by[k][1] += d / 1e3
    by[k][2] += g / 1e3
    if len(sys.argv) > 3:
        print("%9.1f %7.1f gap %6.1f  %s" % ((s - t0) / 1e3, d / 1e3, g / 1e3, k))
    prev_end = max(prev_end, e)
print("solve %d: %d kernels, span %.1f us, busy %.1f us, gaps %.1f us" % (which, len(seg), (prev_end - t0) / 1e3,
                                                                           busy / 1e3, gap / 1e3))
print("setup+symbolic: busy %.1f gaps %.1f | iterations: busy %.1f gaps %.1f (us)" % (
    phase_busy[0] / 1e3, phase_gap[0] / 1e3, phase_busy[1] / 1e3, phase_gap[1] / 1e3))
for k, (n, d, g) in sorted(by.items(), key=lambda kv: -(kv[1][1] + kv[1][2]))[:40]:
    print("%-40s %4d  busy %8.1f  gaps-before %8.1f" % (k, n, d, g))
