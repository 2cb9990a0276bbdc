"""Lab: per-kernel totals of a rocprofv3 kernel trace inside a time window
printed by the traced program ("[window] <tag> <t0_ns> <t1_ns> solves <k>",
time.monotonic_ns, the trace's clock).  Also the busy time (union of kernel
intervals) and the gaps between consecutive kernels.
Usage: python tools/lab/trace_window.py TRACE.csv LOG [tag]"""
import csv
import re
import sys
from collections import defaultdict


def main():
    trace, log = sys.argv[1], sys.argv[2]
    tag = sys.argv[3] if len(sys.argv) > 3 else None
    win = None
    for line in open(log, errors="replace"):
        m = re.search(r"\[window\] (.+?) (\d+) (\d+) solves (\d+)", line)
        if m and (tag is None or m.group(1) == tag):
            win = (int(m.group(2)), int(m.group(3)), int(m.group(4)))
    if win is None:
        sys.exit("no [window] line in %s" % log)
    t0, t1, k = win
    rows = []
    with open(trace) as f:
        for r in csv.DictReader(f):
            s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
            if s >= t0 and e <= t1:
                rows.append((s, e, r["Kernel_Name"], int(r["Grid_Size_X"])))
    rows.sort()
    tot = defaultdict(lambda: [0, 0.0])
    busy, last_e, gaps = 0.0, None, 0.0
    for s, e, name, g in rows:
        short = name.split("(")[0][:90]
        tot[short][0] += 1
        tot[short][1] += (e - s) / 1e3
        if last_e is None or s >= last_e:
            busy += (e - s) / 1e3
            if last_e is not None:
                gaps += (s - last_e) / 1e3
            last_e = e
        elif e > last_e:
            busy += (e - last_e) / 1e3
            last_e = e
    span = (t1 - t0) / 1e3
    print("window %.1f us over %d solves: %d kernels, busy %.1f us, gaps %.1f us (per solve: %.1f / %.1f / %.1f)"
          % (span, k, len(rows), busy, gaps, span / k, busy / k, gaps / k))
    print("%8s %8s %9s  kernel" % ("calls/s", "us/call", "us/solve"))
    for name, (c, us) in sorted(tot.items(), key=lambda kv: -kv[1][1]):
        print("%8.1f %8.2f %9.1f  %s" % (c / k, us / c, us / k, name))


if __name__ == "__main__":
    main()
