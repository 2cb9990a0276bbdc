"""Per-Newton-pass timeline of the last nonlinear solve in a rocprofv3 kernel
trace: each pass runs from one k_assemble_rows to the next; prints the pass
span, kernel-busy time, idle time, the long idle gaps (host checks) with the
kernel before them, and the per-kernel totals of the pass.
usage: python tools/lab/newton_tl.py TRACE.csv PASSES [SOLVE_FROM_END (1: the last)]
(bench.py's last two solves are its cold first solves: the timed step is 3)"""
import csv, sys
from collections import defaultdict

rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
npass = int(sys.argv[2])
asm = [i for i, r in enumerate(rows) if r['Kernel_Name'].startswith('k_assemble_rows')]
back = int(sys.argv[3]) if len(sys.argv) > 3 else 1
starts = asm[len(asm) - back * npass:len(asm) - (back - 1) * npass]
nxt = len(asm) - (back - 1) * npass
ends = starts[1:] + [asm[nxt] if nxt < len(asm) else len(rows)]
grand = defaultdict(float)
for p, (a, b) in enumerate(zip(starts, ends)):
    seg = rows[a:b]
    nr = [k for k, r in enumerate(seg) if r['Kernel_Name'].startswith('k_newton_res')]
    if nr:   # (the pass ends with its Newton residual)
        seg = seg[:nr[0] + 1]
    t0 = int(seg[0]['Start_Timestamp'])
    t1 = max(int(r['End_Timestamp']) for r in seg)
    busy = 0.0
    prev = t0
    gaps = []
    agg = defaultdict(float)
    cnt = defaultdict(int)
    last = ''
    for r in seg:
        s, e = int(r['Start_Timestamp']), int(r['End_Timestamp'])
        if s > prev:
            g = (s - prev) / 1e3
            if g > 15:
                gaps.append((g, last, r['Kernel_Name'][:40], (s - t0) / 1e3))
        busy += max(0, e - max(s, prev)) / 1e3
        prev = max(prev, e)
        name = r['Kernel_Name'][:40]
        agg[name] += (e - s) / 1e3
        cnt[name] += 1
        grand[name] += (e - s) / 1e3
        last = name
    span = (t1 - t0) / 1e3
    print("pass %d: span %.1f us, busy %.1f, idle %.1f, launches %d, cg_axpy %d" %
          (p, span, busy, span - busy, len(seg), cnt.get('k_cg_axpy', 0)))
    for g, before, after, at in gaps:
        print("    gap %7.1f us at %8.1f after %-40s before %s" % (g, at, before, after))
    for k, v in sorted(agg.items(), key=lambda x: -x[1])[:14]:
        print("    %8.1f %4d %s" % (v, cnt[k], k))
print("all passes, per kernel:")
for k, v in sorted(grand.items(), key=lambda x: -x[1])[:30]:
    print("%9.1f %s" % (v, k))
