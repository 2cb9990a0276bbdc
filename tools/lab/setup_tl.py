"""Setup timeline of one solve from a rocprofv3 kernel trace: every kernel
between the end of k_assemble_rows and k_cg_init_r, with its gap to the
previous kernel, plus per-kernel totals.
usage: python tools/lab/setup_tl.py TRACE.csv [OCCURRENCE (default: the last hinted setup)] [--gaps]"""
import csv, sys
from collections import defaultdict

rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
asm = [i for i, r in enumerate(rows) if r['Kernel_Name'].startswith('k_assemble_rows')]
spans = []
for a in asm:
    j = a
    while j < len(rows) and not rows[j]['Kernel_Name'].startswith('k_cg_init_r'):
        j += 1
    hinted = not any(r['Kernel_Name'].startswith('k_spgemm_nprod') for r in rows[a:j])
    spans.append((a, j, hinted))
args = [x for x in sys.argv[2:] if not x.startswith('--')]
a, j, _ = spans[int(args[0])] if args else [s for s in spans if s[2]][-1]
gaps_only = '--gaps' in sys.argv
t0 = int(rows[a]['End_Timestamp'])
prev = t0
agg = defaultdict(float)
for r in rows[a + 1:j + 1]:
    s, e = int(r['Start_Timestamp']), int(r['End_Timestamp'])
    g = (s - prev) / 1e3
    if not gaps_only or g > 3:
        print("%8.1f dur %6.1f gap %6.1f q%s %s" % ((s - t0) / 1e3, (e - s) / 1e3, g, r['Queue_Id'], r['Kernel_Name'][:50]))
    prev = max(prev, e)
    agg[r['Kernel_Name'][:40]] += (e - s) / 1e3
print("span %.1f us" % ((int(rows[j]['Start_Timestamp']) - t0) / 1e3))
for k, v in sorted(agg.items(), key=lambda x: -x[1])[:25]:
    print("%7.1f %s" % (v, k))
