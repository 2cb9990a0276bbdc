"""Compare bench.py JSON lines: step time, setup, PCG iteration and the phases.
usage: python tools/lab/phases.py A.json B.json ..."""
import json, sys
ds = [(p, json.loads(open(p).read().strip().splitlines()[-1])) for p in sys.argv[1:]]
for p, d in ds:
    c = d["config"]
    print("%-40s %8.3f ms/step  setup %.3f  pcg it %3d x %.1f us  sym %.3f asm %.3f  spmv %.1f us" % (
        p[-40:], d["ms_per_step"], c["ms_amg_setup"], c["pcg_iters"], 1e3 * c["ms_per_pcg_iteration"],
        c["ms_symbolic"], c["ms_assemble"], d["roofline"]["launch_us"]))
names = []
for _, d in ds:
    for ph in d["roofline"].get("phases", []):
        if ph["phase"] not in names:
            names.append(ph["phase"])
for nm in names:
    row = []
    for _, d in ds:
        m = {ph["phase"]: ph for ph in d["roofline"].get("phases", [])}
        row.append("%8.1f" % m[nm]["us_per_launch"] if nm in m else "       -")
    print("%-62s %s" % (nm[:62], " ".join(row)))
