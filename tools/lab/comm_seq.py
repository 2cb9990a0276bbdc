"""The collective sequence of one sharded solve (in-process ranks on one GPU,
recording transport): each call's op and payload, run-length compressed, to
see which collectives the setup and each PCG iteration issue."""
import os
import sys
import threading

sys.path.insert(0, os.getcwd())
from xfemm_amd import kernels, synth  # noqa: E402

cells = int(sys.argv[1]) if len(sys.argv) > 1 else 1500
R = int(sys.argv[2]) if len(sys.argv) > 2 else 8
kw = synth.magnetostatic(cells)
comms = kernels.Comm.local_group(R)
probs = [kernels.Static2DProblem(**kw, comm=comms[q]) for q in range(R)]
out = [None] * R


def work(q):
    probs[q].solve(rebuild_symbolic=True)
    comms[q].record(1)
    out[q] = probs[q].solve(rebuild_symbolic=True)


th = [threading.Thread(target=work, args=(q,)) for q in range(R)]
for t in th:
    t.start()
for t in th:
    t.join()
log = comms[0].log()
seq = []
cur = None
for o in log:
    if o["op"] in ("send", "recv"):
        if o["op"] == "recv":
            cur[1] += o["bytes"]
        continue
    cur = [o["op"], o["bytes"] if o["op"] != "exchange" else 0]
    seq.append(cur)
print("rank 0: %d calls, pcg %d, levels %d" % (len(seq), out[0]["cg_iters"], out[0]["amg_levels"]))
toks = ["%s:%d" % (a[:2], b) for a, b in seq]
i = 0
while i < len(toks):
    # the shortest period p <= 16 repeating from i at least 3 times
    best = None
    for p in range(1, 17):
        k = 1
        while toks[i + k * p:i + (k + 1) * p] == toks[i:i + p] and i + (k + 1) * p <= len(toks):
            k += 1
        if k >= 3 and (best is None or k * p > best[0] * best[1]):
            best = (k, p)
    if best:
        k, p = best
        print("%4d  %d x [%s]" % (i, k, " ".join(toks[i:i + p])))
        i += k * p
    else:
        print("%4d  %s" % (i, toks[i]))
        i += 1
for p in probs:
    p.close()
