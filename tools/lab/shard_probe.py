"""In-process sharded solve (N ranks on one GPU) vs single device: iterations, agreement."""
import os, sys, threading, time
R = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, R)
import numpy as np
from xfemm_amd import kernels, synth
cells = int(sys.argv[1]) if len(sys.argv) > 1 else 400
ranks = [int(a) for a in sys.argv[2:] if not a.startswith("--")] or [2, 4, 8]
opt = {}
for a in sys.argv[2:]:
    if a.startswith("--omega="):
        opt["amg_omega"] = float(a.split("=")[1])
    if a.startswith("--sweeps="):
        opt["amg_sweeps"] = int(a.split("=")[1])
    if a.startswith("--theta="):
        opt["amg_theta"] = float(a.split("=")[1])
    if a.startswith("--rep="):
        opt["amg_replicate"] = int(a.split("=")[1])
    if a == "--single-only":
        ranks = []
kw = synth.magnetostatic(cells)
P = kernels.Static2DProblem(**kw, **opt); r1 = P.solve(); A1 = P.solution(); P.close()
print("single: iters %d levels %d setup %.1f ms solve %.1f ms" % (r1["cg_iters"], r1["amg_levels"],
      r1["ms_amg_setup"], r1["ms_solve"]), flush=True)
for n in ranks:
    comms = kernels.Comm.local_group(n)
    probs = [kernels.Static2DProblem(**kw, comm=comms[q], **opt) for q in range(n)]
    out = [None] * n
    def work(q):
        out[q] = (probs[q].solve(), probs[q].solution())
    t0 = time.time()
    th = [threading.Thread(target=work, args=(q,)) for q in range(n)]
    [t.start() for t in th]; [t.join() for t in th]
    dt = time.time() - t0
    r, A = out[0]
    print("ranks %d: iters %d precond %d levels %d err vs single %.2e (%.2f s; rank 0: setup %.1f ms solve %.1f ms)" % (
        n, r["cg_iters"], r["precond"], r["amg_levels"], np.abs(A - A1).max() / np.abs(A1).max(), dt,
        r["ms_amg_setup"], r["ms_solve"]), flush=True)
    [p.close() for p in probs]; [c.close() for c in comms]
