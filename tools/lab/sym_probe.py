"""Symbolic-phase timing probe: rebuild the 2M-tri problem's symbolic data a
few times (tools/lab/timeline.py reads the kernel trace of this under rocprofv3)."""
import os, sys, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from xfemm_amd import kernels, synth

n = int(sys.argv[1]) if len(sys.argv) > 1 else 1000
kw = synth.magnetostatic(n)
P = kernels.Static2DProblem(**kw)
for k in range(3):
    t = time.time()
    r = P.solve(rebuild_symbolic=True)
    print("n=%d run %d: wall %.1f ms symbolic %.2f ms colours %d rounds %d" % (
        n, k, 1e3 * (time.time() - t), r["ms_symbolic"], r["ncolors"], r["color_rounds"]), flush=True)
