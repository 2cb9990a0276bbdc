"""Lab: a problem's arena footprint after its first solve (configs[2] linear and
nonlinear, configs[1]-size), to size the reservation taken at creation."""
import os, sys, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from xfemm_amd import kernels, synth
for cells, nl in ((1000, False), (1000, True), (320, False), (100, False)):
    kw = synth.magnetostatic(cells, nonlinear=nl)
    kernels.alloc_stats(reset=True)
    P = kernels.Static2DProblem(**kw)
    a0 = kernels.alloc_stats(reset=True)
    m0 = P.memory()
    P.solve()
    a1 = kernels.alloc_stats(reset=True)
    m1 = P.memory()
    P.solve()
    m2 = P.memory()
    n = len(kw["x"]); ne = len(kw["p"]) // 3
    print("cells %d nl %d: N %d NE %d | create %s %s | first solve %s %s | second %s" % (cells, nl, n, ne, a0, m0, a1, m1, m2),
          flush=True)
    P.close()
