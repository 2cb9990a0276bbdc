"""Level sizes of the configs[2] hierarchy (XFK_AMG_DEBUG=1 prints them)."""
import os
import sys
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
from xfemm_amd import kernels, synth
from util import synth_to_oracle
cells = int(sys.argv[1]) if len(sys.argv) > 1 else 1000
kw = synth.magnetostatic(cells)
P = kernels.Static2DProblem(**kw)
print(P.solve(rebuild_symbolic=True))
P.close()
