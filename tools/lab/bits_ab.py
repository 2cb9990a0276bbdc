"""Lab: solve a few problems and save their solutions, with the in-tree
library or another build of it (argv[2]): bit checks of a change that must
not move a bit.  Usage: python tools/lab/bits_ab.py OUT.npz [LIB.so]"""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from xfemm_amd import kernels, synth  # noqa: E402

if len(sys.argv) > 2:
    kernels.load_library(sys.argv[2])
out = {}
for name, kw in [("c2", synth.magnetostatic(1000)), ("nl", synth.magnetostatic(300, nonlinear=True)),
                 ("axi", synth.axisymmetric(300)), ("bc", synth.bc_showcase(200, anti=True))]:
    P = kernels.Static2DProblem(**kw)
    r = P.solve(rebuild_symbolic=True)
    out[name] = P.solution().copy()
    print(name, r.get("cg_iters"), flush=True)
    P.close()
np.savez(sys.argv[1], **out)
