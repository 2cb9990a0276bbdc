"""Lab (round 6): solve a nonlinear planar problem and save A (compare the
element-matrix pass XFK_ASM_EM=1 with the rows' own evaluation =0)."""
import os
import sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import numpy as np  # noqa: E402
from xfemm_amd import kernels, synth  # noqa: E402
kw = synth.magnetostatic(int(sys.argv[2]), nonlinear=True)
P = kernels.Static2DProblem(**kw)
st = P.solve()
np.save(sys.argv[1], P.solution())
print(sys.argv[1], st["newton_iters"] if "newton_iters" in st else "", st.get("cg_iters"))
P.close()
