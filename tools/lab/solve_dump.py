"""Lab: solve the configs[2] mesh once (default options) and save A (bit checks across builds / env switches)."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from xfemm_amd import kernels, synth  # noqa: E402

cells = int(os.environ.get("CELLS", "1000"))
P = kernels.Static2DProblem(**synth.magnetostatic(cells))
P.solve(rebuild_symbolic=True)
r = P.solve(rebuild_symbolic=True)
np.save(sys.argv[1], P.solution())
print("solved", cells, r["cg_iters"])
