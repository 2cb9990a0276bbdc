"""One AMG static-2D solve of the configs[2] problem (profiling target)."""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
from xfemm_amd import kernels, synth  # noqa: E402
n = int(sys.argv[1]) if len(sys.argv) > 1 else 1000
pc = sys.argv[2] if len(sys.argv) > 2 else "amg"
P = kernels.Static2DProblem(device=0, precond=pc, **synth.magnetostatic(n))
for _ in range(3):
    r = P.solve(rebuild_symbolic=True)
print(r)
