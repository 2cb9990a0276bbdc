"""Lab: PCG iterations launched one by one vs replayed from a hipGraph
(xfk_pcg_time with XFK_PCG_GRAPH=K), on the configs[2] problem."""
import os, sys
R = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, R)
from xfemm_amd import kernels, synth
cells = int(sys.argv[1]) if len(sys.argv) > 1 else 1000
P = kernels.Static2DProblem(**synth.magnetostatic(cells))
P.solve(rebuild_symbolic=True)
for K in (2, 8, 20):
    os.environ["XFK_PCG_GRAPH"] = str(K)
    for rep in range(2):
        s, g = P.pcg_time(40)
        print("K=%2d stream %.1f us/iteration, graph %.1f us/iteration" % (K, 1e3 * s, 1e3 * g), flush=True)
