"""GPU probe: time-harmonic planar solve (COCG + complex Jacobi) at growing sizes."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
from xfemm_amd import kernels, synth  # noqa: E402

pcs = [a.split("=")[1] for a in sys.argv if a.startswith("--pc=")] or ["amg", "jacobi"]
for n, pc in [(int(a), pc) for a in sys.argv[1:] if not a.startswith("--") for pc in pcs] or [(300, "amg")]:
    freq = float(([a.split("=")[1] for a in sys.argv if a.startswith("--freq=")] or ["60"])[0])
    kw = synth.harmonic(n, circuits=False, frequency=freq, nonlinear="--nonlinear" in sys.argv)
    P = kernels.Harmonic2DProblem(**kw, precond=pc)
    r = P.solve()
    t0 = time.perf_counter()
    r = P.solve()
    dt = time.perf_counter() - t0
    print("n=%d dof=%d %s: %.1f ms passes %d cg %d asm %.1f ms solve %.1f ms amg_setup %.1f ms levels %d" % (
        n, P.n_nodes, pc, dt * 1e3, r["newton_iters"], r["cg_iters"], r["ms_assemble"], r["ms_solve"],
        r["ms_amg_setup"], r["amg_levels"]), flush=True)
    P.close()
