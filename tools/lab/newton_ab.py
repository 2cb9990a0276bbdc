"""configs[3] (2M-tri, M-19 Newton) with the inexact-Newton passes on / off:
the pass trace of one solve each, then the step time of 3 solves each (the
bench's step: symbolic phase included) and the answers' distance."""
import os
import subprocess
import sys
import time

sys.path.insert(0, os.getcwd())
import numpy as np  # noqa: E402

from xfemm_amd import kernels, synth  # noqa: E402

cells = int(sys.argv[1]) if len(sys.argv) > 1 else 1000
kw = synth.magnetostatic(cells, nonlinear=True)
sync = kernels.load_library()
hip = __import__("ctypes").CDLL("libamdhip64.so")
out = {}
for mode in (0, 1):
    P = kernels.Static2DProblem(**kw, newton_inexact=bool(mode))
    os.environ["XFK_TRACE_NEWTON"] = "1"
    r = P.solve(rebuild_symbolic=True)
    os.environ.pop("XFK_TRACE_NEWTON")
    hip.hipDeviceSynchronize()
    t0 = time.perf_counter()
    for _ in range(3):
        r = P.solve(rebuild_symbolic=True)
    hip.hipDeviceSynchronize()
    dt = (time.perf_counter() - t0) / 3
    out[mode] = P.solution()
    print("mode %d: %.2f ms/step (%.1f M DoF/s), newton %d, pcg %d, setup %.2f ms" % (
        mode, 1e3 * dt, P.n_nodes / dt / 1e6, r["newton_iters"], r["cg_iters"], r["ms_amg_setup"]), flush=True)
    P.close()
print("answers: max |dA| / max |A| = %.3e" % (np.abs(out[1] - out[0]).max() / np.abs(out[0]).max()))
