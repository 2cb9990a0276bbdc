"""Lab: one configs[3] solve (2M-tri M-19 Newton, bench settings) inside a
[window] for a rocprofv3 kernel trace; XFK_TRACE_NEWTON=1 prints the passes."""
import ctypes
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
from xfemm_amd import kernels, synth  # noqa: E402


def sync():
    ctypes.CDLL("libamdhip64.so").hipDeviceSynchronize()


kw = synth.magnetostatic(1000, nonlinear=True)
P = kernels.Static2DProblem(newton_inexact=True, **kw)
for _ in range(2):
    P.solve(rebuild_symbolic=True)
sync()
w0 = time.monotonic_ns()
t0 = time.perf_counter()
r = P.solve(rebuild_symbolic=True)
sync()
t1 = time.perf_counter()
print("[window] newton %d %d solves 1" % (w0, time.monotonic_ns()), file=sys.stderr, flush=True)
print("configs[3] solve %.3f ms: newton %d pcg %d setup %.3f" % (1e3 * (t1 - t0), r["newton_iters"], r["cg_iters"],
                                                               r["ms_amg_setup"]), flush=True)
