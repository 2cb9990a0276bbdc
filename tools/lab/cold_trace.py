"""Lab: the configs[2] cold first solve (bench.py cold_first_solve: a fresh
problem, the process's AMG hints dropped, the bench's own problem alive) inside
a [window] for a rocprofv3 kernel trace (tools/lab/trace_window.py)."""
import ctypes
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
from xfemm_amd import kernels, synth  # noqa: E402


def sync():
    ctypes.CDLL("libamdhip64.so").hipDeviceSynchronize()


kw = synth.magnetostatic(1000)
P0 = kernels.Static2DProblem(**kw)
for _ in range(3):
    P0.solve(rebuild_symbolic=True)
kernels.forget_amg_hints()
P = kernels.Static2DProblem(**kw)
sync()
w0 = time.monotonic_ns()
t0 = time.perf_counter()
r = P.solve(rebuild_symbolic=True)
sync()
t1 = time.perf_counter()
print("[window] cold %d %d solves 1" % (w0, time.monotonic_ns()), file=sys.stderr, flush=True)
print("cold first solve %.3f ms, setup %.3f ms" % (1e3 * (t1 - t0), r["ms_amg_setup"]), flush=True)
w0 = time.monotonic_ns()
t0 = time.perf_counter()
r = P.solve(rebuild_symbolic=True)
sync()
t1 = time.perf_counter()
print("[window] warm %d %d solves 1" % (w0, time.monotonic_ns()), file=sys.stderr, flush=True)
print("repeated solve %.3f ms, setup %.3f ms" % (1e3 * (t1 - t0), r["ms_amg_setup"]), flush=True)
