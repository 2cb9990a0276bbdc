"""GPU probe: Jacobi vs AMG PCG on synthetic magnetostatic problems (iterations,
timings, hierarchy, agreement).  Usage: python tools/lab/amg_probe.py [cells ...]"""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
from xfemm_amd import kernels, synth  # noqa: E402

cells = [int(a) for a in sys.argv[1:] if not a.startswith("-")] or [100, 1000]
nonlin = "--nonlinear" in sys.argv
sweeps = [int(a.split("=")[1]) for a in sys.argv if a.startswith("--sweeps=")] or [2]
omegas = [float(a.split("=")[1]) for a in sys.argv if a.startswith("--omega=")] or [None]
reuse = [int(a.split("=")[1]) for a in sys.argv if a.startswith("--reuse=")]
nojac = "--no-jacobi" in sys.argv
denses = [int(a.split("=")[1]) for a in sys.argv if a.startswith("--dense=")] or [None]
for n in cells:
    kw = synth.magnetostatic(n, nonlinear=nonlin)
    sols = {}
    cases = ([] if nojac else ["jacobi"]) + ["amg%d" % k + ("" if w is None else "w%g" % w)
                                            + ("" if d is None else "d%d" % d)
                                            for k in sweeps for w in omegas for d in denses]
    for pc in cases:
        if pc == "jacobi":
            opt = dict(precond="jacobi")
        else:
            k, _, d = pc[3:].partition("d")
            k, _, w = k.partition("w")
            opt = dict(precond="amg", amg_sweeps=int(k), amg_omega=float(w) if w else None,
                       amg_dense=int(d) if d else None)
            if reuse:
                opt["amg_reuse"] = bool(reuse[0])
        P = kernels.Static2DProblem(device=0, **opt, **kw)
        r = P.solve()
        t0 = time.perf_counter()
        reps = 3
        for _ in range(reps):
            r = P.solve()
        dt = (time.perf_counter() - t0) / reps
        A = P.solution()
        sols[pc] = A
        print("n=%d %s: %.2f ms/step newton %d cg %d sym %.2f asm %.2f solve %.2f amg_setup %.2f levels %d opc %.2f"
              % (n, pc, dt * 1e3, r["newton_iters"], r["cg_iters"], r["ms_symbolic"], r["ms_assemble"],
                 r["ms_solve"], r["ms_amg_setup"], r["amg_levels"], r["amg_op_complexity"]), flush=True)
        P.close()
    ref = sols[cases[0]]
    for k in sols:
        d = np.abs(sols[k] - ref).max() / np.abs(ref).max()
        print("   %s: max|A - A_jac|/max|A| = %.3e" % (k, d), flush=True)
