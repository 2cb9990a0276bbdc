"""Diagnostic: AMG-PCG vs direct solve on assembled oracle systems (true residual)."""
import os, sys
R = os.environ.get("GRAFT_REPO_ROOT", os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
sys.path.insert(0, R); sys.path.insert(0, os.path.join(R, "tests"))
import numpy as np
import scipy.sparse.linalg as sla
from oracle import oracle
from util import synth_to_oracle
from xfemm_amd import kernels, synth
cases = {"showcase": synth.bc_showcase(24), "showcase_anti": synth.bc_showcase(24, anti=True),
         "linear": synth.magnetostatic(40), "chain": synth.bc_chain(20)}
for name, kw0 in cases.items():
    pr, mesh, kw = synth_to_oracle(kw0)
    O, b = oracle.system(pr, mesh)
    O = O.tocsr(); O.sort_indices()
    xd = sla.spsolve(O.tocsc(), b)
    sym = abs(O - O.T).max()
    for pc in ["jacobi", "amg"]:
        for prec in [1e-8, 1e-12]:
            V, it, er = kernels.pcg_solve_csr(O.indptr, O.indices, O.data, b, precision=prec, precond=pc)
            res = np.linalg.norm(b - O @ V) / np.linalg.norm(b)
            print("%-14s %-6s prec %.0e it %4d er %.2e relres %.2e err %.2e (asym %.1e, diag<=0: %d)" % (
                name, pc, prec, it, er, res, np.abs(V - xd).max() / np.abs(xd).max(), sym, (O.diagonal() <= 0).sum()))
print("--- flag = 1 (initial guess) ---")
for name, kw0 in cases.items():
    pr, mesh, kw = synth_to_oracle(kw0)
    O, b = oracle.system(pr, mesh)
    O = O.tocsr(); O.sort_indices()
    xd = sla.spsolve(O.tocsc(), b)
    rng = np.random.default_rng(0)
    for scale in [1e-2, 1e-6]:
        V0 = xd * (1 + scale * rng.standard_normal(len(xd)))
        for pc in ["jacobi", "amg"]:
            V, it, er = kernels.pcg_solve_csr(O.indptr, O.indices, O.data, b, V0=V0, flag=1, precision=1e-12, precond=pc)
            res = np.linalg.norm(b - O @ V) / np.linalg.norm(b)
            print("%-14s %-6s pert %.0e it %4d er %.2e relres %.2e err %.2e" % (
                name, pc, scale, it, er, res, np.abs(V - xd).max() / np.abs(xd).max()))
