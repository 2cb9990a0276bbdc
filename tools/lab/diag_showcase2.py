import os, sys
R = os.environ.get("GRAFT_REPO_ROOT", os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
sys.path.insert(0, R); sys.path.insert(0, os.path.join(R, "tests"))
import numpy as np, scipy.sparse as sp, scipy.sparse.linalg as sla
from oracle import oracle
from util import rel_err, synth_to_oracle
from xfemm_amd import kernels, synth
pr, mesh, kw = synth_to_oracle(synth.bc_showcase(24, nonlinear=True))
C = np.pi * 4e-5
for prec in [1e-8, 1e-12]:
    kw["precision"] = prec
    for pc in ["jacobi", "amg"]:
        P = kernels.Static2DProblem(precond=pc, **kw)
        r = P.solve(); A = P.solution()
        rp, col, val, b = P.csr()
        M = sp.csr_matrix((val, col, rp), shape=(len(rp) - 1,) * 2)
        V = A / C
        xd = sla.spsolve(M.tocsc(), b)
        ev = np.linalg.eigvalsh(M.toarray()) if M.shape[0] < 2000 else None
        print("prec %.0e %-6s newton %d relres(final sys) %.2e  |V-solve(final)|/|V| %.2e  minEig %.3e maxEig %.3e asym %.1e" % (
            prec, pc, r["newton_iters"], np.linalg.norm(b - M @ V) / np.linalg.norm(b), np.abs(V - xd).max() / np.abs(xd).max(),
            ev.min(), ev.max(), abs(M - M.T).max()))
