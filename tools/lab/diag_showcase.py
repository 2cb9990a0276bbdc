import sys, os
sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", "/root/repo")); sys.path.insert(0, os.path.join(os.environ.get("GRAFT_REPO_ROOT", "/root/repo"), "tests"))
import numpy as np
from oracle import oracle
from util import rel_err, synth_to_oracle
from xfemm_amd import kernels, synth
pr, mesh, kw = synth_to_oracle(synth.bc_showcase(24, nonlinear=True))
Ao, st, _ = oracle.solve(pr, mesh)
print("oracle", st)
for pc in ["jacobi", "amg"]:
    P = kernels.Static2DProblem(precond=pc, **kw)
    r = P.solve(); A = P.solution()
    print(pc, "newton", r["newton_iters"], "cg", r["cg_iters"], "last_res", r["last_res"], "final_er", r["final_er"], "err", rel_err(A, Ao))
    i = np.argmax(np.abs(A - Ao)); print("   worst node", i, A[i], Ao[i])
for prec in [1e-10, 1e-12]:
    kw2 = dict(kw); kw2["precision"] = prec
    P = kernels.Static2DProblem(precond="amg", **kw2)
    r = P.solve(); A = P.solution()
    pr2 = pr; pr2.Precision = prec
    Ao2, st2, _ = oracle.solve(pr2, mesh)
    print("amg prec", prec, "newton", r["newton_iters"], "cg", r["cg_iters"], "err vs oracle(same prec)", rel_err(A, Ao2), "oracle newton", st2["newton_iters"])
    P = kernels.Static2DProblem(precond="jacobi", **kw2)
    r = P.solve(); A = P.solution()
    print("jac prec", prec, "newton", r["newton_iters"], "cg", r["cg_iters"], "err", rel_err(A, Ao2))
