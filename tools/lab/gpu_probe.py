"""Quick GPU probe: HIP path vs oracle on the golden problems + synthetic ones.
Run on the GPU box:  python tools/lab/gpu_probe.py"""
import os
import sys
import time

import numpy as np
import scipy.sparse as sp

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))

from oracle import ansmesh, femfile, oracle  # noqa: E402
from util import kernel_kwargs, rel_err, synth_to_oracle  # noqa: E402
from xfemm_amd import kernels, synth  # noqa: E402


def compare_system(P, pr, mesh):
    rp, col, val, b = P.csr()
    n = len(rp) - 1
    G = sp.csr_matrix((val, col, rp), shape=(n, n))
    O, bo = oracle.system(pr, mesh)
    D = (G - O)
    dmax = abs(D).max() if D.nnz else 0.0
    print("   system: |G-O|max %.3e  |O|max %.3e  b err %.3e  zero diags gpu %d oracle %d" % (
        dmax, abs(O).max(), rel_err(b, bo), int((G.diagonal() == 0).sum()), int((O.diagonal() == 0).sum())))
    zd = np.nonzero(G.diagonal() == 0)[0][:5]
    for i in zd:
        print("     row", i, "gpu cols", col[rp[i]:rp[i + 1]], "vals", val[rp[i]:rp[i + 1]])
        print("            oracle cols", O[i].indices, "vals", O[i].data)


def run(kw, label, pr=None, mesh=None):
    t = time.time()
    P = kernels.Static2DProblem(**kw)
    try:
        r = P.solve()
    except Exception as ex:
        print("%s: FAILED %s" % (label, ex))
        if pr is not None:
            compare_system(P, pr, mesh)
        return None, P
    A = P.solution()
    print("%s: gpu solve %.1f ms wall, %s" % (label, 1e3 * (time.time() - t),
                                             {k: (round(v, 3) if isinstance(v, float) else v) for k, v in r.items()}))
    if pr is not None and not r["newton_iters"] > 1:
        compare_system(P, pr, mesh)
    return A, P


print("devices", kernels.device_count(), flush=True)
for n, nl in [(40, False), (40, True), (200, False)]:
    kw = synth.magnetostatic(n, nonlinear=nl)
    prs, meshs, kws = synth_to_oracle(kw)
    A, P = run(kws, "synth n=%d nonlinear=%s" % (n, nl), prs, meshs)
    Ao, st, _ = oracle.solve(prs, meshs)
    if A is not None:
        print("   rel err vs oracle: %.3e  oracle %s" % (rel_err(A, Ao), st), flush=True)

for name in ["Temp", "Temp1"]:
    pr = femfile.prepare_problem(femfile.parse_fem(os.path.join(ROOT, "tests/golden/%s.fem" % name)))
    femfile.get_fill_factor(pr)
    mesh, sol = ansmesh.mesh_from_ans(os.path.join(ROOT, "tests/golden/%s.fem" % name),
                                      os.path.join(ROOT, "tests/golden/%s.ans.check" % name), pr)
    A, P = run(kernel_kwargs(pr, mesh), name, pr, mesh)
    if A is not None:
        print("   rel err vs golden .ans.check: %.3e" % rel_err(A, sol.A), flush=True)
        cc, J, dV = P.circuits()
        print("   circuits J", J[:8])

pr, mesh = femfile.load_problem(os.path.join(ROOT, "tests/golden/Temp"))
A, P = run(kernel_kwargs(pr, mesh), "Temp mesh files", pr, mesh)
if A is not None:
    Ao, st, _ = oracle.solve(pr, mesh)
    print("   rel err vs oracle: %.3e  oracle %s" % (rel_err(A, Ao), st), flush=True)

for n in [1000]:
    kw = synth.magnetostatic(n)
    P = kernels.Static2DProblem(**{k: v for k, v in kw.items()})
    for k in range(3):
        t = time.time()
        r = P.solve(rebuild_symbolic=True)
        print("n=%d run %d: wall %.1f ms %s" % (n, k, 1e3 * (time.time() - t), r), flush=True)
    ms_spmv, ms_iter = P.pcg_time(100)
    nnz = r["nnz"]
    N = P.n_nodes
    b = 12 * nnz + 4 * (N + 1) + 16 * N
    print("spmv %.4f ms (%.1f GB/s algorithmic), iteration (2 launches + gaps) %.4f ms" % (ms_spmv, b / ms_spmv / 1e6, ms_iter))
