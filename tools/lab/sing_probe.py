import sys, numpy as np, scipy.sparse as sp
sys.path.insert(0, '/root/repo'); sys.path.insert(0, '/root/repo/tests')
from xfemm_amd import kernels
from test_gpu_amg import _laplace_random
M = _laplace_random(30, 11, shift=0.0)
n = M.shape[0]
b = np.random.default_rng(5).standard_normal(n); b -= b.mean()
for pc in ["jacobi", "amg"]:
    try:
        V, it, er = kernels.pcg_solve_csr(M.indptr, M.indices, M.data, b, precision=1e-10, precond=pc)
        print(pc, it, er, np.linalg.norm(M @ V - b) / np.linalg.norm(b), flush=True)
    except Exception as e:
        print(pc, "ERR", e, flush=True)
