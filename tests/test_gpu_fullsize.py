"""The bench workloads themselves, at full size (BASELINE configs[2] and [3]).

The oracle's linked-list solver is far too slow at 2M triangles, so these use
size-independent properties and an independent vectorised restatement of the
same element loop (tests/fullsize.py, pinned against the oracle's system to
3e-16 on smaller meshes by tests/test_fullsize_cpu.py):

configs[2] (2M-tri linear, what bench.py times):
  * the device's assembled system after boundary conditions equals the
    restatement's: max |dK| <= 1e-12 max |K|, same for b;
  * the device's A equals a direct (SuperLU) solve of that system to 1e-6 of
    max |A| (the linear parity tolerance);
  * two solves from scratch are bit-identical.
configs[3] (2M-tri M-19 steel, Newton):
  * the device's A is a fixed point of the secant system it converged to
    (restated assembly at the returned A): |b - K(A) V| / |b| <= 1e-6;
  * bit-identical repeat.
"""
import numpy as np
import pytest
import scipy.sparse as sp
import scipy.sparse.linalg as spla

import fullsize
from util import assert_parity, rel_err, synth_to_oracle
from xfemm_amd import kernels, synth

pytestmark = pytest.mark.gpu

CELLS = 1000          # 2 * 1000^2 = 2M triangles (configs[2] / configs[3])


def _device_system(P):
    rp, col, val, b = P.csr()
    n = len(rp) - 1
    return sp.csr_matrix((val, col, rp), shape=(n, n)), b


def test_configs2_full_size_matches_direct_solve():
    pr, mesh, kw = synth_to_oracle(synth.magnetostatic(CELLS))
    P = kernels.Static2DProblem(**kw)
    r = P.solve(rebuild_symbolic=True)
    A = P.solution()
    G, bg = _device_system(P)
    P.solve(rebuild_symbolic=True)
    A2 = P.solution()
    P.close()
    assert len(mesh.p) == 2_000_000 and r["newton_iters"] == 1
    assert np.array_equal(A, A2)
    K, b, _ = fullsize.assemble(pr, mesh)
    assert abs(G - K).max() <= 1e-12 * abs(K).max()
    assert np.abs(bg - b).max() <= 1e-12 * np.abs(b).max()
    exact = spla.spsolve(K.tocsc(), b) * fullsize.C_ANS
    err = rel_err(A, exact)
    assert err <= 1e-6, "max|A - A_direct| / max|A| = %.3e after %d PCG iterations" % (err, r["cg_iters"])


def test_configs3_full_size_newton_fixed_point():
    pr, mesh, kw = synth_to_oracle(synth.magnetostatic(CELLS, nonlinear=True))
    P = kernels.Static2DProblem(**kw)
    r = P.solve(rebuild_symbolic=True)
    A = P.solution()
    P.solve(rebuild_symbolic=True)
    A2 = P.solution()
    P.close()
    assert r["newton_iters"] >= 3
    assert np.array_equal(A, A2)
    V = A / fullsize.C_ANS
    K, b, _ = fullsize.assemble(pr, mesh, V)
    res = np.linalg.norm(b - K @ V) / np.linalg.norm(b)
    assert res <= 1e-6, "secant residual %.3e after %d Newton / %d PCG iterations" % (
        res, r["newton_iters"], r["cg_iters"])


_CONVERGED = {}


@pytest.mark.parametrize("inexact", [True, False])
def test_nonlinear_180k_matches_converged_oracle(inexact):
    """configs[3]'s problem at 180k triangles (the largest the CPU oracle runs
    to convergence in seconds): the device's Newton loop -- inexact passes
    with a last pass at Precision (the default), or every pass at Precision as
    the reference's loop -- against the oracle run to Precision 1e-13, at the
    nonlinear tolerance 1e-5 of max |A| (tests/test_gpu_static2d.py)."""
    from util import converged
    pr, mesh, kw = synth_to_oracle(synth.magnetostatic(300, nonlinear=True))
    P = kernels.Static2DProblem(newton_inexact=inexact, **kw)
    r = P.solve()
    A = P.solution()
    P.close()
    if "nl180k" not in _CONVERGED:   # (one oracle run of each kind for both cases)
        from oracle import oracle
        _CONVERGED["nl180k"] = converged(pr, mesh), oracle.solve(pr, mesh)[0]
    Ac, Ao = _CONVERGED["nl180k"]
    assert r["newton_iters"] >= 3
    assert_parity(A, Ao, Ac, 1e-5, " (%d Newton / %d PCG iterations)" % (r["newton_iters"], r["cg_iters"]))
