"""HarmonicAxisymmetric on the device (xfk_harmonic.hip, problem_type
XFK_AXISYMMETRIC) against the oracle (tests/test_oracle_harmonic_axi.py pins
it: exact uniform field, the reference's own cspars.cpp).

Tolerances (f64 / complex f64), as for the planar harmonic path:
  * assembled complex system after all boundary conditions: <= 1e-12 max |A|
  * flux at every node: <= 1e-6 of max |flux| against the converged oracle
    (Precision 1e-13, util.converged); nonlinear: 1e-5
  * uniform axial field: the exact flux pi B0 r^2 to 1e-9
"""
import numpy as np
import pytest
import scipy.sparse as sp

from oracle import harmonic as oh
from util import assert_parity, converged, rel_err, synth_to_oracle
from xfemm_amd import kernels, synth

pytestmark = pytest.mark.gpu


def test_harmonic_axi_system_matches_oracle():
    kw = synth.harmonic_axisymmetric(16)
    pr, mesh, kk = synth_to_oracle(kw)
    P = kernels.Harmonic2DProblem(**kk)
    P.solve()
    rp, col, val, b = P.csr()
    n = len(rp) - 1
    G = sp.csr_matrix((val, col, rp), shape=(n, n))
    O, bo = oh.system(pr, mesh)
    assert abs(G - O).max() <= 1e-12 * abs(O).max()
    assert np.abs(b - bo).max() <= 1e-12 * np.abs(bo).max()
    P.close()


@pytest.mark.parametrize("opts", [dict(), dict(circuits=False), dict(external=True)])
def test_harmonic_axi_solution_matches_oracle(opts):
    kw = synth.harmonic_axisymmetric(24, **opts)
    pr, mesh, kk = synth_to_oracle(kw)
    P = kernels.Harmonic2DProblem(**kk)
    P.solve()
    A = P.solution()
    Ao, _, circ_o = oh.solve(pr, mesh)
    Ac = converged(pr, mesh, oh.solve)
    assert_parity(A, Ao, Ac, 1e-6)
    cc, J, dV = P.circuits()
    for k, (case, Jo, dVo) in enumerate(circ_o):
        assert cc[k] == case and abs(J[k] - Jo) <= 1e-12 * max(1.0, abs(Jo))
        assert abs(dV[k] - dVo) <= 1e-12 * max(1.0, abs(dVo))
    P.close()


def test_harmonic_axi_uniform_field_exact():
    kw = synth.axisymmetric_uniform(20, B0=1.0)
    kw["frequency"] = 60.0
    pr, mesh, kk = synth_to_oracle(kw)
    P = kernels.Harmonic2DProblem(**kk)
    P.solve()
    A = P.solution()
    P.close()
    exact = np.pi * (0.01 * mesh.x) ** 2
    assert np.abs(A.real - exact).max() <= 1e-9 * exact.max()
    assert np.abs(A.imag).max() <= 1e-9 * exact.max()


def test_harmonic_axi_nonlinear_matches_oracle():
    kw = synth.harmonic_axisymmetric(16, nonlinear=True)
    pr, mesh, kk = synth_to_oracle(kw)
    Ao, st, _ = oh.solve(pr, mesh)
    P = kernels.Harmonic2DProblem(**kk)
    r = P.solve()
    A = P.solution()
    P.close()
    assert st["newton_iters"] > 1 and r["newton_iters"] > 1
    assert rel_err(A, Ao) <= 1e-5


def test_harmonic_axi_file_interface_end_to_end(tmp_path):
    """.fem ([ProblemType] axisymmetric, [Frequency] > 0) -> FSolver -> .ans (flux)."""
    from oracle import femfile
    from xfemm_amd import fsolver
    from test_gpu_harmonic import _read_harmonic_ans
    kw = synth.harmonic_axisymmetric(14, circuits=False)
    kw["marker"] = None
    kw["points"] = []
    base = str(tmp_path / "ha")
    synth.write_problem(base, kw)
    pr, mesh = femfile.load_problem(base)
    assert pr.ProblemType == 1 and pr.Frequency == kw["frequency"]
    Ao, _, _ = oh.solve(pr, mesh)
    fs = fsolver.FSolver()
    fs.PathName = base
    assert fs.LoadProblemFile()
    assert fs.runSolver(False), fs.last_error()
    nodes, _ = _read_harmonic_ans(base + ".ans")
    A = nodes[:, 2] + 1j * nodes[:, 3]
    assert rel_err(A, Ao) <= 1e-6


def test_harmonic_axi_case2_circuit_matches_oracle():
    kw = synth.harmonic_axisymmetric(20)
    kw["circuits"][1] = dict(type=0, amps_re=500.0, amps_im=-100.0)   # the ring: specified current
    pr, mesh, kk = synth_to_oracle(kw)
    Ao, _, circ_o = oh.solve(pr, mesh)
    assert circ_o[1][0] == 2
    P = kernels.Harmonic2DProblem(**kk)
    P.solve()
    A = P.solution()
    cc, J, dV = P.circuits()
    P.close()
    assert rel_err(A, Ao) <= 1e-6
    assert cc[1] == 2 and abs(dV[1] - circ_o[1][2]) <= 1e-6 * abs(circ_o[1][2])
