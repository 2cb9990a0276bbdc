"""The oracle's StaticAxisymmetric restatement (oracle/static2d_oracle.c:
ora_assemble_axi, following cfemm/fsolver/staticaxi.cpp:45-794), CPU only.

staticaxi.cpp itself is not compilable here (it needs the Lua instance whose
header cmake generates), so the restatement is pinned by physics the
formulation reproduces exactly -- a uniform axial field is in its
c0 + c1 r^2 + c2 z flux space -- and by the linear algebra being the
reference's own spars.cpp (identical answers through oracle/_ref)."""
import numpy as np
import pytest

from oracle import oracle
from util import synth_to_oracle
from xfemm_amd import synth


@pytest.mark.parametrize("B0", [0.3, 1.7])
def test_uniform_axial_field_is_exact(B0):
    pr, mesh, _ = synth_to_oracle(synth.axisymmetric_uniform(16, B0=B0))
    A, st, _ = oracle.solve(pr, mesh)
    exact = np.pi * B0 * (0.01 * mesh.x) ** 2
    assert np.abs(A - exact).max() <= 1e-10 * np.abs(exact).max()


def test_reference_linear_algebra_gives_identical_answer():
    pr, mesh, _ = synth_to_oracle(synth.axisymmetric(16))
    try:
        A_ref, _, _ = oracle.solve(pr, mesh, linprob="reference")
    except OSError:
        pytest.skip("oracle/_ref not built (reference absent)")
    A, _, _ = oracle.solve(pr, mesh)
    assert np.array_equal(A, A_ref)


def test_axis_nodes_carry_zero_flux_and_system_is_symmetric():
    pr, mesh, _ = synth_to_oracle(synth.axisymmetric(12))
    A, _, _ = oracle.solve(pr, mesh)
    assert np.all(A[mesh.x == 0.0] == 0.0)
    M, b = oracle.system(pr, mesh)
    assert abs(M - M.T).max() == 0.0


def test_nonlinear_newton_converges():
    pr, mesh, _ = synth_to_oracle(synth.axisymmetric(12, nonlinear=True))
    A, st, _ = oracle.solve(pr, mesh)
    assert st["newton_iters"] >= 3 and st["last_res"] < 100 * pr.Precision
