"""HarmonicAxisymmetric oracle (oracle/harmonic2d_oracle.c, restating
cfemm/fsolver/harmonicaxi.cpp) -- CPU only.

harmonicaxi.cpp needs the reference's cmake-generated headers to build, so the
element loop is pinned by (1) the exact solution of a uniform axial field --
the flux 2 pi r A = pi B0 r^2 lies in the formulation's c0 + c1 r^2 + c2 z
space and is reproduced to roundoff at any frequency when nothing conducts --
and (2) the loop driving the reference's own CBigComplexLinProb (cspars.cpp
compiled into oracle/_ref) to the same bits as the restated one."""
import numpy as np
import pytest

from oracle import harmonic as oh
from oracle import oracle
from util import synth_to_oracle
from xfemm_amd import synth

needs_ref = pytest.mark.skipif(not oracle.ref_available(), reason="oracle/_ref not built (reference absent)")


@pytest.mark.parametrize("freq", [60.0, 5000.0])
def test_uniform_axial_field_exact(freq):
    kw = synth.axisymmetric_uniform(16, B0=1.0)
    kw["frequency"] = freq
    pr, mesh, _ = synth_to_oracle(kw)
    A, st, _ = oh.solve(pr, mesh)
    exact = np.pi * 1.0 * (0.01 * mesh.x) ** 2
    assert np.abs(A.real - exact).max() <= 1e-9 * exact.max()
    assert np.abs(A.imag).max() <= 1e-9 * exact.max()


@needs_ref
@pytest.mark.parametrize("opts", [dict(), dict(circuits=False), dict(external=True), dict(nonlinear=True)])
def test_restated_loop_matches_reference_linprob(opts):
    kw = synth.harmonic_axisymmetric(12, **opts)
    pr, mesh, _ = synth_to_oracle(kw)
    A1, s1, c1 = oh.solve(pr, mesh, "oracle")
    A2, s2, c2 = oh.solve(pr, mesh, "reference")
    assert np.array_equal(A1, A2) and s1["newton_iters"] == s2["newton_iters"]
    assert c1 == c2
