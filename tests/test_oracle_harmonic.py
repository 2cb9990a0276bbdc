"""The harmonic oracle pinned to the reference: the restated Harmonic2D
element loop driving (a) the restated CBigComplexLinProb and (b) the
reference's own cspars.cpp compiled from /root/reference (oracle/_ref) gives
bit-identical A and circuit results; and the answer solves the exported
system to the reference's tolerance.  CPU only."""
import numpy as np
import pytest
import scipy.sparse.linalg as sla

from oracle import harmonic as oh
from oracle import oracle
from util import C_ANS, synth_to_oracle
from xfemm_amd import synth


def _case(kind):
    if kind == "plain":
        return synth.harmonic(14)
    if kind == "periodic":
        return synth.harmonic(14, periodic=True)
    if kind == "case2":
        kw = synth.harmonic(14)
        kw["circuits"][1] = dict(type=0, amps_re=1.5, amps_im=-0.5)
        return kw
    return synth.harmonic(14, frequency=5000.0, circuits=False)


@pytest.mark.skipif(not oracle.ref_available(), reason="reference build (oracle/_ref) absent")
@pytest.mark.parametrize("kind", ["plain", "periodic", "case2", "hf"])
def test_restated_complex_linprob_is_bit_identical_to_reference(kind):
    pr, mesh, _ = synth_to_oracle(_case(kind))
    A1, st1, c1 = oh.solve(pr, mesh, "oracle")
    A2, st2, c2 = oh.solve(pr, mesh, "reference")
    assert np.array_equal(A1, A2)
    assert c1 == c2
    assert st1["cg_iters"] > 0


@pytest.mark.parametrize("kind", ["plain", "periodic", "hf"])
def test_oracle_solves_its_system(kind):
    pr, mesh, _ = synth_to_oracle(_case(kind))
    A, _, _ = oh.solve(pr, mesh)
    M, b = oh.system(pr, mesh)
    V = A / C_ANS
    assert np.linalg.norm(b - M @ V) / np.linalg.norm(b) <= 2 * pr.Precision
    exact = sla.spsolve(M.tocsc(), b)
    assert np.abs(V - exact).max() / np.abs(exact).max() <= 1e-4
