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
    if kind in ("case2", "case2_periodic", "case2_anti"):
        kw = synth.harmonic(14, periodic=kind != "case2", anti=kind == "case2_anti")
        kw["circuits"][1] = dict(type=0, amps_re=1.5, amps_im=-0.5)
        return kw
    return synth.harmonic(14, frequency=5000.0, circuits=False)


@pytest.mark.skipif(not oracle.ref_available(), reason="reference build (oracle/_ref) absent")
@pytest.mark.parametrize("kind", ["plain", "periodic", "case2", "case2_periodic", "case2_anti", "hf"])
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


def _newton_case(kind):
    if kind == "axi":
        kw = synth.harmonic_axisymmetric(12, nonlinear=True)
    elif kind == "axi_ext":
        kw = synth.harmonic_axisymmetric(12, nonlinear=True, external=True)
    elif kind in ("periodic", "case2_periodic", "case2_anti"):
        kw = synth.harmonic(14, nonlinear=True, periodic=True, anti=kind == "case2_anti")
        if kind != "periodic":   # a Case-2 circuit together with (anti)periodic pairs (harmonic2d.cpp:157, 811-812)
            kw["circuits"][1] = dict(type=0, amps_re=1.5, amps_im=-0.5)
    elif kind == "hf":
        kw = synth.harmonic(14, nonlinear=True, frequency=5000.0)
    elif kind == "stiff":   # KludgeSolve stagnates (line-search step -> 0): the reference's path, bit for bit
        kw = synth.harmonic(24, nonlinear=True)
    else:
        kw = synth.harmonic(14, nonlinear=True)
    kw["ac_solver"] = 1
    return kw


@pytest.mark.skipif(not oracle.ref_available(), reason="reference build (oracle/_ref) absent")
@pytest.mark.parametrize("kind", ["planar", "periodic", "case2_periodic", "case2_anti", "hf", "stiff", "axi",
                                  "axi_ext"])
def test_newton_ac_solver_is_bit_identical_to_reference(kind):
    """[ACSolver] = 1: the element Newton terms (harmonic2d.cpp:611-639 /
    harmonicaxi.cpp:520-547) into the auxiliary matrices and KludgeSolve
    (cspars.cpp), the restated linprob against the compiled one."""
    kw = _newton_case(kind)
    pr, mesh, _ = synth_to_oracle(kw)
    A1, st1, c1 = oh.solve(pr, mesh, "oracle")
    A2, st2, c2 = oh.solve(pr, mesh, "reference")
    assert np.array_equal(A1, A2)
    assert c1 == c2 and st1["newton_iters"] == st2["newton_iters"]
    # the Newton path is taken: a different iteration and answer than ACSolver 0
    kw["ac_solver"] = 0
    pr0, mesh0, _ = synth_to_oracle(kw)
    A0, st0, _ = oh.solve(pr0, mesh0, "oracle")
    assert st0["newton_iters"] != st1["newton_iters"] and not np.array_equal(A0, A1)
