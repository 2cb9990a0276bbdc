"""FSolver::StaticAxisymmetric on the GPU (cfemm/fsolver/staticaxi.cpp:45-794)
against the oracle's restatement (oracle/static2d_oracle.c: ora_assemble_axi).

The reference's staticaxi.cpp cannot be compiled here (it pulls in the Lua
instance whose header cmake generates), so the axisymmetric restatement is
pinned two ways instead: by the uniform axial field, which lies in the
formulation's c0 + c1 r^2 + c2 z flux space and must come out exact
(tests/test_oracle_axisymmetric.py, and here for the device), and by the
linear algebra being the reference's own spars.cpp (identical answers with
linprob="reference").  Tolerances: assembled system 1e-12 relative; answers
as the planar tests (1e-6 linear, vs the converged oracle for the nonlinear and
ill-conditioned cases); answers are the flux 2 pi r A in Webers.
"""
import os

import numpy as np
import pytest
import scipy.sparse as sp

from oracle import oracle
from util import assert_parity, converged, rel_err, synth_to_oracle
from xfemm_amd import kernels, synth

pytestmark = pytest.mark.gpu

TOL_SYSTEM = 1e-12
TOL_LINEAR = 1e-6
TOL_NONLINEAR = 1e-5


def _system_err(P, pr, mesh):
    rp, col, val, b = P.csr()
    n = len(rp) - 1
    G = sp.csr_matrix((val, col, rp), shape=(n, n))
    Go, bo = oracle.system(pr, mesh)
    d = abs(G - Go)
    return d.max() / abs(Go).max(), np.abs(b - bo).max() / max(np.abs(bo).max(), 1e-300)


def test_uniform_axial_field_is_exact():
    kw = synth.axisymmetric_uniform(24, B0=0.8)
    P = kernels.Static2DProblem(**kw)
    P.solve()
    flux = P.solution()
    P.close()
    exact = np.pi * 0.8 * (0.01 * np.asarray(kw["x"])) ** 2
    assert rel_err(flux, exact) <= 1e-9


@pytest.mark.parametrize("variant", ["plain", "circuit", "external", "no_mixed"])
def test_linear_matches_oracle(variant):
    opt = dict(circuit=variant == "circuit", external=variant == "external", mixed=variant != "no_mixed")
    pr, mesh, kw = synth_to_oracle(synth.axisymmetric(40, **opt))
    Ao, _, circ_o = oracle.solve(pr, mesh)
    P = kernels.Static2DProblem(**kw)
    assert kw["problem_type"] == kernels.XFK_AXISYMMETRIC
    P.solve()
    A = P.solution()
    es, eb = _system_err(P, pr, mesh)
    circ = P.circuits()
    P.close()
    Ac = converged(pr, mesh)
    assert es <= TOL_SYSTEM and eb <= TOL_SYSTEM, (es, eb)
    assert_parity(A, Ao, Ac, TOL_LINEAR)
    if variant == "circuit":
        assert circ[0][0] == circ_o[0][0]
        assert abs(circ[1][0] - circ_o[0][1]) <= 1e-12 * abs(circ_o[0][1])


@pytest.mark.parametrize("reuse", [True, False])
def test_nonlinear_matches_oracle(reuse):
    pr, mesh, kw = synth_to_oracle(synth.axisymmetric(32, nonlinear=True))
    Ao, st, _ = oracle.solve(pr, mesh)
    P = kernels.Static2DProblem(**kw, amg_reuse=reuse)
    r = P.solve()
    A = P.solution()
    P.close()
    Ac = converged(pr, mesh)
    assert r["newton_iters"] >= 3
    assert_parity(A, Ao, Ac, TOL_NONLINEAR)


def test_jacobi_preconditioner():
    pr, mesh, kw = synth_to_oracle(synth.axisymmetric(24))
    Ao, _, _ = oracle.solve(pr, mesh)
    P = kernels.Static2DProblem(**kw, precond="jacobi")
    P.solve()
    A = P.solution()
    P.close()
    assert rel_err(A, Ao) <= TOL_LINEAR


def test_sharded_axisymmetric():
    import threading
    kw = synth.axisymmetric(40)
    P = kernels.Static2DProblem(**kw)
    P.solve()
    A1 = P.solution()
    P.close()
    comms = kernels.Comm.local_group(3)
    probs = [kernels.Static2DProblem(**kw, comm=comms[q]) for q in range(3)]
    out = [None] * 3

    def work(q):
        probs[q].solve()
        out[q] = probs[q].solution()

    th = [threading.Thread(target=work, args=(q,)) for q in range(3)]
    for t in th:
        t.start()
    for t in th:
        t.join()
    for p in probs:
        p.close()
    for c in comms:
        c.close()
    for A in out:
        assert rel_err(A, A1) <= TOL_LINEAR


def test_fem_file_interface(tmp_path):
    """.fem with [ProblemType] = axisymmetric through the C++ FSolver host:
    the .ans carries the oracle's flux 2 pi r A (same Cuthill-McKee order)."""
    from oracle import femfile
    from xfemm_amd import fsolver
    kw = synth.axisymmetric(24, external=True)
    base = str(tmp_path / "axi")
    synth.write_problem(base, kw)
    pr, mesh = femfile.load_problem(base)
    assert pr.ProblemType == 1 and pr.extRo == kw["ext_ro"]
    Ao, _, _ = oracle.solve(pr, mesh)
    fs = fsolver.FSolver()
    fs.PathName = base
    assert fs.LoadProblemFile()
    assert fs.runSolver(False), fs.last_error()
    ans = femfile.read_ans(base + ".ans")
    assert rel_err(ans.A, Ao) <= TOL_LINEAR
    assert np.array_equal(ans.p, mesh.p) and np.array_equal(ans.lbl, mesh.lbl)
