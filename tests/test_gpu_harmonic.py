"""Time-harmonic planar path (xfemm_amd/csrc/xfk_harmonic.hip) against the
harmonic oracle (oracle/harmonic2d_oracle.c, itself bit-identical to the
reference's cspars.cpp -- tests/test_oracle_harmonic.py).

Tolerances (f64 / complex f64):
  * assembled complex system after all boundary conditions vs the oracle:
    max |diff| <= 1e-12 * max |A|  (element scatter order only)
  * A at every node: max |dA| <= 1e-6 * max |A| against the CONVERGED oracle
    (the reference's algorithm re-run at Precision 1e-13, util.converged):
    both stop at |r| / |b| <= Precision, the reference preconditioning COCG
    with SSOR, the device with the AMG V-cycle of the real surrogate
    Re A +- Im A, or complex Jacobi, so the iterates differ inside the
    reference's own stopping error; the plain distance to the oracle at the
    problem's Precision is reported in every message
  * the device solution solves its own system: |b - A V| / |b| <= 2 Precision
"""
import numpy as np
import pytest
import scipy.sparse as sp

from oracle import harmonic as oh
from util import C_ANS, assert_parity, converged, rel_err, synth_to_oracle
from xfemm_amd import kernels, synth

pytestmark = pytest.mark.gpu

TOL_SYSTEM = 1e-12
TOL_A = 1e-6


def _problem(kw):
    pr, mesh, kk = synth_to_oracle(kw)
    return pr, mesh, kk


@pytest.mark.parametrize("periodic", [False, True])
def test_harmonic_system_matches_oracle(periodic):
    pr, mesh, kk = _problem(synth.harmonic(20, periodic=periodic))
    P = kernels.Harmonic2DProblem(**kk)
    P.solve()
    rp, col, val, b = P.csr()
    n = len(rp) - 1
    G = sp.csr_matrix((val, col, rp), shape=(n, n))
    O, bo = oh.system(pr, mesh)
    scale = abs(O).max()
    assert abs(G - O).max() <= TOL_SYSTEM * scale
    assert np.abs(b - bo).max() <= TOL_SYSTEM * max(np.abs(bo).max(), 1e-300)
    P.close()


@pytest.mark.parametrize("cells,periodic", [(20, False), (24, True), (60, False)])
def test_harmonic_solution_matches_oracle(cells, periodic):
    pr, mesh, kk = _problem(synth.harmonic(cells, periodic=periodic))
    P = kernels.Harmonic2DProblem(**kk)
    r = P.solve()
    A = P.solution()
    Ao, st, circ_o = oh.solve(pr, mesh)
    rp, col, val, b = P.csr()
    n = len(rp) - 1
    G = sp.csr_matrix((val, col, rp), shape=(n, n))
    Ac = converged(pr, mesh, oh.solve)
    assert_parity(A, Ao, Ac, TOL_A)
    V = A / C_ANS
    assert np.linalg.norm(b - G @ V) / np.linalg.norm(b) <= 2 * kk["precision"]
    cc, J, dV = P.circuits()
    for k, (case, Jo, dVo) in enumerate(circ_o):
        assert cc[k] == case
        assert abs(J[k] - Jo) <= 1e-12 * max(1.0, abs(Jo)) and abs(dV[k] - dVo) <= 1e-12 * max(1.0, abs(dVo))
    assert r["cg_iters"] > 0
    P.close()


def test_harmonic_without_circuits_and_high_frequency():
    kw = synth.harmonic(30, frequency=2000.0, circuits=False)
    pr, mesh, kk = _problem(kw)
    P = kernels.Harmonic2DProblem(**kk)
    P.solve()
    A = P.solution()
    Ao, _, _ = oh.solve(pr, mesh)
    Ac = converged(pr, mesh, oh.solve)
    assert_parity(A, Ao, Ac, TOL_A)
    P.close()


def test_harmonic_unsupported_cases_are_reported():
    kw = synth.harmonic(10)
    kw["blocks"][1] = dict(kw["blocks"][1], LamType=1)
    with pytest.raises(kernels.XfkError, match="On-edge lamination"):
        kernels.Harmonic2DProblem(**kw)
    kw = synth.magnetostatic(10)
    with pytest.raises(kernels.XfkError):
        kernels.Harmonic2DProblem(**dict(kw, frequency=0.0))


@pytest.mark.parametrize("wiretype", [0, 1, 2, 3])
def test_harmonic_proximity_winding_matches_oracle(wiretype):
    """Wound region of a LamType 3 + wiretype block at 20 kHz: the element
    permeability is the label's ProximityMu (FSolver::GetFillFactor,
    fsolver.cpp:1083-1193; harmonic2d.cpp:664-668) and the region carries no
    bulk eddy current.  A vs the converged oracle; the winding moves the
    answer by > 10x the tolerance (the proximity term is exercised)."""
    kw = synth.harmonic(20, frequency=20000.0, prox=wiretype)
    pr, mesh, kk = _problem(kw)
    pm = pr.labels[3].ProximityMu
    assert abs(pm - 1) > 0.01 and kk["labels"][3]["prox_mu"] == pm
    P = kernels.Harmonic2DProblem(**kk)
    P.solve()
    A = P.solution()
    P.close()
    Ao, _, _ = oh.solve(pr, mesh)
    Ac = converged(pr, mesh, oh.solve)
    assert_parity(A, Ao, Ac, TOL_A)
    pr0, mesh0, _ = _problem(synth.harmonic(20, frequency=20000.0))
    A0 = converged(pr0, mesh0, oh.solve)
    assert rel_err(A0, Ac) > 10 * TOL_A


@pytest.mark.parametrize("wiretype", [1, 3])
def test_harmonic_axisymmetric_proximity_winding_matches_oracle(wiretype):
    """HarmonicAxisymmetric with the coil (a Case-1 circuit) wound of LamType
    3 + wiretype wire at 20 kHz (harmonicaxi.cpp:571-575): A vs the converged
    oracle, and the winding changes the answer."""
    kw = synth.harmonic_axisymmetric(16, frequency=20000.0, prox=wiretype)
    pr, mesh, kk = _problem(kw)
    assert abs(pr.labels[2].ProximityMu - 1) > 0.01
    P = kernels.Harmonic2DProblem(**kk)
    P.solve()
    A = P.solution()
    P.close()
    Ao, _, _ = oh.solve(pr, mesh)
    Ac = converged(pr, mesh, oh.solve)
    assert_parity(A, Ao, Ac, TOL_A)
    pr0, mesh0, _ = _problem(synth.harmonic_axisymmetric(16, frequency=20000.0))
    assert rel_err(converged(pr0, mesh0, oh.solve), Ac) > 10 * TOL_A


def test_harmonic_proximity_winding_file_interface(tmp_path):
    """.fem with a stranded-wire winding (LamType 4, WireD, NStrands, Turns)
    -> FSolver (its own GetFillFactor) on the GPU -> .ans, vs the oracle's
    restatement loaded from the same files."""
    from oracle import femfile
    from xfemm_amd import fsolver
    kw = synth.harmonic(18, circuits=False, frequency=20000.0, prox=1)
    kw["marker"] = None
    kw["points"] = []
    base = str(tmp_path / "hp")
    synth.write_problem(base, kw)
    pr, mesh = femfile.load_problem(base)
    assert pr.blocks[3].LamType == 4 and pr.labels[3].Turns == 30 and abs(pr.labels[3].ProximityMu - 1) > 0.1
    Ao, _, _ = oh.solve(pr, mesh)
    Ac = converged(pr, mesh, oh.solve)
    fs = fsolver.FSolver()
    fs.PathName = base
    assert fs.LoadProblemFile()
    assert fs.runSolver(False), fs.last_error()
    nodes, _ = _read_harmonic_ans(base + ".ans")
    A = nodes[:, 2] + 1j * nodes[:, 3]
    assert_parity(A, Ao, Ac, TOL_A)


@pytest.mark.parametrize("frequency", [60.0, 2000.0])
def test_harmonic_amg_preconditioner(frequency):
    """The V-cycle preconditioner reaches the same answer as complex Jacobi in
    a mesh-independent handful of iterations (the surrogate's sign follows Im A)."""
    kw = synth.harmonic(150, frequency=frequency, circuits=False)
    res = {}
    for pc in ("amg", "jacobi"):
        P = kernels.Harmonic2DProblem(**kw, precond=pc)
        r = P.solve()
        rp, col, val, b = P.csr()
        G = sp.csr_matrix((val, col, rp), shape=(len(rp) - 1,) * 2)
        V = P.solution() / C_ANS
        assert np.linalg.norm(b - G @ V) / np.linalg.norm(b) <= 2 * kw["precision"]
        res[pc] = (r, P.solution())
        P.close()
    ra, rj = res["amg"][0], res["jacobi"][0]
    assert ra["amg_levels"] >= 2 and rj["amg_levels"] == 0
    assert ra["cg_iters"] <= 80 and ra["cg_iters"] * 4 < rj["cg_iters"]
    assert rel_err(res["amg"][1], res["jacobi"][1]) <= 1e-6


def test_harmonic_repeatable():
    kw = synth.harmonic(40)
    P = kernels.Harmonic2DProblem(**kw)
    P.solve()
    A1 = P.solution()
    P.solve(rebuild_symbolic=True)
    A2 = P.solution()
    P.close()
    assert np.array_equal(A1, A2)


def _read_harmonic_ans(path):
    """Nodes (x, y, A re, A im, marker) and elements (p, lbl, e) of a
    WriteHarmonic2D .ans (harmonic2d.cpp:793-960)."""
    lines = open(path).read().splitlines()
    k = lines.index("[Solution]") + 1
    n = int(lines[k])
    nodes = np.array([[float(v) for v in ln.split()] for ln in lines[k + 1:k + 1 + n]])
    k += 1 + n
    ne = int(lines[k])
    els = np.array([[int(v) for v in ln.split()] for ln in lines[k + 1:k + 1 + ne]])
    return nodes, els


def test_harmonic_file_interface_end_to_end(tmp_path):
    """.fem (Frequency > 0) + fmesher files -> FSolver on the GPU -> harmonic .ans."""
    import os
    from oracle import femfile
    from xfemm_amd import fsolver
    kw = synth.harmonic(18, circuits=False)
    kw["marker"] = None
    kw["points"] = []
    base = str(tmp_path / "h")
    synth.write_problem(base, kw)
    pr, mesh = femfile.load_problem(base)
    assert pr.Frequency == kw["frequency"]
    Ao, _, _ = oh.solve(pr, mesh)
    fs = fsolver.FSolver()
    fs.PathName = base
    assert fs.LoadProblemFile()
    assert fs.runSolver(False), fs.last_error()
    nodes, els = _read_harmonic_ans(base + ".ans")
    A = nodes[:, 2] + 1j * nodes[:, 3]
    Ac = converged(pr, mesh, oh.solve)
    assert_parity(A, Ao, Ac, TOL_A)
    assert np.array_equal(els[:, :3], mesh.p) and np.array_equal(els[:, 3], mesh.lbl)
    assert open(base + ".ans").read().startswith(open(base + ".fem").read())


@pytest.mark.parametrize("cells", [10, 20, 40])
def test_harmonic_nonlinear_matches_oracle(cells):
    """Successive approximation of a nonlinear AC problem (M-19 steel on its
    GetSlopes(omega) curve: hysteresis lag, lamination eddy currents): A at
    every node vs the oracle (whose loop is bit-identical to the reference's
    cspars.cpp solver), within 1e-5 of max |A| -- both loops stop at
    |dV| / |V| < 100 Precision, from COCG solves that each stop at Precision
    with different preconditioners."""
    kw = synth.harmonic(cells, nonlinear=True)
    pr, mesh, kk = _problem(kw)
    Ao, st, _ = oh.solve(pr, mesh)
    P = kernels.Harmonic2DProblem(**kk)
    r = P.solve()
    A = P.solution()
    P.close()
    assert st["newton_iters"] > 1 and r["newton_iters"] > 1
    assert rel_err(A, Ao) <= 1e-5
    assert abs(r["newton_iters"] - st["newton_iters"]) <= max(3, st["newton_iters"] // 5)


def test_harmonic_nonlinear_file_interface_end_to_end(tmp_path):
    """.fem with a nonlinear laminated lossy steel (raw M-19 points, Sigma,
    d_lam, Phi_h) -> FSolver (GetSlopes(omega) on the host, successive
    approximation on the GPU) -> .ans, against the oracle."""
    from xfemm_amd import fsolver
    kw = synth.harmonic(16, circuits=False, nonlinear=True)
    kw["marker"] = None
    kw["points"] = []
    base = str(tmp_path / "hn")
    synth.write_problem(base, kw)
    from oracle import femfile
    pr, mesh = femfile.load_problem(base)   # the files' node order (as in the .ans)
    for m in pr.blocks:
        if m.BHpoints:   # the harmonic curve of the raw points (GetSlopes(omega))
            B, H, S, mu, _ = fsolver.bh_get_slopes_ac(*synth.m19_curve(), 2 * np.pi * pr.Frequency, m.LamType,
                                                      m.LamFill, m.Theta_hn, m.Lam_d, m.Cduct)
            m.Bdata, m.Hdata, m.slope, m.mu_x, m.mu_y = list(B), list(H), list(S), mu, mu
            m.Theta_hx = m.Theta_hy = m.Theta_hn
    Ao, st, _ = oh.solve(pr, mesh)
    assert st["newton_iters"] > 1
    fs = fsolver.FSolver()
    fs.PathName = base
    assert fs.LoadProblemFile()
    assert fs.runSolver(False), fs.last_error()
    nodes, _ = _read_harmonic_ans(base + ".ans")
    A = nodes[:, 2] + 1j * nodes[:, 3]
    assert rel_err(A, Ao) <= 1e-5


@pytest.mark.parametrize("cells,nonlinear,periodic", [(20, False, False), (36, False, False), (16, True, False),
                                                      (20, False, True), (30, False, "anti"), (16, True, True),
                                                      (16, True, "anti")])
def test_harmonic_case2_circuit_matches_oracle(cells, nonlinear, periodic):
    """Case-2 circuit (a specified total current in the conducting plate: its
    voltage gradient is an extra unknown, harmonic2d.cpp:441-472): the device
    solves the bordered system through its Schur complement; A and the
    circuit's voltage gradient against the oracle (which assembles the
    bordered system like the reference)."""
    kw = synth.harmonic(cells, nonlinear=nonlinear, periodic=bool(periodic), anti=periodic == "anti")
    kw["circuits"][1] = dict(type=0, amps_re=2.0, amps_im=0.5)
    pr, mesh, kk = _problem(kw)
    assert len(mesh.pbc) == (cells + 1 if periodic else 0)
    Ao, st, circ_o = oh.solve(pr, mesh)
    assert circ_o[1][0] == 2
    P = kernels.Harmonic2DProblem(**kk)
    P.solve()
    A = P.solution()
    cc, J, dV = P.circuits()
    P.close()
    tol = 1e-5 if nonlinear else 1e-6
    assert rel_err(A, Ao) <= tol
    assert cc[1] == 2 and abs(dV[1] - circ_o[1][2]) <= tol * abs(circ_o[1][2])
