"""The AMG-preconditioned PCG (xfemm_amd/csrc/xfk_amg.hip) against the oracle.

The reference preconditions CBigLinProb::PCGSolve with SSOR
(cfemm/libfemm/spars.cpp:186-236); the device's default is a smoothed-
aggregation AMG V-cycle, with the same stopping test.  Tolerances as in
test_gpu_static2d.py: A within 1e-6 (linear) / 1e-5 (nonlinear) of max |A|.
"""
import numpy as np
import pytest
import scipy.sparse as sp
import scipy.sparse.linalg as sla

from oracle import oracle
from util import C_ANS, assert_parity, converged, rel_err, synth_to_oracle
from xfemm_amd import kernels, synth

pytestmark = pytest.mark.gpu

TOL_LINEAR = 1e-6
TOL_NONLINEAR = 1e-5


def _solve(kw, **opt):
    P = kernels.Static2DProblem(**kw, **opt)
    r = P.solve()
    A = P.solution()
    P.close()
    return A, r


def _solve_vs(kw, pr, mesh, **opt):
    """A, result and the converged oracle (util.converged) of one solve"""
    P = kernels.Static2DProblem(**kw, **opt)
    r = P.solve()
    A = P.solution()
    P.close()
    return A, r, converged(pr, mesh)


@pytest.mark.parametrize("cells,nonlinear", [(60, False), (50, True)])
def test_amg_matches_oracle(cells, nonlinear):
    pr, mesh, kw = synth_to_oracle(synth.magnetostatic(cells, nonlinear=nonlinear))
    Ao, st, _ = oracle.solve(pr, mesh)
    tol = TOL_NONLINEAR if nonlinear else TOL_LINEAR
    A, r, Ac = _solve_vs(kw, pr, mesh, precond="amg")
    assert r["precond"] == kernels.XFK_PRECOND_AMG and r["amg_levels"] >= 2
    assert_parity(A, Ao, Ac, tol)


@pytest.mark.parametrize("anti", [False, True])
def test_amg_periodic_boundaries(anti):
    pr, mesh, kw = synth_to_oracle(synth.bc_showcase(30, anti=anti, nonlinear=True))
    Ao, _, _ = oracle.solve(pr, mesh)
    A, r, Ac = _solve_vs(kw, pr, mesh, precond="amg")
    assert r["precond"] == kernels.XFK_PRECOND_AMG
    assert_parity(A, Ao, Ac, TOL_NONLINEAR)


def test_amg_iterations_nearly_mesh_independent():
    its = []
    for cells in (100, 400):
        kw = synth.magnetostatic(cells)
        A_amg, r_amg = _solve(kw, precond="amg")
        A_jac, r_jac = _solve(kw, precond="jacobi")
        assert rel_err(A_amg, A_jac) <= TOL_LINEAR
        assert r_amg["cg_iters"] * 10 < r_jac["cg_iters"]
        its.append(r_amg["cg_iters"])
    assert its[1] <= 2 * its[0] and its[1] <= 60, its


@pytest.mark.parametrize("sweeps", [1, 3])
def test_amg_sweep_counts(sweeps):
    pr, mesh, kw = synth_to_oracle(synth.magnetostatic(50))
    Ao, _, _ = oracle.solve(pr, mesh)
    A, r, Ac = _solve_vs(kw, pr, mesh, precond="amg", amg_sweeps=sweeps)
    assert_parity(A, Ao, Ac, TOL_LINEAR)


def test_amg_is_deterministic():
    kw = synth.magnetostatic(200)
    P = kernels.Static2DProblem(**kw, precond="amg")
    P.solve()
    A1 = P.solution()
    P.solve(rebuild_symbolic=True)
    A2 = P.solution()
    P.close()
    A3, _ = _solve(kw, precond="amg")
    assert np.array_equal(A1, A2) and np.array_equal(A1, A3)


def test_spgemm_capacity_overflow_rebuilds(monkeypatch):
    """The SpGEMMs of a setup take their slot capacity from the previous setup
    of the same call site without a host check; a product that no longer
    fits is detected in the kernel and the hierarchy is rebuilt with measured
    capacities.  XFK_AMG_TEST_SMALL_HINT stores too-small capacities, so every
    later setup overflows and rebuilds: the answer must not change."""
    kw = synth.magnetostatic(200)
    P = kernels.Static2DProblem(**kw, precond="amg")
    P.solve()
    A1 = P.solution()
    monkeypatch.setenv("XFK_AMG_TEST_SMALL_HINT", "1")
    for _ in range(3):
        r = P.solve(rebuild_symbolic=True)
        assert np.array_equal(P.solution(), A1)
    P.close()
    assert r["precond"] == kernels.XFK_PRECOND_AMG


def _laplace_random(n, seed, shift=1.0):
    """5-point operator with random positive conductances and a Dirichlet-like
    diagonal shift on the first row of nodes (SPD; shift = 0: pure Neumann,
    constants are the null space)."""
    rng = np.random.default_rng(seed)
    N = n * n
    idx = np.arange(N).reshape(n, n)
    rows, cols, vals = [], [], []
    diag = np.zeros(N)
    for a, b in [(idx[:, :-1], idx[:, 1:]), (idx[:-1, :], idx[1:, :])]:
        a = a.ravel()
        b = b.ravel()
        c = np.exp(rng.uniform(-3, 3, len(a)))
        rows += [a, b]
        cols += [b, a]
        vals += [-c, -c]
        np.add.at(diag, a, c)
        np.add.at(diag, b, c)
    diag[idx[0]] += shift
    rows.append(np.arange(N))
    cols.append(np.arange(N))
    vals.append(diag)
    M = sp.csr_matrix((np.concatenate(vals), (np.concatenate(rows), np.concatenate(cols))), shape=(N, N))
    M.sort_indices()
    return M


def test_amg_is_closer_to_the_exact_solution_than_the_reference():
    """Nonlinear steel, Precision 1e-8: the reference's SSOR-PCG answer carries
    slow-mode error; the AMG answer solves the final system to ~1e-7."""
    import scipy.sparse.linalg as spla
    from util import C_ANS
    pr, mesh, kw = synth_to_oracle(synth.bc_showcase(24, nonlinear=True))
    Ao, _, _ = oracle.solve(pr, mesh)
    P = kernels.Static2DProblem(**kw, precond="amg")
    P.solve()
    A = P.solution()
    rp, col, val, b = P.csr()
    M = sp.csr_matrix((val, col, rp), shape=(len(rp) - 1,) * 2)
    exact = spla.spsolve(M.tocsc(), b) * C_ANS
    P.close()
    assert rel_err(A, exact) <= 1e-6
    assert rel_err(A, exact) < rel_err(Ao, exact)


@pytest.mark.parametrize("n", [8, 150])
def test_standalone_amg_pcg(n):
    M = _laplace_random(n, 3)
    b = np.random.default_rng(1).standard_normal(M.shape[0])
    V, it, er = kernels.pcg_solve_csr(M.indptr, M.indices, M.data, b, precision=1e-12, precond="amg")
    Vd = sla.spsolve(M.tocsc(), b)
    assert er <= 1e-12
    assert rel_err(V, Vd) <= 1e-8
    if n == 8:   # 64 rows: the whole matrix is the dense coarsest level (applied in f32)
        assert it <= 3


@pytest.mark.parametrize("n,nd", [(20, True), (30, True), (45, True), (45, False)])
def test_dense_coarsest_blocked_inverse(monkeypatch, n, nd):
    """n*n <= 2048 rows: the whole matrix is the dense coarsest level, inverted
    by blocked Gauss-Jordan (several 64-wide block columns, ragged last block):
    PCG converges in one step to the direct solution.  From 512 rows on the
    level is reordered by nested dissection (two parts eliminated side by
    side, then the separator); XFK_NO_ND=1 keeps the plain order.  The
    V-cycle applies the inverse rounded to f32, so each PCG step contracts the
    error by ~1e-7: three steps reach 1e-12."""
    if not nd:
        monkeypatch.setenv("XFK_NO_ND", "1")
    M = _laplace_random(n, 7)
    b = np.random.default_rng(2).standard_normal(M.shape[0])
    V, it, er = kernels.pcg_solve_csr(M.indptr, M.indices, M.data, b, precision=1e-12, precond="amg")
    Vd = sla.spsolve(M.tocsc(), b)
    assert it <= 3
    assert rel_err(V, Vd) <= 1e-10


def test_dense_coarsest_null_direction():
    """A pure-Neumann operator (no Dirichlet shift: constants are its null
    space) with a consistent right-hand side: the Gauss-Jordan inverse meets
    a vanishing pivot, zeroes that direction (generalised inverse on the
    range) and the PCG still solves the system."""
    M = _laplace_random(30, 11, shift=0.0)
    n = M.shape[0]
    b = np.random.default_rng(5).standard_normal(n)
    b -= b.mean()
    V, it, er = kernels.pcg_solve_csr(M.indptr, M.indices, M.data, b, precision=1e-10, precond="amg")
    assert np.all(np.isfinite(V))
    assert np.linalg.norm(M @ V - b) <= 1e-8 * np.linalg.norm(b)


def test_amg_without_couplings_uses_smoother_only():
    N = 1000
    rp = np.arange(N + 1, dtype=np.int32)
    col = np.arange(N, dtype=np.int32)
    val = np.linspace(1.0, 5.0, N)
    b = np.ones(N)
    V, it, er = kernels.pcg_solve_csr(rp, col, val, b, precision=1e-12, precond="amg")
    assert np.allclose(V, 1.0 / val, rtol=1e-10)


def test_precond_option_validation():
    kw = synth.magnetostatic(10)
    P = kernels.Static2DProblem(**kw)
    with pytest.raises(kernels.XfkError):
        P.set_option(kernels.XFK_OPT_PRECOND, 7)
    with pytest.raises(kernels.XfkError):
        P.set_option(kernels.XFK_OPT_AMG_SWEEPS, 0)
    for bad in (0.0, 2.0):   # the cycle is SPD only for 0 < omega < 2
        with pytest.raises(kernels.XfkError):
            P.set_option(kernels.XFK_OPT_AMG_OMEGA, bad)
    P.close()


@pytest.mark.parametrize("reuse", [False, True])
def test_newton_hierarchy_reuse(reuse):
    """Later Newton iterations keep the hierarchy of the first (fine-level
    smoother refreshed) or rebuild it: both reach the oracle's answer within
    the solver tolerance; reuse builds it once."""
    pr, mesh, kw = synth_to_oracle(synth.magnetostatic(32, nonlinear=True))
    Ao, st, _ = oracle.solve(pr, mesh)
    P = kernels.Static2DProblem(**kw, amg_reuse=reuse)
    r = P.solve()
    A = P.solution()
    P.close()
    Ac = converged(pr, mesh)
    assert r["newton_iters"] >= 3
    assert_parity(A, Ao, Ac, TOL_NONLINEAR)


@pytest.mark.parametrize("omega", [1.0, 1.9])
def test_jacobi_weight_factor(omega):
    """Any weight factor in (0, 2) gives an SPD cycle: same answer, within the
    solver tolerance of the oracle."""
    pr, mesh, kw = synth_to_oracle(synth.magnetostatic(40))
    Ao, _, _ = oracle.solve(pr, mesh)
    P = kernels.Static2DProblem(**kw, amg_omega=omega)
    P.solve()
    A = P.solution()
    P.close()
    Ac = converged(pr, mesh)
    assert_parity(A, Ao, Ac, TOL_LINEAR)


@pytest.mark.parametrize("cells,nonlinear", [(200, False), (60, True)])
def test_folded_cycle_equals_plain_cycle(cells, nonlinear):
    """The folded V(1,1) levels (XFK_OPT_AMG_FOLD, default on: one pass over
    P~ = (I - w D^-1 A) P for prolongation + post-sweep, coarse pre-steps with
    R~ = P~^T) equal the plain cycle in exact arithmetic.  Both answers meet
    the parity tolerance against the converged oracle, agree with each other
    to it, and take the same PCG iterations within one (roundoff only); the
    nonlinear case also runs the Newton refresh of the hierarchy (which runs
    level 0 unfolded, P~ belonging to the previous matrix)."""
    pr, mesh, kw = synth_to_oracle(synth.magnetostatic(cells, nonlinear=nonlinear))
    Ao, _, _ = oracle.solve(pr, mesh)
    tol = TOL_NONLINEAR if nonlinear else TOL_LINEAR
    Af, rf, Ac = _solve_vs(kw, pr, mesh, precond="amg", amg_fold=True)
    Ap, rp = _solve(kw, precond="amg", amg_fold=False)
    assert rf["precond"] == rp["precond"] == kernels.XFK_PRECOND_AMG
    assert_parity(Af, Ao, Ac, tol)
    assert_parity(Ap, Ao, Ac, tol)
    assert rel_err(Af, Ap) <= tol
    assert not np.array_equal(Af, Ap)                      # two different cycles really ran
    if nonlinear:
        assert rf["newton_iters"] == rp["newton_iters"] >= 3
        assert abs(rf["cg_iters"] - rp["cg_iters"]) <= rf["newton_iters"]
    else:
        assert abs(rf["cg_iters"] - rp["cg_iters"]) <= 1, (rf["cg_iters"], rp["cg_iters"])


def test_col16_tiles_are_bit_identical_with_wide_tile_fallback():
    """Level 0's 16-bit tile columns (XFK_OPT_AMG_COL16, default on) give the
    same bits as the int columns (f64 operator values in both, since the f32
    level-0 operators come with the 16-bit columns): once on the banded numbering (every tile
    fits: 2 B per nonzero) and once with the first half of the nodes in a
    random order (those tiles span > 65535 columns and read the int array:
    between 2 and 4 B per nonzero)."""
    kw = synth.magnetostatic(400)
    N = len(kw["x"])
    perm = np.arange(N)
    perm[: N // 2] = np.random.default_rng(5).permutation(N // 2)
    inv = np.argsort(perm)
    kws = dict(kw)
    kws["x"] = np.asarray(kw["x"])[inv]
    kws["y"] = np.asarray(kw["y"])[inv]
    kws["p"] = perm[np.asarray(kw["p"])]
    for k, lo, hi in ((kw, 2.0, 2.0), (kws, 2.05, 3.95)):
        out = []
        for c16 in (True, False):
            P = kernels.Static2DProblem(**k, precond="amg", amg_col16=c16, amg_f32=False)
            r = P.solve()
            out.append((P.solution(), r["cg_iters"], P.spmv_col_bytes()))
            if c16:
                rp, col, val, b = P.csr()
            P.close()
        (A1, i1, cb1), (A0, i0, cb0) = out
        assert lo <= cb1 <= hi, cb1
        assert cb0 == 4.0
        assert i1 == i0
        assert np.array_equal(A1.view(np.int64), A0.view(np.int64))
        M = sp.csr_matrix((val, col, rp), shape=(len(rp) - 1,) * 2)
        V = A1 / C_ANS
        assert np.linalg.norm(M @ V - b) <= 1e-5 * np.linalg.norm(b)


@pytest.mark.parametrize("cells,nonlinear", [(200, False), (60, True)])
def test_f32_level0_operators_meet_parity(cells, nonlinear):
    """The V-cycle's level-0 transfers with f32 values (XFK_OPT_AMG_F32,
    default on: R and P~; products and sums in f64, the sweeps and the PCG's
    SpMV in f64) change the preconditioner by f32 rounding only: both answers
    meet the parity tolerance against the converged oracle, agree with each
    other to it, take the same PCG iterations within one per Newton step, and
    the f32 path is deterministic (the nonlinear case also runs the Newton
    refresh of the hierarchy)."""
    pr, mesh, kw = synth_to_oracle(synth.magnetostatic(cells, nonlinear=nonlinear))
    Ao, _, _ = oracle.solve(pr, mesh)
    tol = TOL_NONLINEAR if nonlinear else TOL_LINEAR
    A32, r32, Ac = _solve_vs(kw, pr, mesh, precond="amg", amg_f32=True)
    A64, r64 = _solve(kw, precond="amg", amg_f32=False)
    A32b, _ = _solve(kw, precond="amg", amg_f32=True)
    assert_parity(A32, Ao, Ac, tol)
    assert_parity(A64, Ao, Ac, tol)
    assert rel_err(A32, A64) <= tol
    assert not np.array_equal(A32, A64)                    # the two precisions really ran
    assert np.array_equal(A32.view(np.int64), A32b.view(np.int64))
    assert r32["newton_iters"] == r64["newton_iters"]
    assert abs(r32["cg_iters"] - r64["cg_iters"]) <= r32["newton_iters"], (r32["cg_iters"], r64["cg_iters"])


@pytest.mark.parametrize("nonlinear", [False, True])
def test_w_cycle_level_meets_parity_in_fewer_iterations(nonlinear):
    """The W-cycle at the level above the last V-cycle level (default:
    a second coarse correction from the Galerkin coarse residual) is a
    symmetric preconditioner like the V-cycle: both answers meet the parity
    tolerance against the converged oracle, and the W-cycle takes no more
    PCG iterations."""
    pr, mesh, kw = synth_to_oracle(synth.magnetostatic(200, nonlinear=nonlinear))
    tol = TOL_NONLINEAR if nonlinear else TOL_LINEAR
    # a 256-row dense coarsest: four levels on this 40k-node mesh
    Aw, rw, Ac = _solve_vs(kw, pr, mesh, precond="amg", amg_dense=256)
    Av, rv = _solve(kw, precond="amg", amg_dense=256, amg_wlevel=-1)
    Ao, _, _ = oracle.solve(pr, mesh)
    assert rw["amg_levels"] >= 4, rw["amg_levels"]
    assert_parity(Aw, Ao, Ac, tol)
    assert_parity(Av, Ao, Ac, tol)
    assert not np.array_equal(Aw, Av)
    assert rw["cg_iters"] <= rv["cg_iters"], (rw["cg_iters"], rv["cg_iters"])


def test_amg_is_deterministic_through_newton_refreshes():
    """Repeated nonlinear solves (fresh builds + Newton refreshes of the
    hierarchy, folded levels) give the same bits."""
    kw = synth.magnetostatic(80, nonlinear=True)
    P = kernels.Static2DProblem(**kw, precond="amg")
    r1 = P.solve()
    A1 = P.solution()
    r2 = P.solve(rebuild_symbolic=True)
    A2 = P.solution()
    P.close()
    A3, r3 = _solve(kw, precond="amg")
    assert r1["newton_iters"] >= 3
    assert r1["cg_iters"] == r2["cg_iters"] == r3["cg_iters"]
    assert np.array_equal(A1, A2) and np.array_equal(A1, A3)


def test_high_contrast_f32_matches_f64_iterations():
    """Steel at mu_r 1e4 with a thin air gap through the core, Precision
    1e-10 (the coarse levels then carry condition numbers of 1e7 and more):
    the f32 parts of the V-cycle -- level-0 transfers, and the coarsest
    inverse rounded from its symmetrised unit-diagonal form -- need no more
    PCG iterations than the f64 cycle (within 2), both answers meet parity
    against the converged oracle, and no stagnation fallback is taken."""
    pr, mesh, kw = synth_to_oracle(synth.magnetostatic(160, mu_steel=1e4, precision=1e-10))
    Ao, _, _ = oracle.solve(pr, mesh)
    A32, r32, Ac = _solve_vs(kw, pr, mesh, precond="amg", amg_f32=True)
    A64, r64 = _solve(kw, precond="amg", amg_f32=False)
    print("mu_r 1e4, 1e-10: f32 %d, f64 %d PCG iterations" % (r32["cg_iters"], r64["cg_iters"]))
    assert r32["prec_fallback"] == 0 and r64["prec_fallback"] == 0
    assert r32["cg_iters"] <= r64["cg_iters"] + 2, (r32["cg_iters"], r64["cg_iters"])
    assert_parity(A32, Ao, Ac, TOL_LINEAR)
    assert_parity(A64, Ao, Ac, TOL_LINEAR)


def test_dense_coarsest_high_contrast_f32():
    """A 1600-row dense-coarsest matrix whose conductances span 1e12: the
    f32 inverse (symmetrised, unit-diagonal scaled) still converges to the
    direct solution within four PCG steps."""
    rng = np.random.default_rng(4)
    M = _laplace_random(40, 13)
    d = np.exp(rng.uniform(-14, 14, M.shape[0]))        # diagonal similarity: cond up to ~1e12
    M = (sp.diags(np.sqrt(d)) @ M @ sp.diags(np.sqrt(d))).tocsr()
    b = rng.standard_normal(M.shape[0])
    V, it, er = kernels.pcg_solve_csr(M.indptr, M.indices, M.data, b, precision=1e-12, precond="amg")
    Vd = sla.spsolve(M.tocsc(), b)
    assert it <= 4, it
    assert rel_err(V, Vd) <= 1e-9


def test_stagnation_falls_back_to_f64(monkeypatch):
    """The stagnation guard (XFK_TEST_F64_FALLBACK forces it at the first
    poll): the hierarchy is rebuilt with f64 transfers and an f64 coarsest
    inverse, the PCG restarts from its iterate, the answer meets parity and
    the fallback is reported (and kept for the problem's later solves)."""
    pr, mesh, kw = synth_to_oracle(synth.magnetostatic(120))
    Ao, _, _ = oracle.solve(pr, mesh)
    monkeypatch.setenv("XFK_TEST_F64_FALLBACK", "1")
    P = kernels.Static2DProblem(**kw)
    r = P.solve()
    A = P.solution()
    r2 = P.solve()
    P.close()
    Ac = converged(pr, mesh)
    assert r["prec_fallback"] == 1 and r2["prec_fallback"] == 1
    assert_parity(A, Ao, Ac, TOL_LINEAR)


def test_newton_refresh_refolds_level0(monkeypatch):
    """A Newton refresh keeps level 0 folded: P~ = (I - w D^-1 A) P re-formed
    numerically for the new matrix over its own pattern (k_refold_p).  The
    answer meets the nonlinear parity tolerance, is deterministic, is the same
    bit for bit when no row is staged in LDS (XFK_REFOLD_STAGE=0), and needs
    no more PCG iterations than the unfolded refresh (XFK_AMG_REFOLD=0) plus
    one per Newton step."""
    pr, mesh, kw = synth_to_oracle(synth.magnetostatic(80, nonlinear=True))
    Ao, _, _ = oracle.solve(pr, mesh)
    A1, r1, Ac = _solve_vs(kw, pr, mesh, precond="amg")
    A1b, _ = _solve(kw, precond="amg")
    monkeypatch.setenv("XFK_REFOLD_STAGE", "0")   # every row's products read from memory, same order
    A1m, _ = _solve(kw, precond="amg")
    monkeypatch.delenv("XFK_REFOLD_STAGE")
    monkeypatch.setenv("XFK_AMG_REFOLD", "0")
    A0, r0 = _solve(kw, precond="amg")
    print("refold: %d PCG / %d Newton; unfolded refresh: %d / %d"
          % (r1["cg_iters"], r1["newton_iters"], r0["cg_iters"], r0["newton_iters"]))
    assert_parity(A1, Ao, Ac, TOL_NONLINEAR)
    assert rel_err(A0, Ac) <= TOL_NONLINEAR
    assert np.array_equal(A1.view(np.int64), A1b.view(np.int64))
    assert np.array_equal(A1.view(np.int64), A1m.view(np.int64))
    assert r1["cg_iters"] <= r0["cg_iters"] + r1["newton_iters"], (r1["cg_iters"], r0["cg_iters"])


def test_bh_bisection_matches_the_knot_scan(monkeypatch):
    """The B-H interval lookup bisects non-decreasing tables instead of the
    reference's first-match scan (CMaterialProp.cpp:1039): the same
    knot interval for every B, so the nonlinear solve is the same bit for bit
    as with the scan forced (XFK_BH_SCAN)."""
    pr, mesh, kw = synth_to_oracle(synth.magnetostatic(80, nonlinear=True))
    A1, r1 = _solve(kw, precond="amg")
    monkeypatch.setenv("XFK_BH_SCAN", "1")
    A0, r0 = _solve(kw, precond="amg")
    assert r1["newton_iters"] == r0["newton_iters"] and r1["cg_iters"] == r0["cg_iters"]
    assert np.array_equal(A1.view(np.int64), A0.view(np.int64))


def test_newton_state_pass_matches_per_row_evaluation(monkeypatch):
    """A planar Newton pass evaluates each element's new state (B, GetBHProps,
    the permeabilities, dv) once (k_planar_state) for the three rows that
    gather the element, instead of once per row (XFK_ASM_STATE=0): the same
    arithmetic, so the same solve bit for bit."""
    pr, mesh, kw = synth_to_oracle(synth.magnetostatic(80, nonlinear=True))
    A1, r1 = _solve(kw, precond="amg")
    monkeypatch.setenv("XFK_ASM_STATE", "0")
    A0, r0 = _solve(kw, precond="amg")
    assert r1["newton_iters"] == r0["newton_iters"] and r1["cg_iters"] == r0["cg_iters"]
    assert np.array_equal(A1.view(np.int64), A0.view(np.int64))


def test_refold_threshold_unfolds_short_passes(monkeypatch):
    """A refresh re-forms P~ only when the last Newton pass ran at least
    XFK_REFOLD_MIN PCG iterations; below it level 0 runs unfolded for the pass.
    A threshold no pass reaches gives the always-unfolded solve bit for bit
    (XFK_AMG_REFOLD=0), and the parity tolerance either way."""
    pr, mesh, kw = synth_to_oracle(synth.magnetostatic(80, nonlinear=True))
    monkeypatch.setenv("XFK_REFOLD_MIN", "100000")
    A1, r1, Ac = _solve_vs(kw, pr, mesh, precond="amg")
    monkeypatch.delenv("XFK_REFOLD_MIN")
    monkeypatch.setenv("XFK_AMG_REFOLD", "0")
    A0, r0 = _solve(kw, precond="amg")
    assert rel_err(A1, Ac) <= TOL_NONLINEAR
    assert np.array_equal(A1.view(np.int64), A0.view(np.int64))
    # a threshold between the passes' counts: refreshes switch between folded
    # and unfolded level 0 within one Newton loop -- parity, and the same bits
    # on a repeat
    monkeypatch.delenv("XFK_AMG_REFOLD")
    counts = sorted(set([r1["cg_iters"] // max(1, r1["newton_iters"]), 3]))
    monkeypatch.setenv("XFK_REFOLD_MIN", str(counts[-1]))
    A2, r2 = _solve(kw, precond="amg")
    A2b, _ = _solve(kw, precond="amg")
    assert rel_err(A2, Ac) <= TOL_NONLINEAR
    assert np.array_equal(A2.view(np.int64), A2b.view(np.int64))


def test_lane_parallel_joins_select_the_same_aggregates(monkeypatch):
    """The aggregation joins take 4 / 8 lanes per row on the coarse levels
    (rows of 128-256 entries under the smoothed prolongator), each lane's
    candidate combined in the one-thread loop's own order: the same neighbour
    as one thread per row (XFK_JOIN_LANES=1), so the same hierarchy and the
    same solution bits."""
    kw = synth.magnetostatic(300)
    A, r = _solve(kw, precond="amg")
    monkeypatch.setenv("XFK_JOIN_LANES", "1")
    A1, r1 = _solve(kw, precond="amg")
    assert r["amg_levels"] >= 3
    assert (r1["cg_iters"], r1["amg_levels"]) == (r["cg_iters"], r["amg_levels"])
    assert np.array_equal(A.view(np.int64), A1.view(np.int64))
