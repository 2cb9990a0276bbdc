"""Magnetisation-direction functions (MagDirFctn) on the GPU.

The reference evaluates a label's Lua expression per element inside
FSolver::Static2D / StaticAxisymmetric (static2d.cpp:509-598,
staticaxi.cpp:350-410).  The device path evaluates it natively at problem
creation (xfk_magdir.cpp, bit-identical to the reference Lua: test_magdir.py)
and gives each such element its own direction; the oracle takes the
directions from the reference's own Lua (oracle/_ref/libreflua.so).

  * the reference fixture test/test_lua_mag_direction.fem ("theta" and
    "theta+180" magnets in an air disc): meshed by oracle/mesher.py, solved
    .fem -> .ans through FSolver on the GPU, A within 1e-6 of max |A| of the
    converged oracle.  The fixture has no boundary condition at all, so A is
    defined up to a constant: both sides are compared with their mean removed
    (the reference's own SSOR-PCG answer differs from the converged one by
    such a constant as well);
  * synthetic planar and axisymmetric magnets with functional directions vs the
    converged oracle (1e-6), and the reference's error text for an expression
    that does not evaluate.
"""
import os
import shutil

import numpy as np
import pytest

from oracle import femfile, mesher, oracle
from util import GOLDEN, assert_parity, converged, rel_err, synth_to_oracle
from xfemm_amd import fsolver, kernels, synth

pytestmark = [pytest.mark.gpu,
              pytest.mark.skipif(not oracle.ref_lua_available(), reason="oracle/_ref/libreflua.so not built")]

TOL = 1e-6


def centred(A):
    A = np.asarray(A)
    return A - A.mean()


def test_lua_mag_direction_fixture_fem_to_ans(tmp_path):
    src = os.path.join(GOLDEN, "test_lua_mag_direction.fem")
    base = str(tmp_path / "test_lua_mag_direction")
    shutil.copy(src, base + ".fem")
    mesher.write_mesh(mesher.mesh_problem(mesher.parse_geometry(src)), base)
    pr, mesh = femfile.load_problem(base)
    assert [lb.MagDirFctn for lb in pr.labels] == ["theta", "", "theta+180"] and not pr.bdrys
    fs = fsolver.FSolver(delete_mesh_files=False)
    fs.PathName = base
    assert fs.LoadProblemFile(), fs.last_error()
    assert fs.runSolver(False), fs.last_error()
    st = fs.stats()
    ans = femfile.read_ans(base + ".ans")
    assert np.array_equal(ans.p, mesh.p)
    Ac = converged(pr, mesh)
    err = rel_err(centred(ans.A), centred(Ac))
    print("fixture: %d nodes, %d PCG iterations, max|dA|/max|A| (mean removed) %.3e" % (len(mesh.x), st["cg_iters"], err))
    assert np.isfinite(ans.A).all()
    assert err <= TOL, err


def magnet_problem(fctn, axisymmetric=False, nonlinear=False):
    kw = synth.axisymmetric(40, nonlinear) if axisymmetric else synth.magnetostatic(40, nonlinear)
    kw = dict(kw)
    kw["labels"] = [dict(l) for l in kw["labels"]]
    mag = next(k for k, l in enumerate(kw["labels"]) if kw["blocks"][l["block"]].get("H_c", 0) > 0)
    kw["labels"][mag]["mag_dir_fctn"] = fctn
    return kw


@pytest.mark.parametrize("axi", [False, True])
@pytest.mark.parametrize("fctn", ["theta+90", "atan2(y-5,x-5)*180/PI", "x>5 and 30 or -60"])
def test_functional_magnet_matches_oracle(axi, fctn):
    pr, mesh, kw = synth_to_oracle(magnet_problem(fctn, axi))
    P = kernels.Static2DProblem(**kw)
    P.solve()
    A = P.solution()
    P.close()
    Ao, _, _ = oracle.solve(pr, mesh)
    Ac = converged(pr, mesh)
    assert_parity(A, Ao, Ac, TOL)
    # the direction really varies: the constant-direction answer is far away
    pr0, mesh0, kw0 = synth_to_oracle(magnet_problem("", axi))
    A0, _, _ = oracle.solve(pr0, mesh0)
    assert rel_err(A0, Ac) > 1e-3


def test_bad_function_is_refused_with_reference_text():
    kw = synth_to_oracle(magnet_problem("theta +"))[2]
    with pytest.raises(kernels.XfkError, match='Lua error occurred when evaluating:\n"theta \\+"'):
        kernels.Static2DProblem(**kw)
    kw = synth_to_oracle(magnet_problem("nil"))[2]
    with pytest.raises(kernels.XfkError, match='"nil" does not evaluate to a numerical value'):
        kernels.Static2DProblem(**kw)


@pytest.mark.parametrize("nranks", [3])
def test_functional_magnet_sharded(nranks):
    """Sharded: each rank uploads only the per-element label entries its own
    elements reference (renumbered); the answer is the single device's."""
    import threading
    kw = synth_to_oracle(magnet_problem("atan2(y-5,x-5)*180/PI"))[2]
    P = kernels.Static2DProblem(**kw)
    P.solve()
    A1 = P.solution()
    P.close()
    comms = kernels.Comm.local_group(nranks)
    probs = [kernels.Static2DProblem(**kw, comm=comms[q]) for q in range(nranks)]
    out = [None] * nranks

    def work(q):
        probs[q].solve()
        out[q] = probs[q].solution()

    th = [threading.Thread(target=work, args=(q,)) for q in range(nranks)]
    for t in th:
        t.start()
    for t in th:
        t.join()
    for p in probs:
        p.close()
    for c in comms:
        c.close()
    for A in out:
        assert A is not None and rel_err(A, A1) <= TOL


def test_label_without_elements_is_not_evaluated():
    """A MagDirFctn on a label that owns no element is never run by the
    reference (it evaluates per assembled element), so even an expression that
    would fail does not stop the problem."""
    kw = magnet_problem("")
    kw["labels"] = kw["labels"] + [dict(kw["labels"][0], mag_dir_fctn="theta +")]
    P = kernels.Static2DProblem(**synth_to_oracle(kw)[2])
    P.solve()
    P.close()


LUA_PROGRAMS = [
    # statements, a table traversed in the reference's order, a closure
    "call(function() local t = {x, y, 5} local s = 0 for k, v in t do s = s * 2 + v end return s end, {})",
    "call(function() local f = function(a) return a * %theta end return f(0.5) + 45 end, {})",
    # state carried from element to element (one interpreter per problem): a
    # linear problem runs the element loop once, so this is exact
    "call(function() cnt = (cnt or 0) + 1 return mod(cnt, 4) * 90 end, {})",
]


@pytest.mark.parametrize("fctn", LUA_PROGRAMS)
def test_lua_program_magnet_matches_oracle(fctn):
    """MagDirFctn as Lua programs (xfk_lua.cpp, pinned to the reference's
    liblua by tests/test_lua_interp.py) through problem creation: the
    oracle's directions come from the reference's liblua running the same
    element loop on one interpreter (oracle.element_magdir)."""
    pr, mesh, kw = synth_to_oracle(magnet_problem(fctn))
    P = kernels.Static2DProblem(**kw)
    P.solve()
    A = P.solution()
    P.close()
    Ao, _, _ = oracle.solve(pr, mesh)
    Ac = converged(pr, mesh)
    assert_parity(A, Ao, Ac, TOL)


def test_nonlinear_problem_refuses_a_stateful_chunk():
    """A nonlinear problem re-runs the element loop in every Newton pass: a
    chunk whose value depends on earlier runs is refused at creation (named,
    not a Lua error); a pure program is accepted."""
    kw = synth_to_oracle(magnet_problem("call(function() cnt = (cnt or 0) + 1 return cnt end, {})",
                                        nonlinear=True))[2]
    with pytest.raises(kernels.XfkError, match="not supported by the native Lua interpreter"):
        kernels.Static2DProblem(**kw)
    kw = synth_to_oracle(magnet_problem(LUA_PROGRAMS[0], nonlinear=True))[2]
    P = kernels.Static2DProblem(**kw)
    P.close()
