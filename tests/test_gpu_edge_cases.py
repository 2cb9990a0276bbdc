"""Edge cases of the static hot path on the GPU against the oracle (the
reference's algorithm): a multiply connected mesh (two islands, the second
numbered scrambled -- Cuthill's restart path, then one AMG hierarchy over both
components), the smallest meshes (every node on the Dirichlet boundary: the
reference's res_o = 0 early return, A = 0), and a node no element uses (a zero
row: the reference's "singular flag tripped", spars.cpp:245 -- the product
refuses it with XFK_ERR_SINGULAR instead of answering)."""
import numpy as np
import pytest

from oracle import femfile, oracle
from test_renumber_ref import islands
from util import assert_parity, converged, synth_to_oracle
from xfemm_amd import fsolver, kernels, synth

pytestmark = pytest.mark.gpu


def test_two_islands_in_memory_match_oracle():
    pr, mesh, kw = synth_to_oracle(islands())
    P = kernels.Static2DProblem(**kw)
    r = P.solve()
    A = P.solution()
    P.close()
    Ao, st, _ = oracle.solve(pr, mesh)
    assert_parity(A, Ao, converged(pr, mesh), 1e-6, " (%d PCG iterations)" % r["cg_iters"])


def test_two_islands_fem_to_ans_match_oracle(tmp_path):
    base = str(tmp_path / "isl")
    synth.write_problem(base, islands())
    pr, mesh = femfile.load_problem(base)         # (renumbered as the reference does)
    fs = fsolver.FSolver(delete_mesh_files=False)
    fs.PathName = base
    assert fs.LoadProblemFile() and fs.runSolver(False), fs.last_error()
    ans = femfile.read_ans(base + ".ans")
    assert np.array_equal(ans.p, mesh.p)
    Ao, _, _ = oracle.solve(pr, mesh)
    assert_parity(ans.A, Ao, converged(pr, mesh), 1e-6)


@pytest.mark.parametrize("cells", [1, 2])
def test_smallest_meshes_all_fixed(cells):
    pr, mesh, kw = synth_to_oracle(synth.magnetostatic(cells))
    P = kernels.Static2DProblem(**kw)
    P.solve()
    A = P.solution()
    P.close()
    Ao, st, _ = oracle.solve(pr, mesh)
    assert st["cg_iters"] == 0
    assert np.array_equal(A, Ao) and not A.any()


def test_unused_node_is_refused_as_singular():
    kw = synth.magnetostatic(12)
    kw = dict(kw, x=np.append(kw["x"], 20.0), y=np.append(kw["y"], 20.0))
    pr, mesh, kws = synth_to_oracle(kw)
    with pytest.raises(RuntimeError):             # the reference: "singular flag tripped"
        oracle.solve(pr, mesh)
    P = kernels.Static2DProblem(**kws)
    with pytest.raises(kernels.XfkError) as ei:
        P.solve()
    P.close()
    assert "singular" in str(ei.value).lower()
