"""AMG hints across problems (xfk_amg.hip HintStore): a fresh problem of the
size the last setup had takes that setup's SpGEMM capacities, MIS-2 round
counts and coarsest plan as speculation checked on the device.  The answer
must be bit-identical to a fully measured setup, and a capacity of the wrong
class must be refused (XFK_AMG_TEST_FOREIGN_BIG stores every capacity one
class too large: the device check sees no row needing more than half of it
and the hierarchy is rebuilt with measured capacities -- XFK_AMG_HINTS_PRINT
shows which capacities the finished setup holds).
"""
import numpy as np
import pytest

from xfemm_amd import kernels, synth

pytestmark = pytest.mark.gpu


def _fresh(kw, capfd):
    P = kernels.Static2DProblem(**kw, precond="amg")
    r = P.solve()
    A = P.solution()
    P.close()
    err = capfd.readouterr().err
    hints = [ln for ln in err.splitlines() if ln.startswith("[amg hints]")]
    return A, r, hints[-1]


def test_foreign_hints_keep_the_bits(capfd, monkeypatch):
    monkeypatch.setenv("XFK_AMG_HINTS_PRINT", "1")
    kw = synth.magnetostatic(200)
    kernels.forget_amg_hints()
    A1, r1, h1 = _fresh(kw, capfd)            # everything measured
    A2, r2, h2 = _fresh(kw, capfd)            # hints of the first problem
    assert np.array_equal(A1, A2) and r1["cg_iters"] == r2["cg_iters"]
    assert h1 == h2

    kernels.forget_amg_hints()
    monkeypatch.setenv("XFK_AMG_TEST_FOREIGN_BIG", "1")
    A3, _, h3 = _fresh(kw, capfd)             # measured; stores capacities one class too large
    A4, _, h4 = _fresh(kw, capfd)             # refused on the device, rebuilt
    assert h3 == h1 and h4 == h1, (h1, h4)
    assert np.array_equal(A3, A1) and np.array_equal(A4, A1)
    kernels.forget_amg_hints()


def test_foreign_hints_across_materials_and_sizes(capfd, monkeypatch):
    """Hints of another problem of the same size (other permeabilities, same
    mesh) and of a problem of another size (not taken) leave every answer as
    a cold setup gives it."""
    monkeypatch.setenv("XFK_AMG_HINTS_PRINT", "1")
    kw_a = synth.magnetostatic(160)
    kw_b = synth.magnetostatic(160, nonlinear=True)
    kw_c = synth.magnetostatic(120)
    cold = {}
    for name, kw in (("a", kw_a), ("b", kw_b), ("c", kw_c)):
        kernels.forget_amg_hints()
        cold[name] = _fresh(kw, capfd)
    kernels.forget_amg_hints()
    for name, kw in (("a", kw_a), ("b", kw_b), ("c", kw_c), ("a", kw_a)):
        A, r, h = _fresh(kw, capfd)
        assert np.array_equal(A, cold[name][0]), name
        assert r["cg_iters"] == cold[name][1]["cg_iters"], name
    kernels.forget_amg_hints()
