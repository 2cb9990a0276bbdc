"""The reference's antiperiodic flux check on the CPU oracle (tests/antiperiodic.py):
the fixture meshed by oracle/mesher.py, solved by the oracle (the reference's
Static2D restated, bit-exact to the golden .ans files), |B| at the script's 45
points by the restated post-processor (oracle/pointvalues.py) -- every point
within the script's margins of FEMM 4.2's values.  This pins the mesher, the
oracle's nonlinear antiperiodic solve and the post-processor restatement that
the GPU test (test_gpu_antiperiodic_flux.py) then uses."""
import pytest

from antiperiodic import check, drawing_units, flux_post, write_case
from oracle import femfile, oracle


@pytest.mark.skipif(not oracle.ref_available(), reason="oracle/_ref not built (Triangle for the mesher)")
def test_oracle_passes_reference_flux_check(tmp_path):
    pr, mesh = femfile.load_problem(write_case(tmp_path))
    assert len(mesh.pbc) > 0 and any(b.BdryFormat == 5 for b in pr.bdrys)
    A, st, _ = oracle.solve(pr, mesh)
    assert st["newton_iters"] > 3
    x, y = drawing_units(mesh, pr.LengthUnits)
    failed, mx, mx_rel, rows = check(flux_post(pr, x, y, A, mesh.p, mesh.lbl))
    assert failed == 0, [r for r in rows if r[-1]]
