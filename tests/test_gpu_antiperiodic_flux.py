"""The reference's antiperiodic flux check on the GPU (tests/antiperiodic.py;
cfemm/femmcli/test/femmcli_antiperiodicBC_flux.lua).

The nonlinear antiperiodic magnet machine is meshed by oracle/mesher.py and
solved .fem -> .ans through FSolver on the MI355X; then
  * A at every node within 1e-5 of max |A| of the converged oracle (the
    nonlinear parity tolerance);
  * |Bx| + |By| at the script's 45 points, from the GPU's .ans through the
    restated post-processor (oracle/pointvalues.py, fpproc's smoothed
    point values), within the script's margins of FEMM 4.2's values
    (0.02 T and 70 %).
"""
import numpy as np
import pytest

from antiperiodic import check, flux_post, write_case
from oracle import femfile, oracle
from util import assert_parity, converged, rel_err
from xfemm_amd import fsolver

pytestmark = pytest.mark.gpu

TOL_A = 1e-5


def test_antiperiodic_flux_machine_fem_to_ans(tmp_path):
    base = write_case(tmp_path)
    pr, mesh = femfile.load_problem(base)
    fs = fsolver.FSolver(delete_mesh_files=False)
    fs.PathName = base
    assert fs.LoadProblemFile(), fs.last_error()
    assert fs.runSolver(False), fs.last_error()
    st = fs.stats()
    ans = femfile.read_ans(base + ".ans")
    assert np.array_equal(ans.p, mesh.p)
    Ao, _, _ = oracle.solve(pr, mesh)
    Ac = converged(pr, mesh)
    err = rel_err(ans.A, Ac)
    failed, mx, mx_rel, rows = check(flux_post(pr, ans.x, ans.y, ans.A, ans.p, ans.lbl))
    print("antiperiodic flux: %d Newton / %d PCG iterations, A vs converged oracle %.3e; |B| check: %d failed, "
          "max diff %.4f T, %.1f %%" % (st["newton_iters"], st["cg_iters"], err, failed, mx, mx_rel))
    assert_parity(ans.A, Ao, Ac, TOL_A)
    assert failed == 0, [r for r in rows if r[-1]]
    # the AMG on the antiperiodic seam (signed strength: the seam's couplings of
    # the diagonal's sign are weak, so no aggregate spans it): at most 30 PCG
    # iterations per linear solve (round 3: ~100, 1200 over 12 Newton steps)
    assert st["cg_iters"] <= 30 * st["newton_iters"], (st["cg_iters"], st["newton_iters"])
