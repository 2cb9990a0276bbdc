"""TorqueBenchmark (BASELINE configs[0] and configs[1]) end to end on the GPU.

.fem + mesh -> FSolver (libxfemm_fsolver.so, MI355X kernels) -> .ans, then:
  * A at every node vs the CONVERGED oracle (util.converged: the reference's
    algorithm at Precision 1e-13): <= 1e-6 of max |A| (linear problem; the
    plain distance to the oracle at the file's Precision is in the message);
  * the .ans air-gap section equals the oracle's renumbered AGE (the input of
    the reference post-processor's gap integrals);
  * the gap torque computed from the .ans the way mo_gapintegral("AGE", 0)
    does (oracle/gaptorque.py) passes the reference's own benchmark check
    (femmcli/test/femmcli_TorqueBenchmark.lua: |T - sin| <= 4.2e-5 N m and
    <= 0.006 %).
configs[1] is the same machine refined to ~200k triangles (meshed at test
time by oracle/mesher.py), Precision 1e-8.
"""
import numpy as np
import pytest

from oracle import femfile, gaptorque, oracle
from torque import ANGLES, torque_ok, write_case, write_fine_case
from util import assert_parity, converged
from xfemm_amd import fsolver

pytestmark = pytest.mark.gpu

TOL_A = 1e-6


def _gpu_solve(base):
    fs = fsolver.FSolver(delete_mesh_files=False)
    fs.PathName = base
    assert fs.LoadProblemFile(), fs.last_error()
    assert fs.runSolver(False), fs.last_error()
    st = fs.stats()
    return femfile.read_ans(base + ".ans"), st


def _check(base, deg):
    pr, mesh = femfile.load_problem(base)        # the oracle reads the files first (the solver deletes none here)
    ans, st = _gpu_solve(base)
    Ao, _, _ = oracle.solve(pr, mesh)
    Ac = converged(pr, mesh)
    assert np.array_equal(ans.p, mesh.p)         # same Cuthill-McKee numbering as the reference
    assert_parity(ans.A, Ao, Ac, TOL_A)
    (age,) = ans.ages
    (ref_age,) = mesh.ages
    assert np.array_equal(age["qn"], ref_age["qn"]) and np.array_equal(age["qw"], ref_age["qw"])
    for k in ("format", "ri", "ro", "total_arc_length", "inner_shift", "outer_shift"):
        assert age[k] == ref_age[k], k
    assert age["inner_angle"] == float(deg)
    tq = gaptorque.gap_dc_torque(age, ans.A, pr.Depth, pr.LengthUnits)
    tq_ref = gaptorque.gap_dc_torque(ref_age, Ao, pr.Depth, pr.LengthUnits)
    ok, diff, rel = torque_ok(tq, deg)
    assert ok, "GPU torque %.7f at %d deg: diff %.3e (%.4f %%); oracle %.7f" % (tq, deg, diff, rel, tq_ref)
    assert abs(tq - tq_ref) <= 1e-6, (tq, tq_ref)
    print("TorqueBenchmark %d deg: %d nodes, %d PCG iterations, torque %.7f" % (deg, len(mesh.x), st["cg_iters"], tq))
    assert st["cg_iters"] <= 40, st["cg_iters"]   # one linear solve (AMG-PCG to 1e-8)
    return st


@pytest.mark.parametrize("deg", ANGLES)
def test_torque_benchmark_configs0(tmp_path, deg):
    st = _check(write_case(tmp_path, deg), deg)
    assert st["cg_iters"] > 0


@pytest.mark.parametrize("deg", [30, 80])
def test_torque_benchmark_refined_configs1(tmp_path, deg):
    st = _check(write_fine_case(tmp_path, deg), deg)
    assert st["cg_iters"] > 0
