"""TorqueBenchmark (BASELINE configs[0]/[1]) on the CPU: mesh fixtures and the oracle.

* The committed mesh (tests/golden/torque) is what oracle/mesher.py -- the
  fmesher restatement over the reference's own Triangle -- makes of the
  reference's test/TorqueBenchmark.fem (regenerated and compared byte for byte
  when oracle/_ref/libtriangle.so is built).  Parity of the mesh with the
  reference's fmesher is unpinned (no reference mesh exists); what the
  reference does pin is the physics below.
* The oracle (restated Static2D + CBigLinProb, itself bit-exact to the
  reference's golden .ans files) solves the machine at every rotor angle of
  femmcli_TorqueBenchmark.lua and the reference post-processor's gap torque
  (oracle/gaptorque.py) passes that script's own check: |T - sin(angle)| <=
  4.2e-5 N m and <= 0.006 % (its comments record FEMM's worst errors as
  4.1e-5 at 80 deg and 0.0057 % at 10 deg; the oracle gives 4.08e-5 and
  0.0055 %).
"""
import os

import numpy as np
import pytest

from oracle import femfile, gaptorque, mesher, oracle
from torque import ANGLES, TORQUE_DIR, torque_ok, write_case
from util import GOLDEN


def _have_triangle():
    return os.path.exists(os.path.join(os.path.dirname(mesher.__file__), "_ref", "libtriangle.so"))


def _edge_set(path):
    with open(path) as fh:
        rows = [ln.split() for ln in fh.read().splitlines()[1:] if ln.strip()]
    return {(min(int(r[1]), int(r[2])), max(int(r[1]), int(r[2])), int(r[3])) for r in rows}


@pytest.mark.skipif(not _have_triangle(), reason="oracle/_ref/libtriangle.so not built (reference absent)")
def test_mesher_reproduces_committed_fixture(tmp_path):
    res = mesher.mesh_problem(mesher.parse_geometry(os.path.join(GOLDEN, "TorqueBenchmark.fem")))
    base = str(tmp_path / "tb")
    mesher.write_mesh(res, base, {"AGE": (30.0, 0.0)})
    for ext, ref in ((".node", "TorqueBenchmark.node"), (".ele", "TorqueBenchmark.ele"),
                     (".pbc", "TorqueBenchmark_30.pbc")):
        got, exp = open(base + ext).read(), open(os.path.join(TORQUE_DIR, ref)).read()
        same = got == exp      # (no assert on the strings: pytest's diff of 200 kB texts takes minutes)
        assert same, "%s differs: %d vs %d lines" % (ext, got.count("\n"), exp.count("\n"))
    # Triangle numbers edges by comparing triangle addresses (triangle.c
    # writeedges: `trisym.tri < triangleloop.tri`), so the .edge ORDER depends
    # on the heap; the set of (edge, marker) does not
    assert _edge_set(base + ".edge") == _edge_set(os.path.join(TORQUE_DIR, "TorqueBenchmark.edge"))
    assert res.switches == "-pPq33.000000eAazQIY"       # MinAngle 30 + MINANGLE_BUMP, exterior Steiner points off


def test_fixture_structure():
    """Periodic pairs on the two circles (pbc1 / pbc2), the AGE ring: 96 nodes
    per ring at 3.75 deg (the reference's (360/pi)(ro-ri)/(ro+ri) limit, 3.8 deg
    rounded), closed (n + 1 quadNodes, last = first)."""
    base = os.path.join(TORQUE_DIR, "TorqueBenchmark")
    with open(base + "_0.pbc") as fh:
        lines = fh.read().splitlines()
    npbc = int(lines[0])
    assert npbc == 360
    ages, _ = femfile._parse_age_blocks(lines, 2 + npbc, int(lines[1 + npbc]))
    (age,) = ages
    assert age["name"] == "AGE" and age["format"] == 0
    assert age["ri"] == 0.725 and age["ro"] == 0.775 and age["total_arc_length"] == 360
    assert age["qn"].shape == (97, 4)
    assert np.array_equal(age["qn"][0], age["qn"][-1])
    assert (age["qw"] == 1).all()


@pytest.mark.parametrize("deg", ANGLES)
def test_oracle_torque_passes_reference_benchmark(tmp_path, deg):
    base = write_case(tmp_path, deg)
    pr, mesh = femfile.load_problem(base)
    A, st, _ = oracle.solve(pr, mesh)
    tq = gaptorque.gap_dc_torque(mesh.ages[0], A, pr.Depth, pr.LengthUnits)
    ok, diff, rel = torque_ok(tq, deg)
    assert ok, "torque %.7f at %d deg: diff %.3e (%.4f %%)" % (tq, deg, diff, rel)


@pytest.mark.skipif(not _have_triangle(), reason="oracle/_ref/libtriangle.so not built (reference absent)")
def test_refined_machine_is_configs1_size():
    """configs[1]: TorqueBenchmark refined to ~200k triangles."""
    res = mesher.mesh_problem(mesher.parse_geometry(os.path.join(TORQUE_DIR, "TorqueBenchmark_fine.fem")))
    assert 190_000 <= len(res.mesh.tri) <= 210_000
    assert len(res.ages) == 1 and res.ages[0].nodeNums[0] == 192
