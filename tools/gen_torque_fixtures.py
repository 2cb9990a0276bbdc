"""Mesh the reference's TorqueBenchmark machine into committed test fixtures.

BASELINE.json configs[0] is ``test/TorqueBenchmark.fem`` run end-to-end; its
mesh must come from fmesher, which is not buildable here.  This
dev-time tool runs the fmesher restatement (oracle/mesher.py, driving the
reference's own Triangle compiled into oracle/_ref/libtriangle.so) on the
.fem (tests/golden/TorqueBenchmark.fem, a byte copy of the reference's
test/TorqueBenchmark.fem) and writes

  tests/golden/torque/TorqueBenchmark.node / .ele / .edge   the mesh
  tests/golden/torque/TorqueBenchmark_<deg>.pbc             periodic pairs + the
                         air-gap ring at rotor angle <deg> (InnerAngle of the
                         "AGE" boundary; femmcli_TorqueBenchmark.lua sweeps
                         0..90 in steps of 10 -- the mesh does not change)
  tests/golden/torque/TorqueBenchmark_fine.fem              configs[1]: the same
                         machine refined to ~200k triangles (label mesh sizes and
                         boundary-arc side lengths / 6.2, Precision 1e-8); meshed
                         at test time by the same restatement (~1 s)
  tests/golden/torque/TorqueBenchmark_fine_30.tgz           that mesh at rotor angle
                         30 (.fem .node .ele .edge .pbc, gzip): bench.py times the
                         product's FSolver .fem -> .ans on configs[1] from it (the
                         bench may not run the oracle's mesher)

Run in the dev container:  python tools/gen_torque_fixtures.py
"""
import os
import shutil
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from oracle import mesher  # noqa: E402

GOLDEN = os.path.join(ROOT, "tests", "golden")
OUT = os.path.join(GOLDEN, "torque")
ANGLES = list(range(0, 91, 10))
FINE_FACTOR = 6.2
FINE_PRECISION = "1e-008"


def fine_fem_text() -> str:
    src = open(os.path.join(GOLDEN, "TorqueBenchmark.fem")).read()
    txt = mesher.refine_fem_text(src, FINE_FACTOR)
    return txt.replace("[Precision]   =  1e-010", "[Precision]   =  " + FINE_PRECISION)


def main():
    os.makedirs(OUT, exist_ok=True)
    fem = os.path.join(GOLDEN, "TorqueBenchmark.fem")
    g = mesher.parse_geometry(fem)
    res = mesher.mesh_problem(g)
    base = os.path.join(OUT, "TorqueBenchmark")
    mesher.write_mesh(res, base)
    os.remove(base + ".pbc")
    for deg in ANGLES:
        with open(base + "_%d.pbc" % deg, "w") as fh:
            fh.write(mesher.pbc_text(res, {"AGE": (float(deg), 0.0)}))
    with open(base + "_fine.fem", "w") as fh:
        fh.write(fine_fem_text())
    # configs[1] at 30 degrees, packed for bench.py
    import tarfile
    import tempfile
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    from torque import write_fine_case
    with tempfile.TemporaryDirectory() as td:
        fb = write_fine_case(td, 30)
        with tarfile.open(os.path.join(OUT, "TorqueBenchmark_fine_30.tgz"), "w:gz") as tf:
            for ext in (".fem", ".node", ".ele", ".edge", ".pbc"):
                tf.add(fb + ext, arcname=os.path.basename(fb) + ext)
    print("TorqueBenchmark: %d nodes, %d triangles, %d periodic pairs, air gap of %d ring nodes (%s)"
          % (len(res.mesh.x), len(res.mesh.tri), len(res.pbc), res.ages[0].nodeNums[0], res.switches))


if __name__ == "__main__":
    main()
