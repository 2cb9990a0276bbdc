"""Lab: the FSolver host path (LoadMesh, Cuthill-McKee, SortElements) on the
configs[2] mesh without a GPU -- XFEMM_TRACE_LOAD=1 prints the stages; the
run stops at problem creation when no device is present."""
import os
import shutil
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
from xfemm_amd import fsolver, synth  # noqa: E402

td = sys.argv[1] if len(sys.argv) > 1 else "/tmp/hp"
cells = int(sys.argv[2]) if len(sys.argv) > 2 else 1000
name = "square"
if cells == 0:   # configs[1]: the refined TorqueBenchmark fixture
    import tarfile
    name = "TorqueBenchmark_fine_30"
    with tarfile.open(os.path.join(ROOT, "tests", "golden", "torque", name + ".tgz")) as tf:
        tf.extractall(td)
base = os.path.join(td, name)
src = base + "_src"
if not os.path.exists(os.path.join(src, name + ".ele")):
    if cells:
        synth.write_problem(base, synth.magnetostatic(cells))
    os.makedirs(src, exist_ok=True)
    for ext in (".fem", ".node", ".ele", ".edge", ".pbc"):
        shutil.copy(base + ext, os.path.join(src, name + ext))
for it in range(3):
    for ext in (".node", ".ele", ".edge", ".pbc"):
        shutil.copy(os.path.join(src, name + ext), base + ext)
    t0 = time.perf_counter()
    fs = fsolver.FSolver(device=0)
    fs.PathName = base
    ok = fs.LoadProblemFile() and fs.runSolver(False)
    dt = time.perf_counter() - t0
    print("run %d ok=%s %.1f ms %s" % (it, ok, 1e3 * dt, fs.times()), flush=True)
    del fs
