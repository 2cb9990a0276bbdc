"""Problem creation stages (XFK_TRACE_CREATE=1) and the FSolver split on the
configs[1] TorqueBenchmark refinement, three runs in one process."""
import os
import shutil
import sys
import tarfile
import tempfile
import time

sys.path.insert(0, os.getcwd())
os.environ["XFK_TRACE_CREATE"] = "1"
os.environ["XFEMM_TRACE_LOAD"] = "1"
from xfemm_amd import fsolver  # noqa: E402

td = tempfile.mkdtemp()
with tarfile.open("tests/golden/torque/TorqueBenchmark_fine_30.tgz") as tf:
    tf.extractall(td)
base = os.path.join(td, "TorqueBenchmark_fine_30")
src = base + "_src"
os.makedirs(src)
for ext in (".node", ".ele", ".edge", ".pbc"):
    shutil.copy(base + ext, src)
for rep in range(3):
    for ext in (".node", ".ele", ".edge", ".pbc"):
        shutil.copy(os.path.join(src, os.path.basename(base) + ext), base + ext)
    print("---- rep %d" % rep, file=sys.stderr, flush=True)
    t0 = time.perf_counter()
    fs = fsolver.FSolver()
    fs.PathName = base
    ok = fs.LoadProblemFile() and fs.runSolver(False)
    dt = time.perf_counter() - t0
    print("rep %d ok %s wall %.1f ms %s" % (rep, ok, 1e3 * dt, {k: round(v, 1) for k, v in fs.times().items()}),
          file=sys.stderr, flush=True)
    del fs
