"""Host stages of the product path (FSolver .fem -> .ans) on the configs[2]
mesh: XFEMM_TRACE_LOAD=1 stage marks on stderr, the get_times split on
stdout.  Run on the GPU box (its host share is what a user gets)."""
import os
import shutil
import sys
import tempfile
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
os.environ.setdefault("XFEMM_TRACE_LOAD", "1")
from xfemm_amd import fsolver, synth  # noqa: E402

cells = int(sys.argv[1]) if len(sys.argv) > 1 else 1000
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 3
with tempfile.TemporaryDirectory() as td:
    b = os.path.join(td, "sq")
    synth.write_problem(b, synth.magnetostatic(cells))
    src = b + "_src"
    os.makedirs(src)
    for ext in (".node", ".ele", ".edge", ".pbc"):
        shutil.copy(b + ext, os.path.join(src, "x" + ext))
    for rep in range(reps):
        for ext in (".node", ".ele", ".edge", ".pbc"):
            shutil.copy(os.path.join(src, "x" + ext), b + ext)
        print("---- rep %d" % rep, file=sys.stderr, flush=True)
        t0 = time.perf_counter()
        fs = fsolver.FSolver(device=0)
        fs.PathName = b
        ok = fs.LoadProblemFile() and fs.runSolver(False)
        dt = time.perf_counter() - t0
        print("rep %d ok %s wall %.1f ms %s" % (rep, ok, 1e3 * dt, {k: round(v, 1) for k, v in fs.times().items()}),
              flush=True)
        del fs
