"""Lab: the antiperiodic flux machine (and TorqueBenchmark at 0 deg) through
FSolver with the Newton / AMG traces on (XFK_TRACE_NEWTON, XFK_AMG_DEBUG set by
the caller).  Usage: python tools/lab/anti_probe.py [anti] [torque]"""
import os
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
from xfemm_amd import fsolver  # noqa: E402

cases = sys.argv[1:] or ["anti", "torque"]
with tempfile.TemporaryDirectory() as tmp:
    for c in cases:
        if c == "anti":
            from antiperiodic import write_case
            base = write_case(tmp)
        else:
            from torque import write_case
            base = write_case(tmp, 0)
        fs = fsolver.FSolver(delete_mesh_files=False)
        fs.PathName = base
        ok = fs.LoadProblemFile() and fs.runSolver(False)
        st = fs.stats()
        print("%s: ok %s nodes %d newton %d pcg %d precond %d levels %d" % (
            c, ok, fs.NumNodes, st["newton_iters"], st["cg_iters"], st["precond"], st["amg_levels"]), flush=True)
        sys.stderr.flush()
