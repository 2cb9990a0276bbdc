"""Lab: the cold path of a fresh problem (creation stages, first vs repeated
solve, the AMG hints a setup measures).  Run with XFK_TRACE_CREATE=1
XFK_AMG_HINTS_PRINT=1 to get the stage / hint lines on stderr.
Usage: python tools/lab/cold_probe.py [cells ...]"""
import ctypes
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
from xfemm_amd import kernels, synth  # noqa: E402


def sync():
    ctypes.CDLL("libamdhip64.so").hipDeviceSynchronize()


def main():
    cells = [int(a) for a in sys.argv[1:]] or [1000]
    kernels.load_library()
    for n in cells:
        kw = synth.magnetostatic(n)
        for rep in range(2):
            sync()
            t0 = time.perf_counter()
            D, keep = kernels._make_desc(kw["x"], kw["y"], kw["p"], kw["lbl"], kw["blocks"], kw["labels"],
                                         kw.get("lines", ()), kw.get("points", ()), kw.get("circuits", ()),
                                         kw.get("marker"), kw.get("e"), kw.get("pbc"), kw["precision"],
                                         kw["length_units"], kw.get("coords", 0), kw.get("relax", 1.0))
            t1 = time.perf_counter()
            kernels.alloc_stats(reset=True)
            P = kernels.Static2DProblem(**kw)
            sync()
            a_create = kernels.alloc_stats(reset=True)
            t2 = time.perf_counter()
            r1 = P.solve(rebuild_symbolic=True)
            sync()
            a_first = kernels.alloc_stats(reset=True)
            t3 = time.perf_counter()
            r2 = P.solve(rebuild_symbolic=True)
            sync()
            a_rep = kernels.alloc_stats(reset=True)
            t4 = time.perf_counter()
            for tag, a in (("create", a_create), ("first", a_first), ("repeat", a_rep)):
                print("  allocs %-6s: %d hipMalloc %.2f ms, %d hipFree %.2f ms"
                      % (tag, a["n_malloc"], a["ms_malloc"], a["n_free"], a["ms_free"]), flush=True)
            print("cells %d rep %d: desc %.1f ms, create %.1f ms (incl. desc), first solve %.2f ms (setup %.2f, "
                  "symbolic %.2f, pcg %d), repeat %.2f ms (setup %.2f)"
                  % (n, rep, 1e3 * (t1 - t0), 1e3 * (t2 - t1), 1e3 * (t3 - t2), r1["ms_amg_setup"],
                     r1["ms_symbolic"], r1["cg_iters"], 1e3 * (t4 - t3), r2["ms_amg_setup"]), flush=True)
            P.close()
            del keep, D


if __name__ == "__main__":
    main()
