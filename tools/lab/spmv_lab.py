"""Dump the configs[2] system (2M-tri, assembled on the GPU) and run the SpMV
variant lab on it (dev tool).  Usage: python tools/lab/spmv_lab.py [cells]"""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402

from xfemm_amd import kernels, synth  # noqa: E402

cells = int(sys.argv[1]) if len(sys.argv) > 1 else 1000
P = kernels.Static2DProblem(**synth.magnetostatic(cells))
P.solve()
rp, col, val, b = P.csr()
P.close()
path = "/tmp/csr.bin"
with open(path, "wb") as f:
    np.array([len(rp) - 1, len(col)], np.int32).tofile(f)
    rp.astype(np.int32).tofile(f)
    col.astype(np.int32).tofile(f)
    val.astype(np.float64).tofile(f)
sys.exit(subprocess.call([os.path.join(ROOT, "xfemm_amd", "bin", "spmv_lab"), path]))
