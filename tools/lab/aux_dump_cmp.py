"""lab: compare the first Newton pass's auxiliary matrices (XFK_LAB_DUMP_AUX: a
temporary dump patched into harmonic2d_run for the round-5 probe, removed since)
single device vs row blocks, entry by entry in global numbering."""
import glob
import os
import sys

import numpy as np

_root = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "..")
sys.path[:0] = [_root, os.path.join(_root, "tests")]
kind, n, nr = sys.argv[1], int(sys.argv[2]), int(sys.argv[3])
pre = "/tmp/auxdump"
os.environ["XFK_LAB_DUMP_AUX"] = pre
from test_gpu_harmonic_sharded import run_sharded, single  # noqa: E402
from test_gpu_newton_ac import _case  # noqa: E402
from util import synth_to_oracle  # noqa: E402

kw = _case(kind, n)
_, _, kk = synth_to_oracle(kw)
for f in glob.glob(pre + "*"):
    os.remove(f)
single(kk)
run_sharded(kk, nr)


def load(fn):
    b = open(fn, "rb").read()
    hd = np.frombuffer(b, np.int32, 4)
    r, N, NL, nnz = (int(x) for x in hd)
    o = 16
    rp = np.frombuffer(b, np.int32, N + 1, o); o += 4 * (N + 1)
    cl = np.frombuffer(b, np.int32, nnz, o); o += 4 * nnz
    g = np.frombuffer(b, np.int32, NL, o); o += 4 * NL
    av = np.frombuffer(b, np.float64, 8 * nnz, o).reshape(8, nnz)
    o += 8 * 8 * nnz
    bv = np.frombuffer(b, np.float64, 4 * N, o)
    d = {}
    for i in range(N):
        d[("b", int(g[i]))] = np.array([bv[i], bv[N + i], bv[2 * N + 2 * i], bv[2 * N + 2 * i + 1], 0, 0, 0, 0])
    for i in range(N):
        for k in range(rp[i], rp[i + 1]):
            d[(int(g[i]), int(g[cl[k]]))] = av[:, k]
    return d


one = load(pre + "_r0of1.bin")
names = ["hr", "hi", "sr", "si", "ar", "ai", "val", "val_im"]
bnames = ["b", "b_im", "V", "V_im", "", "", "", ""]
sh = {}
for q in range(nr):
    sh.update(load(pre + "_r%dof%d.bin" % (q, nr)))
print("entries single %d sharded %d" % (len(one), len(sh)))
scale = np.max(np.abs(np.array([v for k, v in one.items() if k[0] != "b"])), axis=0)
bscale = np.max(np.abs(np.array([v for k, v in one.items() if k[0] == "b"])), axis=0)
bad = 0
for key in sorted(set(one) | set(sh), key=str):
    a = one.get(key, np.zeros(8))
    b = sh.get(key, np.zeros(8))
    dd = np.abs(a - b) / np.maximum(bscale if key[0] == "b" else scale, 1e-300)
    if dd.max() > (1e-6 if key[0] == "b" else 1e-9):
        bad += 1
        if bad <= 40:
            print(key, "missing" if key not in sh else ("extra" if key not in one else ""),
                  " ".join("%s %.6e/%.6e" % ((bnames if key[0] == "b" else names)[m], a[m], b[m]) for m in range(8) if dd[m] > 1e-9))
print("differing entries", bad)
