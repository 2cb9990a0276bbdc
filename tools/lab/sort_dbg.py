import os, sys, time
import numpy as np
sys.path.insert(0, os.getcwd()); sys.path.insert(0, os.path.join(os.getcwd(), "tests"))
from xfemm_amd import fsolver, kernels, synth
from test_gpu_sort import comb_sort_reference
import tempfile
td = tempfile.mkdtemp()
kw = synth.magnetostatic(200)
rng = np.random.default_rng(11)
nn, ne = len(kw["x"]), len(kw["p"])
perm = rng.permutation(nn); inv = np.argsort(perm); eperm = rng.permutation(ne)
kw = dict(kw, x=kw["x"][inv], y=kw["y"][inv], p=perm[kw["p"]][eperm].astype(np.int32), lbl=kw["lbl"][eperm], e=kw["e"][eperm])
base = td + "/m"
synth.write_problem(base, kw)
os.environ["XFEMM_SORT_DUMP"] = td + "/scores.bin"
fs = fsolver.FSolver(delete_mesh_files=False); fs.PathName = base
assert fs.LoadProblemFile() and fs.LoadMesh() and fs.Cuthill()
sc = np.fromfile(td + "/scores.bin", dtype=np.uint32)
print("n", len(sc), "max", sc.max(), "dtype ok")
t = time.perf_counter(); pd = kernels.sort_elements(sc); print("device %.1f ms" % (1e3 * (time.perf_counter() - t)))
t = time.perf_counter(); pd = kernels.sort_elements(sc); print("device %.1f ms" % (1e3 * (time.perf_counter() - t)))
pr = comb_sort_reference(sc)
print("device == reference:", np.array_equal(pd, pr), "sorted:", (np.diff(sc[pd].astype(np.int64)) >= 0).all())
bad = np.nonzero(pd != pr)[0]
print("mismatch count", len(bad), bad[:10])
os.environ["XFEMM_HOST_SORT"] = "1"
fs2 = fsolver.FSolver(delete_mesh_files=False); fs2.PathName = base
assert fs2.LoadProblemFile() and fs2.LoadMesh() and fs2.Cuthill()
p2 = fs2.elements()[0]
p1 = fs.elements()[0]
# host order: reconstruct permutation via scores? compare element arrays
print("fsolver device vs host elements equal:", np.array_equal(p1, p2))
# reference-order elements from scores: need pre-sort elements; recompute from p1 sets
os.environ.pop("XFEMM_HOST_SORT", None)
os.environ["XFEMM_SORT_DUMP_P"] = td + "/p.bin"
fs3 = fsolver.FSolver(delete_mesh_files=False); fs3.PathName = base
assert fs3.LoadProblemFile() and fs3.LoadMesh() and fs3.Cuthill()
ppre = np.fromfile(td + "/p.bin", dtype=np.int32).reshape(-1, 3)
print("pre scores == dumped:", np.array_equal(ppre.sum(1).astype(np.uint32), sc))
print("device fsolver == ppre[ref]:", np.array_equal(fs3.elements()[0], ppre[pr]))
print("host fsolver == ppre[ref]:", np.array_equal(p2, ppre[pr]))
hs = p2.sum(1)
print("host sorted:", (np.diff(hs) >= 0).all())
bad = np.nonzero((p2 != ppre[pr]).any(1))[0]
print("host mismatches", len(bad), bad[:10])
for T in (1, 2, 4, 8, 16):
    import subprocess
    r = subprocess.run([sys.executable, "-c", """
import os, sys, numpy as np
sys.path.insert(0, os.getcwd())
from xfemm_amd import fsolver
os.environ['XFEMM_HOST_SORT'] = '1'
fs = fsolver.FSolver(delete_mesh_files=False); fs.PathName = '%s'
assert fs.LoadProblemFile() and fs.LoadMesh() and fs.Cuthill()
np.save('%s/h%%d.npy' %% %d, fs.elements()[0])
""" % (base, td, T)], env=dict(os.environ, XFEMM_HOST_THREADS=str(T)))
    h = np.load(td + "/h%d.npy" % T)
    print("host T=%d == ref:" % T, np.array_equal(h, ppre[pr]), "mismatch rows", int((h != ppre[pr]).any(1).sum()))
