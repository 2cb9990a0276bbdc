"""Host side of the product (CPU only): C-ABI exports, the C++ FSolver's
.fem / mesh handling against the oracle restatement, synthetic meshes."""
import ctypes as C
import os
import re
import shutil

import numpy as np
import pytest

from oracle import femfile
from util import GOLDEN, ROOT
from xfemm_amd import fsolver, kernels, synth


def _declared(header):
    txt = open(os.path.join(ROOT, "include", header)).read()
    txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
    return sorted(set(re.findall(r"\b(xf(?:k|emm)_\w+)\s*\(", txt)) - {"xfemm_message_fn"})


@pytest.mark.parametrize("header,so", [("xfemm_kernels.h", kernels.KERNELS_SO),
                                       ("xfemm_fsolver.h", fsolver.FSOLVER_SO)])
def test_c_abi_library_exports_every_declared_symbol(header, so):
    names = _declared(header)
    assert names, header
    lib = C.CDLL(so)
    for nm in names:
        assert hasattr(lib, nm), nm
    exported = kernels.EXPORTED if header == "xfemm_kernels.h" else fsolver.EXPORTED
    assert sorted(exported) == names


def _copy_case(tmp_path, name="Temp"):
    for ext in (".fem", ".node", ".ele", ".edge", ".pbc"):
        shutil.copy(os.path.join(GOLDEN, name + ext), tmp_path / (name + ext))
    return str(tmp_path / name)


def test_host_fsolver_loads_like_the_reference(tmp_path):
    base = _copy_case(tmp_path)
    fs = fsolver.FSolver(delete_mesh_files=False)
    fs.PathName = base
    assert fs.LoadProblemFile()
    assert fs.LoadMesh()
    assert fs.Cuthill()
    pr, mesh = femfile.load_problem(base)
    x, y, m = fs.nodes()
    p, lbl, e = fs.elements()
    assert np.array_equal(x, mesh.x) and np.array_equal(y, mesh.y) and np.array_equal(m, mesh.marker)
    assert np.array_equal(p, mesh.p) and np.array_equal(lbl, mesh.lbl) and np.array_equal(e, mesh.e)
    assert np.array_equal(fs.pbcs(), mesh.pbc)
    assert fs.BandWidth == mesh.bandwidth
    B, H, S, mu = fs.block_bh(0)
    assert np.array_equal(B, pr.blocks[0].Bdata) and np.array_equal(S, pr.blocks[0].slope)
    assert mu == pr.blocks[0].mu_x


def test_host_fsolver_renumbers_large_scrambled_mesh_like_the_reference(tmp_path):
    """Cuthill-McKee and SortElements (cuthill.cpp) on an 80k-element mesh with
    scrambled node and element numbering -- large enough for the parallel
    comb-sort passes and neighbour ordering -- against the oracle's sequential
    restatement: the same node order, element order (equal-score elements
    included) and bandwidth."""
    from xfemm_amd import synth
    kw = synth.magnetostatic(200)
    rng = np.random.default_rng(7)
    nn, ne = len(kw["x"]), len(kw["p"])
    perm = rng.permutation(nn)          # node i -> new id perm[i]
    inv = np.argsort(perm)
    eperm = rng.permutation(ne)
    kw = dict(kw, x=kw["x"][inv], y=kw["y"][inv], p=perm[kw["p"]][eperm].astype(np.int32),
              lbl=kw["lbl"][eperm], e=kw["e"][eperm])
    base = str(tmp_path / "scr")
    synth.write_problem(base, kw)
    fs = fsolver.FSolver(delete_mesh_files=False)
    fs.PathName = base
    assert fs.LoadProblemFile() and fs.LoadMesh() and fs.Cuthill(), fs.last_error()
    pr, mesh = femfile.load_problem(base)
    x, y, m = fs.nodes()
    p, lbl, e = fs.elements()
    assert np.array_equal(x, mesh.x) and np.array_equal(y, mesh.y)
    assert np.array_equal(p, mesh.p) and np.array_equal(lbl, mesh.lbl) and np.array_equal(e, mesh.e)
    assert fs.BandWidth == mesh.bandwidth


def test_host_fsolver_deletes_mesh_files_like_the_reference(tmp_path):
    base = _copy_case(tmp_path)
    fs = fsolver.FSolver()          # deleteFiles = true, as runSolver's LoadMesh()
    fs.PathName = base
    assert fs.LoadProblemFile() and fs.LoadMesh() and fs.Cuthill()
    for ext in (".node", ".ele", ".pbc", ".edge"):
        assert not os.path.exists(base + ext), ext
    assert os.path.exists(base + ".fem")


def test_host_fsolver_reports_missing_files(tmp_path):
    shutil.copy(os.path.join(GOLDEN, "Temp.fem"), tmp_path / "Temp.fem")
    fs = fsolver.FSolver(delete_mesh_files=False)
    fs.PathName = str(tmp_path / "Temp")
    assert fs.LoadProblemFile()
    assert not fs.LoadMesh()
    assert ".node" in fs.last_error()


def test_host_fsolver_rejects_bad_fem(tmp_path):
    (tmp_path / "bad.fem").write_text("[Format] = 4.0\n[Bogus] = 3\n")
    fs = fsolver.FSolver()
    fs.PathName = str(tmp_path / "bad")
    assert not fs.LoadProblemFile()
    assert "Unknown token" in fs.last_error()


def test_parsers_agree_on_torque_benchmark():
    """TorqueBenchmark.fem (reference test/): point props, periodic bdrys,
    magnets, circuits -- the C++ and the oracle parsers agree."""
    pr = femfile.prepare_problem(femfile.parse_fem(os.path.join(GOLDEN, "TorqueBenchmark.fem")))
    fs = fsolver.FSolver()
    fs.PathName = os.path.join(GOLDEN, "TorqueBenchmark")
    assert fs.LoadProblemFile()
    for k, m in enumerate(pr.blocks):
        B, H, S, mu = fs.block_bh(k)
        assert len(B) == m.BHpoints
        if m.BHpoints:
            assert np.array_equal(B, m.Bdata) and np.array_equal(S, m.slope) and mu == m.mu_x


def test_synthetic_mesh_is_valid():
    kw = synth.magnetostatic(16)
    x, y, p = kw["x"], kw["y"], kw["p"]
    assert len(x) == 17 * 17 and len(p) == 2 * 16 * 16
    area = ((x[p[:, 1]] - x[p[:, 0]]) * (y[p[:, 2]] - y[p[:, 0]]) -
            (x[p[:, 2]] - x[p[:, 0]]) * (y[p[:, 1]] - y[p[:, 0]])) / 2
    assert (area > 0).all()
    assert np.isclose(area.sum(), 100.0)
    # every boundary edge marked exactly once (4 sides x 16 edges)
    assert (kw["e"] == 0).sum() == 64
    assert set(np.unique(kw["lbl"])) == {0, 1, 2, 3, 4}


def test_synthetic_problem_roundtrips_through_fem_files(tmp_path):
    kw = synth.magnetostatic(6, nonlinear=True)
    base = str(tmp_path / "syn")
    synth.write_problem(base, kw)
    fs = fsolver.FSolver(delete_mesh_files=False)
    fs.PathName = base
    assert fs.LoadProblemFile() and fs.LoadMesh()
    x, y, m = fs.nodes()
    p, lbl, e = fs.elements()
    assert np.array_equal(p, kw["p"]) and np.array_equal(lbl, kw["lbl"]) and np.array_equal(e, kw["e"])
    assert np.allclose(x, kw["x"]) and np.allclose(y, kw["y"])
    B, H, S, mu = fs.block_bh(1)
    assert np.array_equal(B, kw["blocks"][1]["B"]) and np.array_equal(S, kw["blocks"][1]["slope"])


@pytest.mark.skipif(os.path.exists("/dev/kfd"), reason="GPU present")
def test_product_fails_loudly_without_gpu():
    kw = synth.magnetostatic(4)
    with pytest.raises(kernels.XfkError):
        kernels.Static2DProblem(**kw)


def test_host_loadmesh_odd_layouts_fall_back_to_the_token_stream(tmp_path):
    """Mesh files large enough for the line-parallel parser (> 2 MB) whose
    layout is not one record per line: a node record split over two lines, a
    blank line among the element records, an extra token after the last
    record of .node / .ele / .edge.  Such files are only read correctly by the
    sequential token stream fscanf sees (the parallel parser must detect them
    and fall back): the arrays equal the oracle's token-stream restatement of
    LoadMesh (oracle/femfile.py load_mesh)."""
    kw = synth.magnetostatic(300)
    base = str(tmp_path / "odd")
    synth.write_problem(base, kw)

    def edit(ext, fn):
        with open(base + ext) as fh:
            lines = fh.read().split("\n")
        fn(lines)
        with open(base + ext, "w") as fh:
            fh.write("\n".join(lines))

    def node_edit(ls):
        k = 1 + len(ls) // 2
        f = ls[k].split()
        ls[k] = "\t".join(f[:2])               # index and x ...
        ls.insert(k + 1, "\t".join(f[2:]))     # ... y and marker on the next line
        ls[-2] += "\t17"                       # a token after the last record

    def ele_edit(ls):
        ls.insert(1 + len(ls) // 3, "")        # a blank line among the records
        ls.insert(1 + len(ls) // 3, "   \t ")
        ls[-2] += " 99"

    def edge_edit(ls):
        ls[-2] += "\t5"

    edit(".node", node_edit)
    edit(".ele", ele_edit)
    edit(".edge", edge_edit)
    for ext in (".node", ".ele", ".edge"):
        assert os.path.getsize(base + ext) > (2 << 20), ext
    fs = fsolver.FSolver(delete_mesh_files=False)
    fs.PathName = base
    assert fs.LoadProblemFile() and fs.LoadMesh(), fs.last_error()
    pr = femfile.prepare_problem(femfile.parse_fem(base + ".fem"))
    mesh = femfile.load_mesh(base, pr)
    x, y, m = fs.nodes()
    p, lbl, e = fs.elements()
    assert np.array_equal(x, mesh.x) and np.array_equal(y, mesh.y) and np.array_equal(m, mesh.marker)
    assert np.array_equal(p, mesh.p) and np.array_equal(lbl, mesh.lbl) and np.array_equal(e, mesh.e)
    # and the plain files parse to the same arrays through the parallel path
    base2 = str(tmp_path / "plain")
    synth.write_problem(base2, kw)
    fs2 = fsolver.FSolver(delete_mesh_files=False)
    fs2.PathName = base2
    assert fs2.LoadProblemFile() and fs2.LoadMesh()
    x2, y2, m2 = fs2.nodes()
    p2, lbl2, e2 = fs2.elements()
    assert np.array_equal(x2, x) and np.array_equal(y2, y) and np.array_equal(p2, p) and np.array_equal(e2, e)
