"""The product FSolver's renumbering (index work: bit-exact) against the
REFERENCE's own FEASolver::Cuthill + SortNodes + SortElements
(cfemm/libfemm/cuthill.cpp:33-391), compiled from /root/reference into
oracle/_ref/libref_cuthill.so by oracle/Makefile (oracle/ref_cuthill.cpp
#includes feasolver.cpp and cuthill.cpp as the reference's fsolver.cpp:55-56
does).  Both start from the product's LoadMesh arrays of the same mesh files;
the reference reads the .edge file itself.  Asserted array-equal: node order
(x, y, marker through newnum), element order (corners, labels, edge
properties, including the comb sort's unstable order of equal scores),
BandWidth, the remapped periodic pairs and air-gap quadNodes.

CPU: the product's host comb sort.  GPU (-m gpu): the same meshes through the
product's device comb sort (xfk_sort.hip), which FSolver takes whenever a
device is present."""
import os
import shutil
import tarfile

import numpy as np
import pytest

from oracle import oracle
from util import GOLDEN
from xfemm_amd import fsolver, kernels, synth

import torque

pytestmark = pytest.mark.skipif(not oracle.ref_cuthill_available(),
                                reason="oracle/_ref/libref_cuthill.so not built")


def _temp(tmp_path):
    for ext in (".fem", ".node", ".ele", ".edge", ".pbc"):
        shutil.copy(os.path.join(GOLDEN, "Temp" + ext), tmp_path / ("Temp" + ext))
    return str(tmp_path / "Temp")


def _torque(tmp_path):
    return torque.write_case(tmp_path, 30)


def _torque_fine(tmp_path):
    with tarfile.open(os.path.join(torque.TORQUE_DIR, "TorqueBenchmark_fine_30.tgz")) as tf:
        tf.extractall(tmp_path)
    return str(next(tmp_path.rglob("TorqueBenchmark_fine_30.fem")))[:-4]


def _scrambled(tmp_path, cells=200, seed=7):
    kw = synth.magnetostatic(cells)
    rng = np.random.default_rng(seed)
    nn, ne = len(kw["x"]), len(kw["p"])
    perm = rng.permutation(nn)
    inv = np.argsort(perm)
    eperm = rng.permutation(ne)
    kw = dict(kw, x=kw["x"][inv], y=kw["y"][inv], p=perm[kw["p"]][eperm].astype(np.int32),
              lbl=kw["lbl"][eperm], e=kw["e"][eperm])
    base = str(tmp_path / "scr")
    synth.write_problem(base, kw)
    return base


def _configs2(tmp_path):
    """BASELINE configs[2]: the bench's 2M-triangle mesh (synth.magnetostatic(1000))."""
    base = str(tmp_path / "c2")
    synth.write_problem(base, synth.magnetostatic(1000))
    return base


def islands(cells=(30, 20), seed=3):
    """Two disconnected square problems side by side, the second's node and
    element numbering scrambled and interleaved with the first's: Cuthill's
    restart for a multiply connected mesh (cuthill.cpp:267-301)."""
    a, b = synth.magnetostatic(cells[0]), synth.magnetostatic(cells[1])
    na = len(a["x"])
    rng = np.random.default_rng(seed)
    nb = len(b["x"])
    perm = rng.permutation(nb)
    inv = np.argsort(perm)
    x = np.concatenate([a["x"], b["x"][inv] + 12.0])
    y = np.concatenate([a["y"], b["y"][inv]])
    p = np.concatenate([a["p"], perm[b["p"]] + na]).astype(np.int32)
    lbl = np.concatenate([a["lbl"], b["lbl"]]).astype(np.int32)
    e = np.concatenate([a["e"], b["e"]]).astype(np.int32)
    order = rng.permutation(len(p))
    return dict(a, x=x, y=y, p=p[order], lbl=lbl[order], e=e[order])


def _islands(tmp_path):
    base = str(tmp_path / "isl")
    synth.write_problem(base, islands())
    return base


def _tiny(tmp_path):
    """The smallest mesh: one square cell, two triangles, four nodes."""
    base = str(tmp_path / "tiny")
    synth.write_problem(base, synth.magnetostatic(1))
    return base


def _isolated_node(tmp_path):
    """A node no element or edge uses (numcon 0: the reference's start node)."""
    kw = synth.magnetostatic(12)
    kw = dict(kw, x=np.append(kw["x"], 20.0), y=np.append(kw["y"], 20.0))
    base = str(tmp_path / "iso")
    synth.write_problem(base, kw)
    return base


CASES = {"temp": _temp, "torque": _torque, "torque_fine": _torque_fine, "scrambled80k": _scrambled,
         "configs2": _configs2, "islands": _islands, "tiny": _tiny, "isolated_node": _isolated_node}


def renumber_matches_reference(base):
    fs0 = fsolver.FSolver(delete_mesh_files=False)
    fs0.PathName = base
    assert fs0.LoadProblemFile() and fs0.LoadMesh(), fs0.last_error()
    x0, y0, m0 = fs0.nodes()
    p0, lbl0, e0 = fs0.elements()
    pbc0 = fs0.pbcs()
    cnt0, quad0 = fs0.air_gap_nodes()
    ref = oracle.ref_cuthill(base, fs0.NumNodes, p0, pbc0, cnt0, quad0)
    del fs0

    fs = fsolver.FSolver(delete_mesh_files=False)
    fs.PathName = base
    assert fs.LoadProblemFile() and fs.LoadMesh() and fs.Cuthill(), fs.last_error()
    x, y, m = fs.nodes()
    p, lbl, e = fs.elements()
    nn = newnum = ref["newnum"]
    assert np.array_equal(np.sort(nn), np.arange(len(nn)))
    order = ref["elem_order"]
    assert np.array_equal(p, ref["p"].reshape(-1, 3)), "element corners / order"
    assert np.array_equal(lbl, lbl0[order]) and np.array_equal(e, e0[order]), "element labels / edges"
    assert np.array_equal(x[newnum], x0) and np.array_equal(y[newnum], y0) and np.array_equal(m[newnum], m0)
    assert fs.BandWidth == ref["bandwidth"]
    pbc = fs.pbcs()
    assert np.array_equal(pbc[:, :2], ref["pbc"]) and np.array_equal(pbc[:, 2], pbc0[:, 2])
    cnt, quad = fs.air_gap_nodes()
    assert np.array_equal(cnt, cnt0) and np.array_equal(quad, ref["age_quad"])
    return dict(nodes=len(x), elements=len(p), pbcs=len(pbc), quad=len(quad), bandwidth=fs.BandWidth)


@pytest.mark.parametrize("case", ["temp", "torque", "torque_fine", "scrambled80k", "configs2", "islands", "tiny",
                                  "isolated_node"])
def test_host_renumbering_equals_reference_cuthill(tmp_path, case, monkeypatch):
    monkeypatch.setenv("XFEMM_HOST_SORT", "1")
    info = renumber_matches_reference(CASES[case](tmp_path))
    if case.startswith("torque"):
        assert info["pbcs"] > 0 and info["quad"] > 0


@pytest.mark.gpu
@pytest.mark.parametrize("case", ["temp", "torque", "torque_fine", "scrambled80k", "configs2", "islands", "tiny",
                                  "isolated_node"])
def test_device_sort_renumbering_equals_reference_cuthill(tmp_path, case, monkeypatch):
    monkeypatch.delenv("XFEMM_HOST_SORT", raising=False)
    assert kernels.device_count() > 0
    renumber_matches_reference(CASES[case](tmp_path))
