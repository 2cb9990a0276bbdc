"""FEASolver::SortElements on the device (xfk_sort_elements,
xfemm_amd/csrc/xfk_sort.hip) against the reference's comb sort
(cfemm/libfemm/cuthill.cpp:39-86) restated below, and against the host's
comb sort inside FSolver (XFEMM_HOST_SORT=1) on whole meshes: the same
permutation, bit for bit -- including the (unstable) order of equal scores."""
import os

import numpy as np
import pytest

from xfemm_amd import fsolver, kernels, synth

pytestmark = pytest.mark.gpu


def comb_sort_reference(score):
    """cuthill.cpp:39-86: gap = gap * 10 / 13 (9, 10 -> 11), swap on a strict
    decrease, `while ((gap > 1) && (i > 0))`: the first pass without a swap, or
    the first gap-1 pass, ends the sort (which then need not be sorted)."""
    sc = [int(v) for v in score]
    idx = list(range(len(sc)))
    n = len(sc)
    gap = n
    while True:
        if gap > 1:
            gap = (gap * 10) // 13
            if gap in (9, 10):
                gap = 11
        swapped = False
        for j in range(n - gap):
            if sc[j] > sc[j + gap]:
                sc[j], sc[j + gap] = sc[j + gap], sc[j]
                idx[j], idx[j + gap] = idx[j + gap], idx[j]
                swapped = True
        if not (gap > 1 and swapped):
            break
    return np.array(idx, dtype=np.int32)


@pytest.mark.parametrize("n,spread", [(2, 2), (3, 1), (17, 4), (1000, 50), (5000, 5000), (5000, 7),
                                      (70000, 300), (70000, 10 ** 6)])
def test_device_comb_sort_matches_reference(n, spread):
    rng = np.random.default_rng(n + spread)
    score = rng.integers(0, spread, n).astype(np.uint32)
    perm = kernels.sort_elements(score)
    ref = comb_sort_reference(score)
    assert np.array_equal(perm, ref)


def test_device_comb_sort_nearly_sorted_and_reversed():
    for score in (np.arange(40000, dtype=np.uint32)[::-1].copy(), (np.arange(40000) // 3).astype(np.uint32),
                  np.zeros(30000, dtype=np.uint32)):
        assert np.array_equal(kernels.sort_elements(score), comb_sort_reference(score))


def _renumber(base, host_sort):
    if host_sort:
        os.environ["XFEMM_HOST_SORT"] = "1"
    try:
        fs = fsolver.FSolver(delete_mesh_files=False)
        fs.PathName = base
        assert fs.LoadProblemFile() and fs.LoadMesh() and fs.Cuthill(), fs.last_error()
        return fs.elements()
    finally:
        os.environ.pop("XFEMM_HOST_SORT", None)


@pytest.mark.parametrize("cells,scramble", [(200, True), (1000, False)])
def test_fsolver_device_sort_equals_host_sort(tmp_path, cells, scramble):
    kw = synth.magnetostatic(cells)
    if scramble:
        rng = np.random.default_rng(11)
        nn, ne = len(kw["x"]), len(kw["p"])
        perm = rng.permutation(nn)
        inv = np.argsort(perm)
        eperm = rng.permutation(ne)
        kw = dict(kw, x=kw["x"][inv], y=kw["y"][inv], p=perm[kw["p"]][eperm].astype(np.int32),
                  lbl=kw["lbl"][eperm], e=kw["e"][eperm])
    base = str(tmp_path / "m")
    synth.write_problem(base, kw)
    dev = _renumber(base, False)
    host = _renumber(base, True)
    for a, b in zip(dev, host):
        assert np.array_equal(a, b)
