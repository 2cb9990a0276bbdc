"""The oracle, pinned against the reference (CPU only).

* golden vectors: cfemm/fsolver/test/Temp.ans.check and Temp1.ans.check were
  written by the reference fsolver; the restated Static2D + CBigLinProb must
  reproduce their A column bit for bit (nonlinear steel, 3 Newton iterations,
  SSOR-PCG, periodic boundaries, serial circuits).  The third golden,
  cfemm/femmcli/test/femmcli_femfile.result.ans.check (femmcli_femfile.lua:
  the Temp problem through femmcli's own fmesher + fsolver), is read from its
  own .fem (Windows number formatting: "1e-008") and pinned the same way; its
  bytes equal Temp1.ans.check's (femmcli meshed the problem exactly as the
  fsolver test's Temp1 mesh), which the test records.
* the reference's own spars.cpp / CMaterialProp.cpp compiled into oracle/_ref
  (only where /root/reference was present at build time) must agree bit for
  bit with the restatement.
"""
import os

import numpy as np
import pytest

from oracle import ansmesh, femfile, oracle
from util import GOLDEN, synth_to_oracle
from xfemm_amd import synth

needs_ref = pytest.mark.skipif(not oracle.ref_available(), reason="oracle/_ref not built (reference absent)")


def _golden(name):
    pr = femfile.prepare_problem(femfile.parse_fem(os.path.join(GOLDEN, name + ".fem")))
    femfile.get_fill_factor(pr)
    mesh, sol = ansmesh.mesh_from_ans(os.path.join(GOLDEN, name + ".fem"),
                                      os.path.join(GOLDEN, name + ".ans.check"), pr)
    return pr, mesh, sol


@pytest.mark.parametrize("name", ["Temp", "Temp1", "femmcli_femfile"])
def test_oracle_reproduces_golden_ans_bit_exact(name):
    pr, mesh, sol = _golden(name)
    A, st, circ = oracle.solve(pr, mesh)
    assert st["newton_iters"] == 3
    assert np.array_equal(A, sol.A)
    # per-label circuit lines of the .ans (static2d.cpp:1122-1148)
    for k, lb in enumerate(pr.labels):
        case, J = (1, 0.0) if lb.InCircuit < 0 else (circ[lb.InCircuit][0], circ[lb.InCircuit][1])
        assert sol.circ[k][0] == case
        assert sol.circ[k][1] == J


def test_femmcli_golden_is_the_fsolver_temp1_golden():
    """femmcli_femfile.result.ans.check (fmesher + fsolver driven by femmcli)
    is byte for byte the fsolver test's Temp1.ans.check: the third reference
    golden pins the same mesh and A, reached from a differently formatted
    .fem (parsed by femfile and by the product's FSolver alike)."""
    a = open(os.path.join(GOLDEN, "femmcli_femfile.ans.check"), "rb").read()
    b = open(os.path.join(GOLDEN, "Temp1.ans.check"), "rb").read()
    assert a == b
    fa = open(os.path.join(GOLDEN, "femmcli_femfile.fem")).read()
    assert "1e-008" in fa


@needs_ref
@pytest.mark.parametrize("name", ["Temp", "Temp1", "femmcli_femfile"])
def test_restated_linprob_matches_reference_spars(name):
    pr, mesh, sol = _golden(name)
    A1, _, _ = oracle.solve(pr, mesh, "oracle")
    A2, _, _ = oracle.solve(pr, mesh, "reference")
    assert np.array_equal(A1, A2)


@needs_ref
def test_restated_linprob_matches_reference_on_mesh_files():
    pr, mesh = femfile.load_problem(os.path.join(GOLDEN, "Temp"))
    A1, st, _ = oracle.solve(pr, mesh, "oracle")
    A2, _, _ = oracle.solve(pr, mesh, "reference")
    assert np.array_equal(A1, A2)
    assert st["newton_iters"] >= 2


@needs_ref
@pytest.mark.parametrize("maker", ["showcase", "showcase_anti", "showcase_nl", "chain"])
def test_restated_linprob_matches_reference_boundary_paths(maker):
    kw = {"showcase": lambda: synth.bc_showcase(12),
          "showcase_anti": lambda: synth.bc_showcase(12, anti=True),
          "showcase_nl": lambda: synth.bc_showcase(12, nonlinear=True),
          "chain": lambda: synth.bc_chain(12)}[maker]()
    pr, mesh, _ = synth_to_oracle(kw)
    A1, _, _ = oracle.solve(pr, mesh, "oracle")
    A2, _, _ = oracle.solve(pr, mesh, "reference")
    assert np.array_equal(A1, A2)


def _block_text(path, index):
    """The index-th <BeginBlock>..<EndBlock> text of a .fem / matlib file."""
    txt = open(path).read()
    parts = txt.split("<BeginBlock>")
    body = parts[index + 1].split("<EndBlock>")[0]
    return "<BeginBlock>" + body + "<EndBlock>\n"


@needs_ref
@pytest.mark.parametrize("src,idx,lamfill", [("Temp.fem", 0, None), ("M19_Steel.block", 0, None),
                                             ("M19_Steel.block", 0, 0.9)])
def test_getslopes_matches_reference(src, idx, lamfill):
    import ctypes as C
    text = _block_text(os.path.join(GOLDEN, src), idx)
    if lamfill is not None:
        text = text.replace("<LamFill> = 0.97999999999999998", "<LamFill> = %r" % lamfill)
    R = oracle.ref()
    cap = 256
    B, H, S = np.zeros(cap), np.zeros(cap), np.zeros(cap)
    mu = C.c_double()
    n = R.ref_block_slopes(text.encode(), B.ctypes.data_as(oracle.dptr), H.ctypes.data_as(oracle.dptr),
                           S.ctypes.data_as(oracle.dptr), cap, C.byref(mu))
    assert n > 0
    # python restatement
    lines = femfile._Lines(text)
    m = femfile._parse_block(lines)
    femfile.get_slopes(m)
    assert np.array_equal(np.array(m.Bdata), B[:n])
    assert np.array_equal(np.array(m.Hdata), H[:n])
    assert np.array_equal(np.array(m.slope), S[:n])
    assert m.mu_x == mu.value
    # the product's C++ restatement (xfemm_bh_get_slopes)
    from xfemm_amd.fsolver import bh_get_slopes
    raw = femfile._parse_block(femfile._Lines(text))
    Bc, Hc, Sc, muc = bh_get_slopes(raw.Bdata, raw.Hdata, raw.LamType, raw.LamFill)
    assert np.array_equal(Bc, B[:n]) and np.array_equal(Hc, H[:n]) and np.array_equal(Sc, S[:n])
    assert muc == mu.value


@needs_ref
def test_bhprops_matches_reference():
    import ctypes as C
    text = _block_text(os.path.join(GOLDEN, "M19_Steel.block"), 0)
    m = femfile._parse_block(femfile._Lines(text))
    femfile.get_slopes(m)
    Bq = np.concatenate([[0.0, 1e-9, 0.05, 0.3], np.array(m.Bdata), np.linspace(0, 3.0, 301), [5.0]])
    v, dv = np.zeros(len(Bq)), np.zeros(len(Bq))
    R = oracle.ref()
    R.ref_block_bhprops(text.encode(), Bq.ctypes.data_as(oracle.dptr), len(Bq),
                        v.ctypes.data_as(oracle.dptr), dv.ctypes.data_as(oracle.dptr))
    keep = []
    blk = oracle.OraBlock()
    blk.mu_x, blk.BHpoints = m.mu_x, m.BHpoints
    for nm, arr in (("Bdata", m.Bdata), ("Hdata", m.Hdata), ("slope", m.slope)):
        a = np.array(arr)
        keep.append(a)
        setattr(blk, nm, a.ctypes.data_as(oracle.dptr))
    L = oracle.lib()
    for i, b in enumerate(Bq):
        vo, dvo = C.c_double(), C.c_double()
        L.ora_get_bh_props(C.byref(blk), b, C.byref(vo), C.byref(dvo))
        assert vo.value == v[i] and dvo.value == dv[i], b


def test_oracle_pcg_residual_small():
    """Size-independent property of the restated solver on a synthetic mesh."""
    kw = synth.magnetostatic(24)
    pr, mesh, _ = synth_to_oracle(kw)
    A, st, _ = oracle.solve(pr, mesh)
    K, b = oracle.system(pr, mesh)
    V = A / (np.pi * 4e-5)
    r = b - K @ V
    assert np.linalg.norm(r) <= 1e-6 * np.linalg.norm(b)
