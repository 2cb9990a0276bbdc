"""ctypes driver for the C oracle (static2d_oracle.c) -- TEST INFRASTRUCTURE ONLY.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg import this.

``solve(pr, mesh, linprob="oracle"|"reference")`` runs the restated
FSolver::Static2D (cfemm/fsolver/static2d.cpp:53-1033) on the CPU, with the
linear algebra done either by the restated CBigLinProb or by the reference's
own spars.cpp compiled into oracle/_ref/libxfemm_ref.so.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess
from typing import Optional

import numpy as np

from . import femfile

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "_build", "liboracle.so")
REF_PATH = os.path.join(HERE, "_ref", "libxfemm_ref.so")
LUA_PATH = os.path.join(HERE, "_ref", "libreflua.so")
CUTHILL_PATH = os.path.join(HERE, "_ref", "libref_cuthill.so")

dptr = C.POINTER(C.c_double)
iptr = C.POINTER(C.c_int)


class OraBlock(C.Structure):
    _fields_ = [("mu_x", C.c_double), ("mu_y", C.c_double), ("H_c", C.c_double),
                ("J_re", C.c_double), ("Cduct", C.c_double), ("LamFill", C.c_double),
                ("LamType", C.c_int), ("BHpoints", C.c_int),
                ("Bdata", dptr), ("Hdata", dptr), ("slope", dptr)]


class OraLabel(C.Structure):
    _fields_ = [("InCircuit", C.c_int), ("MagDir", C.c_double), ("bIsWound", C.c_int), ("IsExternal", C.c_int)]


class OraLine(C.Structure):
    _fields_ = [("BdryFormat", C.c_int), ("A0", C.c_double), ("A1", C.c_double),
                ("A2", C.c_double), ("phi", C.c_double), ("c0", C.c_double), ("c1", C.c_double)]


class OraPoint(C.Structure):
    _fields_ = [("A_re", C.c_double), ("A_im", C.c_double), ("J_re", C.c_double),
                ("J_im", C.c_double)]


class OraCirc(C.Structure):
    _fields_ = [("CircType", C.c_int), ("Amps_re", C.c_double), ("dVolts_re", C.c_double),
                ("Case", C.c_int), ("J", C.c_double), ("dV", C.c_double)]


class OraAge(C.Structure):
    """ora_age (static2d_oracle.h): one air-gap element."""
    _fields_ = [("BdryFormat", C.c_int), ("ri", C.c_double), ("ro", C.c_double), ("totalArcLength", C.c_double),
                ("InnerShift", C.c_double), ("OuterShift", C.c_double), ("totalArcElements", C.c_int),
                ("qn", iptr), ("qw", dptr)]


def make_ages(mesh, keep):
    ages = (OraAge * max(1, len(mesh.ages)))()
    for k, a in enumerate(mesh.ages):
        o = ages[k]
        o.BdryFormat, o.ri, o.ro = int(a.get("format", 0)), a["ri"], a["ro"]
        o.totalArcLength, o.InnerShift, o.OuterShift = a["total_arc_length"], a["inner_shift"], a["outer_shift"]
        qn = np.asarray(a["qn"], np.int32).reshape(-1, 4)
        o.totalArcElements = len(qn) - 1
        o.qn, o.qw = keep.i(qn.reshape(-1)), keep.d(np.asarray(a["qw"], float).reshape(-1))
    keep.items.append(ages)
    return len(mesh.ages), ages


class OraProblem(C.Structure):
    _fields_ = [("n_nodes", C.c_int), ("x", dptr), ("y", dptr), ("marker", iptr),
                ("n_elems", C.c_int), ("p", iptr), ("e", iptr), ("lbl", iptr), ("blk", iptr),
                ("n_blocks", C.c_int), ("blocks", C.POINTER(OraBlock)),
                ("n_labels", C.c_int), ("labels", C.POINTER(OraLabel)),
                ("n_lines", C.c_int), ("lines", C.POINTER(OraLine)),
                ("n_points", C.c_int), ("points", C.POINTER(OraPoint)),
                ("n_circs", C.c_int), ("circs", C.POINTER(OraCirc)),
                ("n_pbc", C.c_int), ("pbc", iptr),
                ("precision", C.c_double), ("length_units", C.c_int), ("coords", C.c_int),
                ("bandwidth", C.c_int), ("relax", C.c_double),
                ("axisymmetric", C.c_int), ("ext_ro", C.c_double), ("ext_ri", C.c_double), ("ext_zo", C.c_double),
                ("n_ages", C.c_int), ("ages", C.POINTER(OraAge)), ("elem_magdir", dptr)]


class OraStats(C.Structure):
    _fields_ = [("newton_iters", C.c_int), ("cg_iters", C.c_longlong), ("last_res", C.c_double)]


_CREATE = C.CFUNCTYPE(C.c_void_p, C.c_int, C.c_int, C.c_double)
_DESTROY = C.CFUNCTYPE(None, C.c_void_p)
_ADDTO = C.CFUNCTYPE(None, C.c_void_p, C.c_double, C.c_int, C.c_int)
_GETV = C.CFUNCTYPE(dptr, C.c_void_p)
_SETVAL = C.CFUNCTYPE(None, C.c_void_p, C.c_int, C.c_double)
_PAIR = C.CFUNCTYPE(None, C.c_void_p, C.c_int, C.c_int)
_WIPE = C.CFUNCTYPE(None, C.c_void_p)
_PCG = C.CFUNCTYPE(C.c_int, C.c_void_p, C.c_int, C.POINTER(C.c_longlong))


class OraOps(C.Structure):
    _fields_ = [("create", _CREATE), ("destroy", _DESTROY), ("addto", _ADDTO),
                ("b", _GETV), ("V", _GETV), ("setvalue", _SETVAL),
                ("periodicity", _PAIR), ("antiperiodicity", _PAIR), ("wipe", _WIPE),
                ("pcgsolve", _PCG)]


_lib = None
_ref = None


def build(quiet: bool = True) -> None:
    """Compile the oracle (and oracle/_ref when /root/reference is present)."""
    out = subprocess.run(["make", "-C", HERE], capture_output=True, text=True)
    if out.returncode != 0:
        raise RuntimeError("oracle build failed:\n" + out.stdout + out.stderr)


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            build()
        _lib = C.CDLL(LIB_PATH)
        _lib.ora_static2d.argtypes = [C.POINTER(OraProblem), C.c_void_p, dptr, C.POINTER(OraStats)]
        _lib.ora_static2d.restype = C.c_int
        _lib.ora_get_bh_props.argtypes = [C.POINTER(OraBlock), C.c_double, dptr, dptr]
        _lib.ora_lp_create.restype = C.c_void_p
        _lib.ora_lp_create.argtypes = [C.c_int, C.c_int, C.c_double]
        _lib.ora_lp_destroy.argtypes = [C.c_void_p]
        _lib.ora_lp_addto.argtypes = [C.c_void_p, C.c_double, C.c_int, C.c_int]
        _lib.ora_lp_get.argtypes = [C.c_void_p, C.c_int, C.c_int]
        _lib.ora_lp_get.restype = C.c_double
        _lib.ora_lp_b.argtypes = [C.c_void_p]
        _lib.ora_lp_b.restype = dptr
        _lib.ora_lp_V.argtypes = [C.c_void_p]
        _lib.ora_lp_V.restype = dptr
        _lib.ora_lp_setvalue.argtypes = [C.c_void_p, C.c_int, C.c_double]
        _lib.ora_lp_periodicity.argtypes = [C.c_void_p, C.c_int, C.c_int]
        _lib.ora_lp_antiperiodicity.argtypes = [C.c_void_p, C.c_int, C.c_int]
        _lib.ora_lp_pcgsolve.argtypes = [C.c_void_p, C.c_int, C.POINTER(C.c_longlong)]
        _lib.ora_lp_pcgsolve.restype = C.c_int
        _lib.ora_lp_multA.argtypes = [C.c_void_p, dptr, dptr]
        _lib.ora_lp_export_upper.argtypes = [C.c_void_p, iptr, iptr, dptr, C.c_longlong]
        _lib.ora_lp_export_upper.restype = C.c_longlong
    return _lib


def ref_available() -> bool:
    return os.path.exists(REF_PATH)


def ref():
    """The reference's own spars.cpp / CMaterialProp.cpp (oracle/_ref)."""
    global _ref
    if _ref is None:
        if not os.path.exists(REF_PATH):
            raise FileNotFoundError(REF_PATH)
        _ref = C.CDLL(REF_PATH)
        _ref.ref_block_slopes.argtypes = [C.c_char_p, dptr, dptr, dptr, C.c_int, dptr]
        _ref.ref_block_slopes.restype = C.c_int
        _ref.ref_block_bhprops.argtypes = [C.c_char_p, dptr, C.c_int, dptr, dptr]
        _ref.ref_block_bhprops.restype = C.c_int
        _ref.ref_lp_create.restype = C.c_void_p
        _ref.ref_lp_create.argtypes = [C.c_int, C.c_int, C.c_double]
        _ref.ref_lp_get.restype = C.c_double
        _ref.ref_lp_get.argtypes = [C.c_void_p, C.c_int, C.c_int]
        for nm in ("ref_lp_b", "ref_lp_V"):
            getattr(_ref, nm).restype = dptr
            getattr(_ref, nm).argtypes = [C.c_void_p]
    return _ref


_cut = None


def ref_cuthill_available() -> bool:
    return os.path.exists(CUTHILL_PATH)


def ref_cuthill(base: str, num_nodes: int, p, pbc=None, age_counts=None, age_quad=None):
    """The reference's own FEASolver::Cuthill(false) + SortNodes + SortElements
    (cfemm/libfemm/cuthill.cpp:33-391, compiled into oracle/_ref/libref_cuthill.so
    by ref_cuthill.cpp) on a mesh in LoadMesh order.  It reads ``base``.edge
    itself, as the reference does.  p: (NE, 3) corners; pbc: (NP, 2) node pairs;
    age_counts / age_quad: quadNodes per air gap and their (NQ, 4) node ids.
    Returns dict(p, elem_order, newnum, pbc, age_quad, bandwidth): the
    renumbered corners in the sorted element order, the LoadMesh index of the
    element at each position, the node map old -> new, the remapped pairs and
    quadNodes, and BandWidth."""
    global _cut
    if _cut is None:
        if not os.path.exists(CUTHILL_PATH):
            raise FileNotFoundError(CUTHILL_PATH)
        _cut = C.CDLL(CUTHILL_PATH)
        _cut.ref_cuthill_run.argtypes = [C.c_char_p, C.c_int, C.c_int, iptr, iptr, iptr, C.c_int, iptr,
                                         C.c_int, iptr, iptr]
        _cut.ref_cuthill_run.restype = C.c_int
    p = np.ascontiguousarray(np.asarray(p, dtype=np.int32).reshape(-1, 3)).copy()
    ne = len(p)
    pbc = np.ascontiguousarray(np.zeros((0, 2), np.int32) if pbc is None else np.asarray(pbc, np.int32)[:, :2]).copy()
    counts = np.ascontiguousarray(np.zeros(0, np.int32) if age_counts is None else np.asarray(age_counts, np.int32))
    quad = np.ascontiguousarray(np.zeros((0, 4), np.int32) if age_quad is None else np.asarray(age_quad, np.int32)).copy()
    assert quad.shape[0] == int(counts.sum())
    order = np.zeros(ne, np.int32)
    newnum = np.zeros(num_nodes, np.int32)
    bw = _cut.ref_cuthill_run(base.encode(), num_nodes, ne, p.ctypes.data_as(iptr), order.ctypes.data_as(iptr),
                              newnum.ctypes.data_as(iptr), len(pbc), pbc.ctypes.data_as(iptr), len(counts),
                              counts.ctypes.data_as(iptr), quad.ctypes.data_as(iptr))
    if bw < 0:
        raise RuntimeError("reference Cuthill failed on %s.edge" % base)
    return dict(p=p, elem_order=order, newnum=newnum, pbc=pbc, age_quad=quad, bandwidth=bw)


_lua = None


def ref_lua_available() -> bool:
    return os.path.exists(LUA_PATH)


def ref_magdir(fctn: str, p, x, y, length_units: int, mag_dir: float) -> np.ndarray:
    """Per-element magnetisation directions of a MagDirFctn label computed by
    the reference's own Lua interpreter (oracle/_ref/libreflua.so, the element
    loop of static2d.cpp:509-583).  Raises ValueError with the reference's
    message when the chunk fails."""
    global _lua
    if _lua is None:
        if not os.path.exists(LUA_PATH):
            raise FileNotFoundError(LUA_PATH)
        _lua = C.CDLL(LUA_PATH)
        _lua.ref_lua_magdir.argtypes = [C.c_char_p, C.c_int, iptr, dptr, dptr, C.c_int, C.c_double, dptr,
                                        C.c_char_p, C.c_int]
        _lua.ref_lua_magdir.restype = C.c_int
    p = _arr(np.asarray(p).reshape(-1), np.int32)
    x, y = _arr(x, np.float64), _arr(y, np.float64)
    n = len(p) // 3
    t = np.zeros(max(1, n))
    msg = C.create_string_buffer(8192)
    rc = _lua.ref_lua_magdir(fctn.encode(), n, p.ctypes.data_as(iptr), x.ctypes.data_as(dptr),
                             y.ctypes.data_as(dptr), int(length_units), float(mag_dir), t.ctypes.data_as(dptr), msg,
                             len(msg))
    if rc != 0:
        raise ValueError(msg.value.decode())
    return t[:n]


def _ref_ops() -> OraOps:
    r = ref()
    return OraOps(_CREATE(("ref_lp_create", r)), _DESTROY(("ref_lp_destroy", r)),
                  _ADDTO(("ref_lp_addto", r)), _GETV(("ref_lp_b", r)), _GETV(("ref_lp_V", r)),
                  _SETVAL(("ref_lp_setvalue", r)), _PAIR(("ref_lp_periodicity", r)),
                  _PAIR(("ref_lp_antiperiodicity", r)), _WIPE(("ref_lp_wipe", r)),
                  _PCG(("ref_lp_pcgsolve", r)))


def _arr(a, dt):
    return np.ascontiguousarray(np.asarray(a), dtype=dt)


class _Keep:
    """Holds every numpy buffer the ctypes structure points into."""

    def __init__(self):
        self.items = []

    def d(self, a):
        a = _arr(a, np.float64)
        self.items.append(a)
        return a.ctypes.data_as(dptr)

    def i(self, a):
        a = _arr(a, np.int32)
        self.items.append(a)
        return a.ctypes.data_as(iptr)


def element_magdir(pr: femfile.FemProblem, mesh: femfile.Mesh) -> np.ndarray:
    """Per-element magnetisation direction (degrees): the label's MagDir, or
    what the reference's Lua makes of its MagDirFctn at the element centroid
    -- the whole element loop on one interpreter, in element order, as the
    reference's one Lua state per FSolver (ref_magdir_labels).  Static
    problems only, as the reference."""
    return ref_magdir_labels([lb.MagDirFctn for lb in pr.labels], [lb.MagDir for lb in pr.labels], mesh.p,
                             mesh.lbl, mesh.x, mesh.y, pr.LengthUnits, pr.ProblemType == 1)


def ref_magdir_labels(fctns, mag_dirs, p, lbl, x, y, length_units: int, axisymmetric: bool = False) -> np.ndarray:
    """A whole problem's element loop through the reference's own Lua
    (oracle/_ref/libreflua.so ref_lua_magdir_labels: element i runs label
    lbl[i]'s function on one interpreter, static2d.cpp:509-583 /
    staticaxi.cpp:350-406).  Raises ValueError with the reference's message."""
    ref_magdir("", np.zeros((0, 3), np.int32), np.zeros(1), np.zeros(1), 0, 0.0)   # (loads the library)
    _lua.ref_lua_magdir_labels.argtypes = [C.POINTER(C.c_char_p), dptr, C.c_int, iptr, iptr, dptr, dptr, C.c_int,
                                           C.c_int, dptr, C.c_char_p, C.c_int]
    _lua.ref_lua_magdir_labels.restype = C.c_int
    p = _arr(np.asarray(p).reshape(-1), np.int32)
    lbl = _arr(lbl, np.int32)
    x, y = _arr(x, np.float64), _arr(y, np.float64)
    md = _arr(mag_dirs, np.float64)
    fa = (C.c_char_p * max(1, len(fctns)))(*[(f or "").encode() for f in fctns])
    n = len(lbl)
    t = np.zeros(max(1, n))
    msg = C.create_string_buffer(8192)
    rc = _lua.ref_lua_magdir_labels(fa, md.ctypes.data_as(dptr), n, p.ctypes.data_as(iptr), lbl.ctypes.data_as(iptr),
                                    x.ctypes.data_as(dptr), y.ctypes.data_as(dptr), int(length_units),
                                    int(bool(axisymmetric)), t.ctypes.data_as(dptr), msg, len(msg))
    if rc != 0:
        raise ValueError(msg.value.decode())
    return t[:n]


def make_problem(pr: femfile.FemProblem, mesh: femfile.Mesh):
    keep = _Keep()
    blocks = (OraBlock * max(1, len(pr.blocks)))()
    for k, m in enumerate(pr.blocks):
        b = blocks[k]
        b.mu_x, b.mu_y, b.H_c, b.J_re = m.mu_x, m.mu_y, m.H_c, m.J_re
        b.Cduct, b.LamFill, b.LamType, b.BHpoints = m.Cduct, m.LamFill, m.LamType, m.BHpoints
        if m.BHpoints:
            b.Bdata, b.Hdata, b.slope = keep.d(m.Bdata), keep.d(m.Hdata), keep.d(m.slope)
    labels = (OraLabel * max(1, len(pr.labels)))()
    for k, lb in enumerate(pr.labels):
        labels[k].InCircuit, labels[k].MagDir, labels[k].bIsWound = lb.InCircuit, lb.MagDir, int(lb.bIsWound)
        labels[k].IsExternal = int(lb.IsExternal)
    lines = (OraLine * max(1, len(pr.bdrys)))()
    for k, bd in enumerate(pr.bdrys):
        l = lines[k]
        l.BdryFormat, l.A0, l.A1, l.A2, l.phi, l.c0, l.c1 = bd.BdryFormat, bd.A0, bd.A1, bd.A2, bd.phi, bd.c0, bd.c1
    points = (OraPoint * max(1, len(pr.points)))()
    for k, pt in enumerate(pr.points):
        points[k].A_re, points[k].A_im, points[k].J_re, points[k].J_im = pt.A_re, pt.A_im, pt.J_re, pt.J_im
    circs = (OraCirc * max(1, len(pr.circuits)))()
    for k, cc in enumerate(pr.circuits):
        circs[k].CircType, circs[k].Amps_re, circs[k].dVolts_re = cc.CircType, cc.Amps_re, cc.dVolts_re
    P = OraProblem()
    P.n_nodes = len(mesh.x)
    P.x, P.y, P.marker = keep.d(mesh.x), keep.d(mesh.y), keep.i(mesh.marker)
    P.n_elems = len(mesh.lbl)
    P.p, P.e, P.lbl, P.blk = keep.i(mesh.p.reshape(-1)), keep.i(mesh.e.reshape(-1)), keep.i(mesh.lbl), keep.i(mesh.blk)
    P.n_blocks, P.blocks = len(pr.blocks), blocks
    P.n_labels, P.labels = len(pr.labels), labels
    P.n_lines, P.lines = len(pr.bdrys), lines
    P.n_points, P.points = len(pr.points), points
    P.n_circs, P.circs = len(pr.circuits), circs
    P.n_pbc = len(mesh.pbc)
    P.pbc = keep.i(mesh.pbc.reshape(-1) if len(mesh.pbc) else np.zeros(3, np.int32))
    P.precision, P.length_units, P.coords = pr.Precision, pr.LengthUnits, pr.Coords
    P.bandwidth, P.relax = mesh.bandwidth, pr.Relax
    P.axisymmetric = int(pr.ProblemType == 1)
    P.ext_ro, P.ext_ri, P.ext_zo = pr.extRo, pr.extRi, pr.extZo
    P.n_ages, P.ages = make_ages(mesh, keep)
    P.elem_magdir = keep.d(element_magdir(pr, mesh)) if any(lb.MagDirFctn for lb in pr.labels) else None
    keep.items.extend([blocks, labels, lines, points, circs])
    return P, keep, circs


def solve(pr: femfile.FemProblem, mesh: femfile.Mesh, linprob: str = "oracle"):
    """Run the restated Static2D.  Returns (A, stats, circuits[(Case, J, dV)])."""
    L = lib()
    P, keep, circs = make_problem(pr, mesh)
    A = np.zeros(len(mesh.x))
    st = OraStats()
    ops_ptr = None
    if linprob == "reference":
        ops = _ref_ops()
        keep.items.append(ops)
        ops_ptr = C.cast(C.pointer(ops), C.c_void_p)
    elif linprob != "oracle":
        raise ValueError(linprob)
    ok = L.ora_static2d(C.byref(P), ops_ptr, A.ctypes.data_as(dptr), C.byref(st))
    if not ok:
        raise RuntimeError("oracle Static2D failed")
    circ_out = [(circs[k].Case, circs[k].J, circs[k].dV) for k in range(len(pr.circuits))]
    return A, {"newton_iters": st.newton_iters, "cg_iters": st.cg_iters, "last_res": st.last_res}, circ_out


def system(pr: femfile.FemProblem, mesh: femfile.Mesh):
    """Iter-0 assembled system after all boundary conditions (restated
    Static2D + CBigLinProb): returns (scipy.sparse.csr_matrix full symmetric, b)."""
    import scipy.sparse as sp
    L = lib()
    L.ora_static2d_system.argtypes = [C.POINTER(OraProblem), iptr, iptr, dptr, C.c_longlong, dptr,
                                      C.POINTER(C.c_longlong)]
    P, keep, _ = make_problem(pr, mesh)
    n = len(mesh.x)
    cap = 16 * n + 1024
    rows = np.zeros(cap, np.int32)
    cols = np.zeros(cap, np.int32)
    vals = np.zeros(cap)
    b = np.zeros(n)
    nnz = C.c_longlong()
    L.ora_static2d_system(C.byref(P), rows.ctypes.data_as(iptr), cols.ctypes.data_as(iptr),
                          vals.ctypes.data_as(dptr), cap, b.ctypes.data_as(dptr), C.byref(nnz))
    k = nnz.value
    if k > cap:
        raise RuntimeError("export capacity too small")
    U = sp.coo_matrix((vals[:k], (rows[:k], cols[:k])), shape=(n, n)).tocsr()
    D = sp.diags(U.diagonal())
    return (U + U.T - D).tocsr(), b
