"""ctypes driver for the harmonic-2D oracle (harmonic2d_oracle.c) -- TEST
INFRASTRUCTURE ONLY.  Only tests/ and __graft_entry__.smoke() import this.

``solve(pr, mesh, linprob="oracle"|"reference")`` runs the restated linear
FSolver::Harmonic2D (cfemm/fsolver/harmonic2d.cpp:36-790) on the CPU, with
the complex linear algebra done either by the restated CBigComplexLinProb or
by the reference's own cspars.cpp compiled into oracle/_ref.
"""
from __future__ import annotations

import ctypes as C

import numpy as np

from . import femfile
from .oracle import OraPoint, OraStats, _Keep, dptr, iptr, lib, ref


class OrhBlock(C.Structure):
    _fields_ = [("mu_x", C.c_double), ("mu_y", C.c_double), ("Theta_hx", C.c_double), ("Theta_hy", C.c_double),
                ("Lam_d", C.c_double), ("LamFill", C.c_double), ("J_re", C.c_double), ("J_im", C.c_double),
                ("Cduct", C.c_double), ("LamType", C.c_int), ("BHpoints", C.c_int),
                ("B", dptr), ("H_re", dptr), ("H_im", dptr), ("S_re", dptr), ("S_im", dptr)]


class OrhLabel(C.Structure):
    _fields_ = [("InCircuit", C.c_int), ("bIsWound", C.c_int), ("IsExternal", C.c_int),
                ("ProxMu_re", C.c_double), ("ProxMu_im", C.c_double)]


class OrhLine(C.Structure):
    _fields_ = [("BdryFormat", C.c_int), ("A0", C.c_double), ("A1", C.c_double), ("A2", C.c_double),
                ("phi", C.c_double), ("c0_re", C.c_double), ("c0_im", C.c_double), ("c1_re", C.c_double),
                ("c1_im", C.c_double), ("Mu", C.c_double), ("Sig", C.c_double)]


class OrhCirc(C.Structure):
    _fields_ = [("CircType", C.c_int), ("Amps_re", C.c_double), ("Amps_im", C.c_double),
                ("dVolts_re", C.c_double), ("dVolts_im", C.c_double), ("Case", C.c_int),
                ("J_re", C.c_double), ("J_im", C.c_double), ("dV_re", C.c_double), ("dV_im", C.c_double)]


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


class OrhProblem(C.Structure):
    _fields_ = [("n_nodes", C.c_int), ("x", dptr), ("y", dptr), ("marker", iptr),
                ("n_elems", C.c_int), ("p", iptr), ("e", iptr), ("lbl", iptr), ("blk", iptr),
                ("n_blocks", C.c_int), ("blocks", C.POINTER(OrhBlock)),
                ("n_labels", C.c_int), ("labels", C.POINTER(OrhLabel)),
                ("n_lines", C.c_int), ("lines", C.POINTER(OrhLine)),
                ("n_points", C.c_int), ("points", C.POINTER(OraPoint)),
                ("n_circs", C.c_int), ("circs", C.POINTER(OrhCirc)),
                ("n_pbc", C.c_int), ("pbc", iptr),
                ("precision", C.c_double), ("frequency", C.c_double), ("length_units", C.c_int),
                ("coords", C.c_int), ("bandwidth", C.c_int), ("problem_type", C.c_int),
                ("extZo", C.c_double), ("extRo", C.c_double), ("extRi", C.c_double),
                ("n_ages", C.c_int), ("ages", C.POINTER(OraAge)), ("ac_solver", C.c_int)]


_CREATE = C.CFUNCTYPE(C.c_void_p, C.c_int, C.c_int, C.c_int, C.c_double)
_DESTROY = C.CFUNCTYPE(None, C.c_void_p)
_ADDTO = C.CFUNCTYPE(None, C.c_void_p, C.c_double, C.c_double, C.c_int, C.c_int)
_GET = C.CFUNCTYPE(None, C.c_void_p, C.c_int, C.c_int, dptr, dptr)
_PUT = C.CFUNCTYPE(None, C.c_void_p, C.c_double, C.c_double, C.c_int, C.c_int)
_GETV = C.CFUNCTYPE(dptr, C.c_void_p)
_SETVAL = C.CFUNCTYPE(None, C.c_void_p, C.c_int, C.c_double, C.c_double)
_PAIR = C.CFUNCTYPE(None, C.c_void_p, C.c_int, C.c_int)
_SOLVE = C.CFUNCTYPE(C.c_int, C.c_void_p, C.c_int)
_WIPE = C.CFUNCTYPE(None, C.c_void_p)
_PUTK = C.CFUNCTYPE(None, C.c_void_p, C.c_double, C.c_double, C.c_int, C.c_int, C.c_int)
_GETK = C.CFUNCTYPE(None, C.c_void_p, C.c_int, C.c_int, C.c_int, dptr, dptr)
_NEWTON = C.CFUNCTYPE(C.c_int, C.c_void_p)
_SETPREC = C.CFUNCTYPE(None, C.c_void_p, C.c_double)


class OrhOps(C.Structure):
    _fields_ = [("create", _CREATE), ("destroy", _DESTROY), ("addto", _ADDTO), ("get", _GET), ("put", _PUT),
                ("b", _GETV), ("V", _GETV), ("setvalue", _SETVAL), ("periodicity", _PAIR),
                ("antiperiodicity", _PAIR), ("solve", _SOLVE), ("wipe", _WIPE), ("put_k", _PUTK),
                ("get_k", _GETK), ("newton", _NEWTON), ("set_precision", _SETPREC)]


def _hlib():
    L = lib()
    if not hasattr(L, "_orh_ready"):
        L.orh_harmonic2d.argtypes = [C.POINTER(OrhProblem), C.c_void_p, dptr, C.POINTER(OraStats)]
        L.orh_harmonic2d.restype = C.c_int
        L.orh_harmonic2d_system.argtypes = [C.POINTER(OrhProblem), iptr, iptr, dptr, C.c_longlong, dptr,
                                            C.POINTER(C.c_longlong)]
        L.orh_harmonic2d_system.restype = C.c_int
        L.orh_acprops.argtypes = [C.POINTER(OrhBlock), dptr, C.c_int, dptr, dptr]
        L._orh_ready = True
    return L


def _ref_ops() -> OrhOps:
    r = ref()
    for nm in ("ref_clp_b", "ref_clp_V"):
        getattr(r, nm).restype = dptr
    r.ref_clp_create.restype = C.c_void_p

    def f(proto, name):
        return proto((name, r))
    return OrhOps(f(_CREATE, "ref_clp_create"), f(_DESTROY, "ref_clp_destroy"), f(_ADDTO, "ref_clp_addto"),
                  f(_GET, "ref_clp_get"), f(_PUT, "ref_clp_put"), f(_GETV, "ref_clp_b"), f(_GETV, "ref_clp_V"),
                  f(_SETVAL, "ref_clp_setvalue"), f(_PAIR, "ref_clp_periodicity"),
                  f(_PAIR, "ref_clp_antiperiodicity"), f(_SOLVE, "ref_clp_solve"), f(_WIPE, "ref_clp_wipe"),
                  f(_PUTK, "ref_clp_put_k"), f(_GETK, "ref_clp_get_k"), f(_NEWTON, "ref_clp_newton"),
                  f(_SETPREC, "ref_clp_set_precision"))


def make_problem(pr: femfile.FemProblem, mesh: femfile.Mesh):
    keep = _Keep()
    blocks = (OrhBlock * max(1, len(pr.blocks)))()
    for k, m in enumerate(pr.blocks):
        b = blocks[k]
        b.mu_x, b.mu_y, b.Theta_hx, b.Theta_hy = m.mu_x, m.mu_y, m.Theta_hx, m.Theta_hy
        b.Lam_d, b.LamFill, b.J_re, b.J_im, b.Cduct = m.Lam_d, m.LamFill, m.J_re, m.J_im, m.Cduct
        b.LamType, b.BHpoints = m.LamType, m.BHpoints
        if m.BHpoints:   # the GetSlopes(omega) curve, complex (an input of the restated loop)
            H, S = np.asarray(m.Hdata, dtype=complex), np.asarray(m.slope, dtype=complex)
            b.B, b.H_re, b.H_im = keep.d(np.asarray(m.Bdata, float)), keep.d(H.real), keep.d(H.imag)
            b.S_re, b.S_im = keep.d(S.real), keep.d(S.imag)
    labels = (OrhLabel * max(1, len(pr.labels)))()
    for k, lb in enumerate(pr.labels):
        labels[k].InCircuit, labels[k].bIsWound = lb.InCircuit, int(lb.bIsWound)
        labels[k].IsExternal = int(lb.IsExternal)
        pm = complex(getattr(lb, "ProximityMu", 1.0))
        labels[k].ProxMu_re, labels[k].ProxMu_im = pm.real, pm.imag
    lines = (OrhLine * max(1, len(pr.bdrys)))()
    for k, bd in enumerate(pr.bdrys):
        l = lines[k]
        l.BdryFormat, l.A0, l.A1, l.A2, l.phi = bd.BdryFormat, bd.A0, bd.A1, bd.A2, bd.phi
        l.c0_re, l.c0_im, l.c1_re, l.c1_im, l.Mu, l.Sig = bd.c0, bd.c0i, bd.c1, bd.c1i, bd.Mu, bd.Sig
    points = (OraPoint * max(1, len(pr.points)))()
    for k, pt in enumerate(pr.points):
        points[k].A_re, points[k].A_im, points[k].J_re, points[k].J_im = pt.A_re, pt.A_im, pt.J_re, pt.J_im
    circs = (OrhCirc * max(1, len(pr.circuits)))()
    for k, cc in enumerate(pr.circuits):
        o = circs[k]
        o.CircType, o.Amps_re, o.Amps_im = cc.CircType, cc.Amps_re, cc.Amps_im
        o.dVolts_re, o.dVolts_im = cc.dVolts_re, cc.dVolts_im
    P = OrhProblem()
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
    P.precision, P.frequency = pr.Precision, pr.Frequency
    P.length_units, P.coords, P.bandwidth = pr.LengthUnits, pr.Coords, mesh.bandwidth
    P.problem_type, P.extZo, P.extRo, P.extRi = pr.ProblemType, pr.extZo, pr.extRo, pr.extRi
    P.n_ages, P.ages = make_ages(mesh, keep)
    P.ac_solver = int(getattr(pr, "ACSolver", 0))
    keep.items.extend([blocks, labels, lines, points, circs])
    return P, keep, circs


def solve(pr: femfile.FemProblem, mesh: femfile.Mesh, linprob: str = "oracle"):
    """Restated Harmonic2D (linear, or the successive approximation of
    nonlinear blocks whose femfile.BlockProp carries the GetSlopes(omega)
    curve: Bdata, complex Hdata / slope).  Returns (A complex per node, stats,
    circuits[(Case, J, dV)] with complex J / dV)."""
    L = _hlib()
    P, keep, circs = make_problem(pr, mesh)
    A = np.zeros(2 * len(mesh.x))
    st = OraStats()
    ops_ptr = None
    if linprob == "reference":
        ops = _ref_ops()
        keep.items.append(ops)
        ops_ptr = C.cast(C.pointer(ops), C.c_void_p)
    elif linprob != "oracle":
        raise ValueError(linprob)
    if not L.orh_harmonic2d(C.byref(P), ops_ptr, A.ctypes.data_as(dptr), C.byref(st)):
        raise RuntimeError("oracle Harmonic2D failed (nonlinear or unsupported lamination, or singular)")
    out = [(circs[k].Case, complex(circs[k].J_re, circs[k].J_im), complex(circs[k].dV_re, circs[k].dV_im))
           for k in range(len(pr.circuits))]
    return A[0::2] + 1j * A[1::2], {"newton_iters": st.newton_iters, "cg_iters": st.cg_iters}, out


def system(pr: femfile.FemProblem, mesh: femfile.Mesh):
    """Assembled node system after all boundary conditions: (scipy csr complex
    full symmetric, b complex)."""
    import scipy.sparse as sp
    L = _hlib()
    P, keep, _ = make_problem(pr, mesh)
    n = len(mesh.x)
    cap = 16 * n + 1024
    rows = np.zeros(cap, np.int32)
    cols = np.zeros(cap, np.int32)
    vals = np.zeros(2 * cap)
    b = np.zeros(2 * n)
    nnz = C.c_longlong()
    if not L.orh_harmonic2d_system(C.byref(P), rows.ctypes.data_as(iptr), cols.ctypes.data_as(iptr),
                                   vals.ctypes.data_as(dptr), cap, b.ctypes.data_as(dptr), C.byref(nnz)):
        raise RuntimeError("oracle Harmonic2D system failed")
    k = nnz.value
    if k > cap:
        raise RuntimeError("export capacity too small")
    v = vals[0:2 * k:2] + 1j * vals[1:2 * k:2]
    U = sp.coo_matrix((v, (rows[:k], cols[:k])), shape=(n, n)).tocsr()
    D = sp.diags(U.diagonal())
    return (U + U.T - D).tocsr(), b[0::2] + 1j * b[1::2]
