"""ctypes binding of the C-ABI in include/xfemm_kernels.h (lib/libxfemm_kernels.so).

This is the Python view of the MI355X hot path used by tests and bench.py.
There is no CPU fallback: if the HIP library is missing, or no gfx950 device
is present, every solve raises.
"""
from __future__ import annotations

import ctypes as C
import os
from typing import Optional, Sequence

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_DIR = os.path.join(HERE, "lib")
KERNELS_SO = os.path.join(LIB_DIR, "libxfemm_kernels.so")

dptr = C.POINTER(C.c_double)
iptr = C.POINTER(C.c_int)

XFK_OK = 0
XFK_REBUILD_SYMBOLIC = 1
XFK_TIME_SPMV = 2
XFK_TIME_TAIL = 4
XFK_PRECOND_JACOBI = 0
XFK_PRECOND_AMG = 1
PRECONDS = {"jacobi": XFK_PRECOND_JACOBI, "amg": XFK_PRECOND_AMG}
XFK_OPT_PRECOND = 1
XFK_OPT_AMG_SWEEPS = 2
XFK_OPT_AMG_THETA = 3
XFK_OPT_AMG_OMEGA = 4
XFK_OPT_AMG_REPLICATE = 5
XFK_OPT_AMG_REUSE = 6
XFK_OPT_AMG_DENSE = 7
XFK_OPT_AMG_FOLD = 8
XFK_OPT_AMG_COL16 = 9
XFK_OPT_AMG_WLEVEL = 10
XFK_OPT_AMG_F32 = 11
XFK_OPT_NEWTON_INEXACT = 12

# every symbol include/xfemm_kernels.h declares
EXPORTED = (
    "xfk_last_error", "xfk_age_element_matrix", "xfk_device_count", "xfk_device_init", "xfk_problem_create", "xfk_problem_destroy",
    "xfk_static2d", "xfk_get_solution", "xfk_get_circuits", "xfk_get_csr", "xfk_get_nnz", "xfk_spmv_col_bytes",
    "xfk_get_stream", "xfk_pcg_solve_csr", "xfk_pcg_solve_csr_pc", "xfk_pcg_time", "xfk_phase_profile",
    "xfk_alloc_stats", "xfk_problem_memory", "xfk_cache_stats", "xfk_release_cache",
    "xfk_amg_forget_hints",
    "xfk_set_option",
    "xfk_problem_create_harmonic", "xfk_problem_create_harmonic_dist", "xfk_harmonic2d",
    "xfk_get_solution_complex", "xfk_get_circuits_complex",
    "xfk_get_csr_complex",
    "xfk_comm_unique_id", "xfk_comm_create_rccl", "xfk_comm_create_local", "xfk_comm_destroy",
    "xfk_comm_rank", "xfk_comm_size", "xfk_comm_record", "xfk_comm_log", "xfk_comm_create_replay",
    "xfk_comm_time", "xfk_comm_timing",
    "xfk_partition_plan", "xfk_partition_plan_coupled", "xfk_problem_create_dist", "xfk_dist_get_info",
    "xfk_magdir_eval", "xfk_magdir_eval_labels", "xfk_lua_run", "xfk_sort_elements",
)


class BlockDesc(C.Structure):
    _fields_ = [("mu_x", C.c_double), ("mu_y", C.c_double), ("H_c", C.c_double),
                ("J_re", C.c_double), ("Cduct", C.c_double), ("LamFill", C.c_double),
                ("LamType", C.c_int), ("BHpoints", C.c_int),
                ("B", dptr), ("H", dptr), ("slope", dptr)]


class LabelDesc(C.Structure):
    _fields_ = [("block", C.c_int), ("in_circuit", C.c_int), ("mag_dir", C.c_double),
                ("is_wound", C.c_int), ("is_external", C.c_int), ("mag_dir_fctn", C.c_char_p)]


class LineDesc(C.Structure):
    _fields_ = [("format", C.c_int), ("A0", C.c_double), ("A1", C.c_double), ("A2", C.c_double),
                ("phi", C.c_double), ("c0", C.c_double), ("c1", C.c_double)]


class PointDesc(C.Structure):
    _fields_ = [("A_re", C.c_double), ("A_im", C.c_double), ("J_re", C.c_double),
                ("J_im", C.c_double)]


class CircuitDesc(C.Structure):
    _fields_ = [("type", C.c_int), ("amps_re", C.c_double), ("dvolts_re", C.c_double)]


class AgeDesc(C.Structure):
    """xfk_age_desc: one CAirGapElement as read from the .pbc file."""
    _fields_ = [("format", C.c_int), ("ri", C.c_double), ("ro", C.c_double), ("total_arc_length", C.c_double),
                ("inner_shift", C.c_double), ("outer_shift", C.c_double), ("n_arc", C.c_int),
                ("qn", iptr), ("qw", dptr)]


class ProblemDesc(C.Structure):
    _fields_ = [("n_nodes", C.c_int), ("x", dptr), ("y", dptr), ("marker", iptr),
                ("n_elems", C.c_int), ("p", iptr), ("e", iptr), ("lbl", iptr),
                ("n_blocks", C.c_int), ("blocks", C.POINTER(BlockDesc)),
                ("n_labels", C.c_int), ("labels", C.POINTER(LabelDesc)),
                ("n_lines", C.c_int), ("lines", C.POINTER(LineDesc)),
                ("n_points", C.c_int), ("points", C.POINTER(PointDesc)),
                ("n_circs", C.c_int), ("circs", C.POINTER(CircuitDesc)),
                ("n_pbc", C.c_int), ("pbc", iptr),
                ("precision", C.c_double), ("length_units", C.c_int), ("coords", C.c_int),
                ("relax", C.c_double), ("problem_type", C.c_int), ("ext_zo", C.c_double),
                ("ext_ro", C.c_double), ("ext_ri", C.c_double),
                ("n_ages", C.c_int), ("ages", C.POINTER(AgeDesc))]


XFK_PLANAR = 0
XFK_AXISYMMETRIC = 1


class Result(C.Structure):
    _fields_ = [("newton_iters", C.c_int), ("cg_iters", C.c_longlong), ("last_res", C.c_double),
                ("final_er", C.c_double), ("nnz", C.c_longlong), ("ncolors", C.c_int),
                ("ms_symbolic", C.c_double), ("ms_assemble", C.c_double), ("ms_solve", C.c_double),
                ("spmv_ms_avg", C.c_double), ("spmv_samples", C.c_int),
                ("color_rounds", C.c_int), ("precond", C.c_int), ("amg_levels", C.c_int),
                ("amg_op_complexity", C.c_double), ("ms_amg_setup", C.c_double), ("ms_rep_cycle", C.c_double),
                ("rep_cycles", C.c_int), ("ms_rep_setup", C.c_double), ("prec_fallback", C.c_int)]

    def as_dict(self):
        return {k: getattr(self, k) for k, _ in self._fields_}


class DistInfo(C.Structure):
    _fields_ = [("rank", C.c_int), ("nranks", C.c_int), ("n_global", C.c_int), ("row0", C.c_int),
                ("n_own", C.c_int), ("n_halo", C.c_int), ("n_elems", C.c_int), ("n_send", C.c_int),
                ("n_recv", C.c_int), ("n_extra", C.c_int)]

    def as_dict(self):
        return {k: getattr(self, k) for k, _ in self._fields_}


_lib = None


class XfkError(RuntimeError):
    pass


def load_library(path: str = KERNELS_SO):
    """Load lib/libxfemm_kernels.so (raises if it was not built)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(path):
        raise XfkError("HIP library %s not built (run __graft_entry__.build() / make -C xfemm_amd)" % path)
    L = C.CDLL(path)
    L.xfk_last_error.restype = C.c_char_p
    L.xfk_device_count.restype = C.c_int
    L.xfk_problem_create.argtypes = [C.POINTER(ProblemDesc), C.c_int, C.POINTER(C.c_void_p)]
    L.xfk_problem_destroy.argtypes = [C.c_void_p]
    L.xfk_static2d.argtypes = [C.c_void_p, C.c_int, C.POINTER(Result)]
    L.xfk_get_solution.argtypes = [C.c_void_p, dptr]
    L.xfk_get_circuits.argtypes = [C.c_void_p, iptr, dptr, dptr]
    L.xfk_get_csr.argtypes = [C.c_void_p, iptr, iptr, dptr, dptr]
    L.xfk_get_nnz.argtypes = [C.c_void_p]
    L.xfk_get_nnz.restype = C.c_longlong
    L.xfk_spmv_col_bytes.argtypes = [C.c_void_p]
    L.xfk_spmv_col_bytes.restype = C.c_double
    L.xfk_get_stream.argtypes = [C.c_void_p, C.POINTER(C.c_void_p)]
    L.xfk_pcg_solve_csr.argtypes = [C.c_int, iptr, iptr, dptr, dptr, dptr, C.c_int, C.c_double, C.c_int,
                                    C.POINTER(C.c_longlong), dptr]
    L.xfk_pcg_solve_csr_pc.argtypes = [C.c_int, iptr, iptr, dptr, dptr, dptr, C.c_int, C.c_double, C.c_int,
                                       C.c_int, C.POINTER(C.c_longlong), dptr]
    L.xfk_pcg_time.argtypes = [C.c_void_p, C.c_int, dptr, dptr]
    L.xfk_phase_profile.argtypes = [C.c_void_p, C.c_int, C.c_int, C.c_void_p, C.c_int, C.POINTER(C.c_int)]
    L.xfk_alloc_stats.argtypes = [dptr, C.c_int]
    L.xfk_problem_memory.argtypes = [C.c_void_p, C.POINTER(C.c_longlong)]
    L.xfk_cache_stats.argtypes = [C.POINTER(C.c_longlong)]
    L.xfk_set_option.argtypes = [C.c_void_p, C.c_int, C.c_double]
    L.xfk_problem_create_harmonic.argtypes = [C.POINTER(ProblemDesc), C.c_void_p, C.c_int, C.POINTER(C.c_void_p)]
    L.xfk_problem_create_harmonic_dist.argtypes = [C.POINTER(ProblemDesc), C.c_void_p, C.c_int, C.c_void_p,
                                                   C.POINTER(C.c_void_p)]
    L.xfk_harmonic2d.argtypes = [C.c_void_p, C.c_int, C.POINTER(Result)]
    L.xfk_get_solution_complex.argtypes = [C.c_void_p, dptr]
    L.xfk_get_circuits_complex.argtypes = [C.c_void_p, iptr, dptr, dptr]
    L.xfk_get_csr_complex.argtypes = [C.c_void_p, iptr, iptr, dptr, dptr]
    L.xfk_age_element_matrix.argtypes = [C.c_double, C.c_double, C.c_double, C.c_double, dptr]
    vp = C.c_void_p
    L.xfk_comm_unique_id.argtypes = [C.c_char_p, C.c_int]
    L.xfk_comm_create_rccl.argtypes = [C.c_char_p, C.c_int, C.c_int, C.c_int, C.c_int, C.POINTER(vp)]
    L.xfk_comm_create_local.argtypes = [C.c_int, C.POINTER(vp)]
    L.xfk_comm_destroy.argtypes = [vp]
    L.xfk_comm_rank.argtypes = [vp]
    L.xfk_comm_size.argtypes = [vp]
    L.xfk_comm_record.argtypes = [vp, C.c_int]
    L.xfk_comm_log.argtypes = [vp, vp, C.c_int, C.POINTER(C.c_int)]
    L.xfk_comm_time.argtypes = [vp, C.c_int]
    L.xfk_comm_timing.argtypes = [vp, C.POINTER(C.c_longlong), dptr, dptr]
    L.xfk_comm_create_replay.argtypes = [vp, C.POINTER(vp)]
    L.xfk_partition_plan.argtypes = [C.c_int, C.c_int, iptr, C.c_int, C.c_int, C.POINTER(DistInfo),
                                     iptr, iptr, iptr, iptr]
    L.xfk_partition_plan_coupled.argtypes = [C.c_int, C.c_int, iptr, C.c_int, C.c_int, C.c_int, iptr,
                                             C.POINTER(DistInfo), iptr, iptr, iptr, iptr]
    L.xfk_problem_create_dist.argtypes = [C.POINTER(ProblemDesc), C.c_int, vp, C.POINTER(vp)]
    L.xfk_dist_get_info.argtypes = [vp, C.POINTER(DistInfo)]
    L.xfk_sort_elements.argtypes = [C.c_int, C.POINTER(C.c_uint), C.c_int, iptr]
    L.xfk_magdir_eval.argtypes = [C.c_char_p, C.c_int, iptr, dptr, dptr, C.c_int, C.c_double, dptr]
    L.xfk_lua_run.argtypes = [C.c_char_p, C.c_char_p, C.c_longlong, C.POINTER(C.c_longlong)]
    L.xfk_magdir_eval_labels.argtypes = [C.c_int, C.POINTER(C.c_char_p), dptr, C.c_int, iptr, iptr, dptr, dptr,
                                         C.c_int, C.c_int, C.c_int, dptr]
    _lib = L
    return L


def _check(rc: int):
    if rc != XFK_OK:
        raise XfkError("xfk error %d: %s" % (rc, _lib.xfk_last_error().decode()))


def alloc_stats(reset: bool = False) -> dict:
    """Device allocations of the library since the last reset (diagnostics):
    hipMalloc / hipFree calls and their host milliseconds."""
    out = np.zeros(4)
    _check(load_library().xfk_alloc_stats(out.ctypes.data_as(dptr), int(reset)))
    return dict(n_malloc=int(out[0]), ms_malloc=float(out[1]), n_free=int(out[2]), ms_free=float(out[3]))


def cache_stats() -> dict:
    """The process-wide caches destroyed problems leave for the next one
    (xfk_cache_stats): device bytes, pinned host bytes, idle streams."""
    out = (C.c_longlong * 3)()
    _check(load_library().xfk_cache_stats(out))
    return dict(device_bytes=int(out[0]), pinned_bytes=int(out[1]), idle_streams=int(out[2]))


def release_cache():
    """Give the process-wide caches back to HIP (xfk_release_cache)."""
    _check(load_library().xfk_release_cache())


def forget_amg_hints():
    """Drop the AMG hints the last setup left for the next fresh problem of
    its size (xfk_amg_forget_hints): the next setup measures everything."""
    _check(load_library().xfk_amg_forget_hints())


def sort_elements(score, device: int = 0) -> np.ndarray:
    """FEASolver::SortElements' comb sort of element scores on the device
    (xfk_sort_elements): the permutation (position -> element)."""
    sc = np.ascontiguousarray(score, dtype=np.uint32)
    perm = np.empty(len(sc), dtype=np.int32)
    _check(load_library().xfk_sort_elements(len(sc), sc.ctypes.data_as(C.POINTER(C.c_uint)), device,
                                            perm.ctypes.data_as(iptr)))
    return perm


def device_count() -> int:
    return load_library().xfk_device_count()


class _Keep(list):
    def d(self, a):
        a = np.ascontiguousarray(a, dtype=np.float64)
        self.append(a)
        return a.ctypes.data_as(dptr)

    def i(self, a):
        a = np.ascontiguousarray(a, dtype=np.int32)
        self.append(a)
        return a.ctypes.data_as(iptr)


def _make_desc(x, y, p, lbl, blocks, labels, lines, points, circuits, marker, e, pbc, precision, length_units,
               coords, relax, problem_type=0, ext=(0.0, 0.0, 0.0), ages=()):
    """xfk_problem_desc of plain arrays / dicts (see Static2DProblem); returns
    (desc, keep) where keep holds every buffer the descriptor points into."""
    keep = _Keep()
    nb = max(1, len(blocks))
    bl = (BlockDesc * nb)()
    for k, b in enumerate(blocks):
        o = bl[k]
        o.mu_x, o.mu_y = b.get("mu_x", 1.0), b.get("mu_y", 1.0)
        o.H_c, o.J_re, o.Cduct = b.get("H_c", 0.0), b.get("J_re", 0.0), b.get("Cduct", 0.0)
        o.LamFill, o.LamType = b.get("LamFill", 1.0), b.get("LamType", 0)
        n = len(b.get("B", ()))
        o.BHpoints = n
        if n:
            # (harmonic blocks may carry the complex curve: real parts here)
            o.B, o.H, o.slope = keep.d(b["B"]), keep.d(np.real(b["H"])), keep.d(np.real(b["slope"]))
    lb = (LabelDesc * max(1, len(labels)))()
    for k, l in enumerate(labels):
        lb[k].block, lb[k].in_circuit = l["block"], l.get("in_circuit", -1)
        lb[k].mag_dir, lb[k].is_wound = l.get("mag_dir", 0.0), int(l.get("is_wound", 0))
        lb[k].is_external = int(l.get("is_external", 0))
        f = l.get("mag_dir_fctn") or ""
        if f:
            fb = f.encode()
            keep.append(fb)
            lb[k].mag_dir_fctn = fb
    ln = (LineDesc * max(1, len(lines)))()
    for k, l in enumerate(lines):
        o = ln[k]
        o.format = l.get("format", 0)
        o.A0, o.A1, o.A2, o.phi = l.get("A0", 0.0), l.get("A1", 0.0), l.get("A2", 0.0), l.get("phi", 0.0)
        o.c0, o.c1 = l.get("c0", 0.0), l.get("c1", 0.0)
    pt = (PointDesc * max(1, len(points)))()
    for k, q in enumerate(points):
        pt[k].A_re, pt[k].A_im = q.get("A_re", 0.0), q.get("A_im", 0.0)
        pt[k].J_re, pt[k].J_im = q.get("J_re", 0.0), q.get("J_im", 0.0)
    ci = (CircuitDesc * max(1, len(circuits)))()
    for k, q in enumerate(circuits):
        ci[k].type, ci[k].amps_re, ci[k].dvolts_re = q.get("type", 0), q.get("amps_re", 0.0), q.get("dvolts_re", 0.0)
    D = ProblemDesc()
    x = np.asarray(x, dtype=np.float64)
    D.n_nodes = len(x)
    D.x, D.y = keep.d(x), keep.d(y)
    D.marker = keep.i(marker) if marker is not None else None
    p = np.asarray(p, dtype=np.int32).reshape(-1)
    D.n_elems = len(p) // 3
    D.p = keep.i(p)
    D.e = keep.i(np.asarray(e, dtype=np.int32).reshape(-1)) if e is not None else None
    D.lbl = keep.i(lbl)
    D.n_blocks, D.blocks = len(blocks), bl
    D.n_labels, D.labels = len(labels), lb
    D.n_lines, D.lines = len(lines), ln
    D.n_points, D.points = len(points), pt
    D.n_circs, D.circs = len(circuits), ci
    if pbc is not None and len(pbc):
        pb = np.asarray(pbc, dtype=np.int32).reshape(-1)
        D.n_pbc, D.pbc = len(pb) // 3, keep.i(pb)
    else:
        D.n_pbc, D.pbc = 0, None
    D.precision, D.length_units, D.coords, D.relax = precision, length_units, coords, relax
    D.problem_type = int(problem_type)
    D.ext_zo, D.ext_ro, D.ext_ri = ext
    # air-gap elements: dicts with format, ri, ro, total_arc_length, inner_shift,
    # outer_shift and the quadNode table qn / qw ((n_arc + 1) x 4 each)
    ag = (AgeDesc * max(1, len(ages)))()
    for k, a in enumerate(ages):
        o = ag[k]
        o.format, o.ri, o.ro = int(a.get("format", 0)), a["ri"], a["ro"]
        o.total_arc_length, o.inner_shift, o.outer_shift = a["total_arc_length"], a["inner_shift"], a["outer_shift"]
        qn = np.asarray(a["qn"], dtype=np.int32).reshape(-1, 4)
        o.n_arc = len(qn) - 1
        o.qn, o.qw = keep.i(qn), keep.d(np.asarray(a["qw"], dtype=np.float64).reshape(-1, 4))
    D.n_ages, D.ages = len(ages), ag
    keep.extend([bl, lb, ln, pt, ci, ag])
    return D, keep


def magdir_eval(fctn: str, p, x, y, length_units: int = 0, mag_dir: float = 0.0) -> np.ndarray:
    """Per-element magnetisation direction (degrees) of a label's MagDirFctn
    (xfk_magdir_eval; host only, no device needed).  Raises XfkError with the
    reference's message when the expression does not evaluate."""
    L = load_library()
    p = np.ascontiguousarray(np.asarray(p, dtype=np.int32).reshape(-1))
    x = np.ascontiguousarray(x, dtype=np.float64)
    y = np.ascontiguousarray(y, dtype=np.float64)
    n = len(p) // 3
    t = np.zeros(max(1, n))
    _check(L.xfk_magdir_eval(fctn.encode(), n, p.ctypes.data_as(iptr), x.ctypes.data_as(dptr),
                             y.ctypes.data_as(dptr), int(length_units), float(mag_dir), t.ctypes.data_as(dptr)))
    return t[:n]


def magdir_eval_labels(fctns, mag_dirs, p, lbl, x, y, length_units: int = 0, axisymmetric: bool = False,
                       repeats: bool = False) -> np.ndarray:
    """A whole problem's element loop of MagDirFctn (xfk_magdir_eval_labels):
    element i runs label lbl[i]'s function (None / "" for the label's MagDir)
    on one interpreter, in element order.  Host only."""
    L = load_library()
    p = np.ascontiguousarray(np.asarray(p, dtype=np.int32).reshape(-1))
    lbl = np.ascontiguousarray(lbl, dtype=np.int32)
    x = np.ascontiguousarray(x, dtype=np.float64)
    y = np.ascontiguousarray(y, dtype=np.float64)
    md = np.ascontiguousarray(mag_dirs, dtype=np.float64)
    fa = (C.c_char_p * max(1, len(fctns)))(*[(f or "").encode() for f in fctns])
    n = len(lbl)
    t = np.zeros(max(1, n))
    _check(L.xfk_magdir_eval_labels(len(fctns), fa, md.ctypes.data_as(dptr), n, p.ctypes.data_as(iptr),
                                    lbl.ctypes.data_as(iptr), x.ctypes.data_as(dptr), y.ctypes.data_as(dptr),
                                    int(length_units), int(bool(axisymmetric)), int(bool(repeats)),
                                    t.ctypes.data_as(dptr)))
    return t[:n]


def lua_run(chunk: str) -> str:
    """Run a whole Lua chunk on a fresh native interpreter (xfk_lua_run) and
    return what it printed / wrote to the standard output.  Raises XfkError
    (code -2) for a Lua error, (-1) for a refused construct."""
    L = load_library()
    n = C.c_longlong(0)
    buf = C.create_string_buffer(1 << 16)
    rc = L.xfk_lua_run(chunk.encode(), buf, len(buf), C.byref(n))
    if n.value >= len(buf) and rc == 0:
        buf = C.create_string_buffer(n.value + 1)
        rc = L.xfk_lua_run(chunk.encode(), buf, len(buf), C.byref(n))
    _check(rc)
    return buf.raw[:n.value].decode("latin-1")


def age_element_matrix(ci: float, co: float, K: float, Ki: float) -> np.ndarray:
    """10 x 10 matrix of one air-gap arc element (host math of the C-ABI,
    cfemm/fsolver/static2d.cpp:209-263)."""
    L = load_library()
    out = np.zeros(100)
    rc = L.xfk_age_element_matrix(ci, co, K, Ki, out.ctypes.data_as(dptr))
    if rc != 0:
        raise XfkError("xfk_age_element_matrix failed (%d)" % rc)
    return out.reshape(10, 10)


class Static2DProblem:
    """One device-resident static 2-D magnetostatic problem (FSolver::Static2D).

    Arrays follow the reference's in-memory state after FSolver::LoadMesh and
    LoadProblemFile (cm coordinates, 0-based indices, -1 for "none")."""

    def __init__(self, *, x, y, p, lbl, blocks: Sequence[dict], labels: Sequence[dict],
                 lines: Sequence[dict] = (), points: Sequence[dict] = (), circuits: Sequence[dict] = (),
                 marker=None, e=None, pbc=None, precision=1e-8, length_units=0, coords=0, relax=1.0,
                 device=0, comm: Optional["Comm"] = None, precond: str = "amg", amg_sweeps: Optional[int] = None,
                 amg_theta: Optional[float] = None, frequency: float = 0.0, amg_omega: Optional[float] = None,
                 amg_replicate: Optional[int] = None, amg_reuse: Optional[bool] = None, problem_type: int = 0,
                 ext_zo: float = 0.0, ext_ro: float = 0.0, ext_ri: float = 0.0, amg_dense: Optional[int] = None,
                 ages: Sequence[dict] = (), ac_solver: int = 0, amg_fold: Optional[bool] = None,
                 amg_col16: Optional[bool] = None, amg_wlevel: Optional[int] = None,
                 amg_f32: Optional[bool] = None, newton_inexact: Optional[bool] = None):
        """ac_solver: [ACSolver], read by the harmonic solvers only (ignored here).
        newton_inexact: nonlinear passes before the last solved to a forcing
        tolerance (default on; False: every pass to Precision, as the
        reference; XFK_OPT_NEWTON_INEXACT).
        amg_fold: folded V(1,1) levels (default on; False: the plain cycle).
        amg_col16: 16-bit tile column offsets on level 0 (default on; False:
        int columns; the same bits either way).
        amg_wlevel: the folded coarse level that runs a W-cycle (default: the
        level above the last V-cycle level; -1: a plain V-cycle).
        amg_f32: f32 values for the V-cycle's level-0 transfers R and P~
        (default on; False: f64; the sweeps and the PCG SpMV stay f64).
        comm: shard the mesh by row blocks over this communicator (every rank
        passes the same global problem; solve() and solution() are collective).
        precond: "amg" (smoothed-aggregation V-cycle, default) or "jacobi".
        problem_type: XFK_PLANAR (Static2D) or XFK_AXISYMMETRIC
        (StaticAxisymmetric: x is r, y is z; solution() is the flux 2 pi r A)."""
        if frequency:
            raise XfkError("frequency != 0: use Harmonic2DProblem")
        L = load_library()
        D, keep = _make_desc(x, y, p, lbl, blocks, labels, lines, points, circuits, marker, e, pbc, precision,
                             length_units, coords, relax, problem_type, (ext_zo, ext_ro, ext_ri), ages)
        self._keep = keep
        self.n_nodes = D.n_nodes
        self.n_elems = D.n_elems
        self.n_circs = len(circuits)
        h = C.c_void_p()
        self.comm = comm
        if comm is None:
            _check(L.xfk_problem_create(C.byref(D), device, C.byref(h)))
        else:
            _check(L.xfk_problem_create_dist(C.byref(D), device, comm._h, C.byref(h)))
        self._h = h
        self.set_option(XFK_OPT_PRECOND, PRECONDS[precond])
        if amg_sweeps is not None:
            self.set_option(XFK_OPT_AMG_SWEEPS, amg_sweeps)
        if amg_theta is not None:
            self.set_option(XFK_OPT_AMG_THETA, amg_theta)
        if amg_omega is not None:
            self.set_option(XFK_OPT_AMG_OMEGA, amg_omega)
        if amg_replicate is not None:
            self.set_option(XFK_OPT_AMG_REPLICATE, amg_replicate)
        if amg_reuse is not None:
            self.set_option(XFK_OPT_AMG_REUSE, int(bool(amg_reuse)))
        if amg_dense is not None:
            self.set_option(XFK_OPT_AMG_DENSE, amg_dense)
        if amg_fold is not None:
            self.set_option(XFK_OPT_AMG_FOLD, int(bool(amg_fold)))
        if amg_col16 is not None:
            self.set_option(XFK_OPT_AMG_COL16, int(bool(amg_col16)))
        if amg_f32 is not None:
            self.set_option(XFK_OPT_AMG_F32, int(bool(amg_f32)))
        if amg_wlevel is not None:
            self.set_option(XFK_OPT_AMG_WLEVEL, int(amg_wlevel))
        if newton_inexact is not None:
            self.set_option(XFK_OPT_NEWTON_INEXACT, int(bool(newton_inexact)))
        self.n_rows = self.dist_info()["n_own"] if comm is not None else self.n_nodes
        self.result: Optional[Result] = None

    def set_option(self, option: int, value: float):
        _check(_lib.xfk_set_option(self._h, option, float(value)))

    def memory(self) -> dict:
        """Device memory of this problem (xfk_problem_memory): arena chunk
        bytes and count, bytes carved and live, bytes kept for reuse."""
        out = (C.c_longlong * 4)()
        _check(_lib.xfk_problem_memory(self._h, out))
        return dict(chunk_bytes=int(out[0]), chunks=int(out[1]), live_bytes=int(out[2]), reuse_bytes=int(out[3]))

    def dist_info(self) -> dict:
        info = DistInfo()
        _check(_lib.xfk_dist_get_info(self._h, C.byref(info)))
        return info.as_dict()

    def close(self):
        if getattr(self, "_h", None):
            load_library().xfk_problem_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def solve(self, rebuild_symbolic: bool = False, time_spmv: bool = False, time_tail: bool = False) -> dict:
        r = Result()
        flags = ((XFK_REBUILD_SYMBOLIC if rebuild_symbolic else 0) | (XFK_TIME_SPMV if time_spmv else 0) |
                 (XFK_TIME_TAIL if time_tail else 0))
        _check(_lib.xfk_static2d(self._h, flags, C.byref(r)))
        self.result = r
        return r.as_dict()

    def solution(self) -> np.ndarray:
        A = np.zeros(self.n_nodes)
        _check(_lib.xfk_get_solution(self._h, A.ctypes.data_as(dptr)))
        return A

    def circuits(self):
        n = self.n_circs
        cc = np.zeros(max(1, n), np.int32)
        J = np.zeros(max(1, n))
        dV = np.zeros(max(1, n))
        _check(_lib.xfk_get_circuits(self._h, cc.ctypes.data_as(iptr), J.ctypes.data_as(dptr),
                                     dV.ctypes.data_as(dptr)))
        return cc[:n], J[:n], dV[:n]

    def spmv_col_bytes(self) -> float:
        """Column-index bytes per nonzero of the last solve's PCG SpMV (2: the
        AMG's 16-bit tile offsets, 4: int columns)."""
        return float(_lib.xfk_spmv_col_bytes(self._h))

    def csr(self):
        """This rank's rows (all rows unless sharded; sharded columns are local ids)."""
        nnz = _lib.xfk_get_nnz(self._h)
        rp = np.zeros(self.n_rows + 1, np.int32)
        col = np.zeros(nnz, np.int32)
        val = np.zeros(nnz)
        b = np.zeros(self.n_rows)
        _check(_lib.xfk_get_csr(self._h, rp.ctypes.data_as(iptr), col.ctypes.data_as(iptr),
                                val.ctypes.data_as(dptr), b.ctypes.data_as(dptr)))
        return rp, col, val, b

    def pcg_time(self, iters: int = 50):
        ms_spmv = C.c_double()
        ms_iter = C.c_double()
        _check(_lib.xfk_pcg_time(self._h, iters, C.byref(ms_spmv), C.byref(ms_iter)))
        return ms_spmv.value, ms_iter.value

    def phase_profile(self, iters: int = 10, setup: bool = True):
        """Per-phase HIP-event profile (xfk_phase_profile): list of dicts
        name, calls, ms_total, us_per_call, bytes_per_call."""
        cap = 256
        buf = (Phase * cap)()
        n = C.c_int()
        _check(_lib.xfk_phase_profile(self._h, iters, XFK_PROFILE_SETUP if setup else 0, C.cast(buf, C.c_void_p),
                                      cap, C.byref(n)))
        out = []
        for k in range(n.value):
            ph = buf[k]
            out.append(dict(name=ph.name.decode(), calls=ph.calls, ms_total=ph.ms_total,
                            us_per_call=1e3 * ph.ms_total / max(1, ph.calls), bytes_per_call=ph.bytes_per_call))
        return out


class Phase(C.Structure):
    _fields_ = [("name", C.c_char * 64), ("calls", C.c_int), ("ms_total", C.c_double), ("bytes_per_call", C.c_double)]


XFK_PROFILE_SETUP = 1


class BlockAcDesc(C.Structure):
    _fields_ = [("J_im", C.c_double), ("Theta_hx", C.c_double), ("Theta_hy", C.c_double), ("Lam_d", C.c_double),
                ("H_im", dptr), ("slope_im", dptr)]


class LineAcDesc(C.Structure):
    _fields_ = [("c0_im", C.c_double), ("c1_im", C.c_double), ("Mu", C.c_double), ("Sig", C.c_double)]


class CircuitAcDesc(C.Structure):
    _fields_ = [("amps_im", C.c_double), ("dvolts_im", C.c_double)]


class HarmonicDesc(C.Structure):
    _fields_ = [("frequency", C.c_double), ("blocks", C.POINTER(BlockAcDesc)), ("lines", C.POINTER(LineAcDesc)),
                ("circs", C.POINTER(CircuitAcDesc)), ("ac_solver", C.c_int),
                ("label_prox_mu", C.POINTER(C.c_double))]


class Harmonic2DProblem:
    """One device-resident time-harmonic planar problem (FSolver::Harmonic2D).
    Same keyword arguments as Static2DProblem plus ``frequency`` (Hz) and the
    AC fields: blocks J_im, Theta_hx, Theta_hy, Lam_d; lines c0_im, c1_im, Mu,
    Sig (BdryFormat 1); circuits amps_im, dvolts_im."""

    def __init__(self, *, x, y, p, lbl, blocks: Sequence[dict], labels: Sequence[dict], frequency: float,
                 lines: Sequence[dict] = (), points: Sequence[dict] = (), circuits: Sequence[dict] = (),
                 marker=None, e=None, pbc=None, precision=1e-8, length_units=0, coords=0, relax=1.0, device=0,
                 problem_type: int = 0, ext_zo: float = 0.0, ext_ro: float = 0.0, ext_ri: float = 0.0,
                 precond: str = "amg", ages: Sequence[dict] = (), ac_solver: int = 0,
                 comm: Optional["Comm"] = None):
        """precond: "amg" (V-cycle of the real SPD surrogate Re A +- Im A, the
        sign making Im A positive semi-definite, applied to the real and
        imaginary parts; default) or "jacobi" (complex Jacobi).  ac_solver:
        [ACSolver], 0 successive approximation, 1 Newton (KludgeSolve).
        comm: shard the rows over this communicator, as Static2DProblem does
        (xfk_problem_create_harmonic_dist); solution() gathers the whole field."""
        L = load_library()
        D, keep = _make_desc(x, y, p, lbl, blocks, labels, lines, points, circuits, marker, e, pbc, precision,
                             length_units, coords, relax, problem_type, (ext_zo, ext_ro, ext_ri), ages)
        ba = (BlockAcDesc * max(1, len(blocks)))()
        for k, b in enumerate(blocks):
            ba[k].J_im, ba[k].Lam_d = b.get("J_im", 0.0), b.get("Lam_d", 0.0)
            ba[k].Theta_hx, ba[k].Theta_hy = b.get("Theta_hx", 0.0), b.get("Theta_hy", 0.0)
            if len(b.get("B", ())):   # nonlinear: the complex curve of bh_get_slopes_ac
                ba[k].H_im = keep.d(np.imag(np.asarray(b["H"])))
                ba[k].slope_im = keep.d(np.imag(np.asarray(b["slope"])))
        la = (LineAcDesc * max(1, len(lines)))()
        for k, l in enumerate(lines):
            la[k].c0_im, la[k].c1_im, la[k].Mu, la[k].Sig = (l.get("c0_im", 0.0), l.get("c1_im", 0.0),
                                                             l.get("Mu", 0.0), l.get("Sig", 0.0))
        ca = (CircuitAcDesc * max(1, len(circuits)))()
        for k, q in enumerate(circuits):
            ca[k].amps_im, ca[k].dvolts_im = q.get("amps_im", 0.0), q.get("dvolts_im", 0.0)
        # labels' "prox_mu": ProximityMu after GetFillFactor (wound LamType > 2 regions)
        prox = np.zeros(2 * max(1, len(labels)))
        for k, l in enumerate(labels):
            z = complex(l.get("prox_mu", 1.0))
            prox[2 * k], prox[2 * k + 1] = z.real, z.imag
        H = HarmonicDesc(frequency, ba, la, ca, int(ac_solver), keep.d(prox))
        keep.extend([ba, la, ca])
        self._keep = keep
        self.n_nodes = D.n_nodes
        self.n_circs = len(circuits)
        h = C.c_void_p()
        self.comm = comm
        if comm is None:
            _check(L.xfk_problem_create_harmonic(C.byref(D), C.byref(H), device, C.byref(h)))
        else:
            _check(L.xfk_problem_create_harmonic_dist(C.byref(D), C.byref(H), device, comm._h, C.byref(h)))
        self._h = h
        _check(L.xfk_set_option(self._h, XFK_OPT_PRECOND, float(PRECONDS[precond])))
        self.n_rows = self.dist_info()["n_own"] if comm is not None else self.n_nodes
        self.result: Optional[Result] = None

    def solve(self, rebuild_symbolic: bool = False) -> dict:
        r = Result()
        _check(_lib.xfk_harmonic2d(self._h, XFK_REBUILD_SYMBOLIC if rebuild_symbolic else 0, C.byref(r)))
        self.result = r
        return r.as_dict()

    def memory(self) -> dict:
        """Device memory of this problem (xfk_problem_memory): arena chunk
        bytes and count, bytes carved and live, bytes kept for reuse."""
        out = (C.c_longlong * 4)()
        _check(_lib.xfk_problem_memory(self._h, out))
        return dict(chunk_bytes=int(out[0]), chunks=int(out[1]), live_bytes=int(out[2]), reuse_bytes=int(out[3]))

    def dist_info(self) -> dict:
        info = DistInfo()
        _check(_lib.xfk_dist_get_info(self._h, C.byref(info)))
        return info.as_dict()

    def solution(self) -> np.ndarray:
        A = np.zeros(2 * self.n_nodes)
        _check(_lib.xfk_get_solution_complex(self._h, A.ctypes.data_as(dptr)))
        return A[0::2] + 1j * A[1::2]

    def circuits(self):
        n = self.n_circs
        cc = np.zeros(max(1, n), np.int32)
        J = np.zeros(2 * max(1, n))
        dV = np.zeros(2 * max(1, n))
        _check(_lib.xfk_get_circuits_complex(self._h, cc.ctypes.data_as(iptr), J.ctypes.data_as(dptr),
                                             dV.ctypes.data_as(dptr)))
        return cc[:n], (J[0::2] + 1j * J[1::2])[:n], (dV[0::2] + 1j * dV[1::2])[:n]

    def csr(self):
        nnz = _lib.xfk_get_nnz(self._h)
        rp = np.zeros(self.n_rows + 1, np.int32)
        col = np.zeros(nnz, np.int32)
        val = np.zeros(2 * nnz)
        b = np.zeros(2 * self.n_rows)
        _check(_lib.xfk_get_csr_complex(self._h, rp.ctypes.data_as(iptr), col.ctypes.data_as(iptr),
                                        val.ctypes.data_as(dptr), b.ctypes.data_as(dptr)))
        return rp, col, val[0::2] + 1j * val[1::2], b[0::2] + 1j * b[1::2]

    def close(self):
        if getattr(self, "_h", None):
            load_library().xfk_problem_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def pcg_solve_csr(rowptr, col, val, b, V0=None, flag=0, precision=1e-8, device=0, precond="jacobi"):
    """Stand-alone device PCG on a full symmetric CSR (CBigLinProb::PCGSolve semantics)."""
    L = load_library()
    n = len(rowptr) - 1
    rp = np.ascontiguousarray(rowptr, np.int32)
    cl = np.ascontiguousarray(col, np.int32)
    vl = np.ascontiguousarray(val, np.float64)
    bb = np.ascontiguousarray(b, np.float64)
    V = np.zeros(n) if V0 is None else np.array(V0, dtype=np.float64)
    it = C.c_longlong()
    er = C.c_double()
    _check(L.xfk_pcg_solve_csr_pc(n, rp.ctypes.data_as(iptr), cl.ctypes.data_as(iptr), vl.ctypes.data_as(dptr),
                                  bb.ctypes.data_as(dptr), V.ctypes.data_as(dptr), flag, precision, device,
                                  PRECONDS[precond], C.byref(it), C.byref(er)))
    return V, it.value, er.value


class CommOp(C.Structure):
    _fields_ = [("seq", C.c_longlong), ("op", C.c_int), ("stream", C.c_int), ("waited", C.c_int),
                ("peer", C.c_int), ("bytes", C.c_longlong), ("g0", C.c_longlong)]


COMM_OPS = {1: "allreduce", 2: "exchange", 3: "send", 4: "recv", 5: "allgather"}


class Comm:
    """Communicator of the sharded solve (xfk_comm): RCCL, one process per GPU,
    an in-process group of ranks driven by one host thread each, or the replay
    of one rank's recording (compute-only runs of a sharded rank)."""

    def __init__(self, handle):
        self._h = handle
        L = load_library()
        self.rank = L.xfk_comm_rank(handle)
        self.size = L.xfk_comm_size(handle)

    @staticmethod
    def unique_id() -> bytes:
        buf = C.create_string_buffer(128)
        _check(load_library().xfk_comm_unique_id(buf, 128))
        return buf.raw

    @classmethod
    def rccl(cls, unique_id: bytes, rank: int, size: int, device: int) -> "Comm":
        h = C.c_void_p()
        _check(load_library().xfk_comm_create_rccl(unique_id, len(unique_id), rank, size, device, C.byref(h)))
        return cls(h)

    @classmethod
    def local_group(cls, size: int) -> list:
        hs = (C.c_void_p * size)()
        _check(load_library().xfk_comm_create_local(size, hs))
        return [cls(C.c_void_p(hs[q])) for q in range(size)]

    def record(self, mode: int = 1):
        """Start an empty recording (1: the collective sequence; 2: also every
        received byte, for replay()); 0 stops it (the log stays readable)."""
        _check(load_library().xfk_comm_record(self._h, int(mode)))

    def log(self) -> list:
        """The recorded collectives: dicts seq, op (allreduce / exchange / send /
        recv / allgather), stream, waited, peer, bytes, g0 (xfk_comm_op)."""
        L = load_library()
        n = C.c_int()
        _check(L.xfk_comm_log(self._h, None, 0, C.byref(n)))
        buf = (CommOp * max(1, n.value))()
        _check(L.xfk_comm_log(self._h, C.cast(buf, C.c_void_p), n.value, C.byref(n)))
        return [dict(seq=o.seq, op=COMM_OPS.get(o.op, str(o.op)), stream=o.stream, waited=o.waited, peer=o.peer,
                     bytes=o.bytes, g0=o.g0) for o in buf[:n.value]]

    def time(self, on: bool = True):
        """Bracket every collective with HIP events (xfk_comm_time)."""
        _check(load_library().xfk_comm_time(self._h, int(bool(on))))

    def timing(self) -> dict:
        """Per op (allreduce / exchange / allgather): calls, summed and longest
        microseconds inside the collectives since the last read
        (xfk_comm_timing; waits for the events, then clears them)."""
        calls = (C.c_longlong * 3)()
        tot = (C.c_double * 3)()
        mx = (C.c_double * 3)()
        _check(load_library().xfk_comm_timing(self._h, calls, tot, mx))
        return {nm: {"calls": int(calls[k]), "us": float(tot[k]), "us_max_call": float(mx[k])}
                for k, nm in enumerate(("allreduce", "exchange", "allgather"))}

    def replay(self) -> "Comm":
        """A communicator serving this rank's mode-2 recording cyclically
        (xfk_comm_create_replay): the rank runs alone with the recorded inputs."""
        h = C.c_void_p()
        _check(load_library().xfk_comm_create_replay(self._h, C.byref(h)))
        return Comm(h)

    def close(self):
        if getattr(self, "_h", None):
            load_library().xfk_comm_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def check_comm_logs(logs) -> dict:
    """Issue-order check of one recorded program over all ranks (logs[q] =
    Comm.log() of rank q): every rank made the same sequence of collective
    calls -- op, stream index, payload bytes of all-reduces and all-gathers --
    and in every exchange each send of rank a to rank b matches a receive of b
    from a (length and first global row) in the same exchange, and the reverse.
    Raises AssertionError naming the first mismatch; returns a summary."""
    R = len(logs)
    calls = []
    for q, lg in enumerate(logs):
        cs = {}
        for o in lg:
            c = cs.setdefault(o["seq"], {"head": None, "send": [], "recv": []})
            if o["op"] in ("send", "recv"):
                c[o["op"]].append((o["peer"], o["bytes"], o["g0"]))
            else:
                c["head"] = (o["op"], o["stream"], o["bytes"] if o["op"] != "exchange" else 0)
        calls.append([cs[k] for k in sorted(cs)])
    n = len(calls[0])
    for q in range(1, R):
        assert len(calls[q]) == n, "rank %d made %d collective calls, rank 0 %d" % (q, len(calls[q]), n)
    waits = 0
    streams = set()
    for k in range(n):
        h0 = calls[0][k]["head"]
        for q in range(1, R):
            assert calls[q][k]["head"] == h0, "call %d: rank 0 %s, rank %d %s" % (k, h0, q, calls[q][k]["head"])
        streams.add(h0[1])
        if h0[0] != "exchange":
            continue
        for a in range(R):
            for (b, nb, g0) in calls[a][k]["send"]:
                assert (a, nb, g0) in calls[b][k]["recv"], \
                    "exchange %d: rank %d sends %d B (row %d) to %d, which posts no such receive" % (k, a, nb, g0, b)
            for (b, nb, g0) in calls[a][k]["recv"]:
                assert (a, nb, g0) in calls[b][k]["send"], \
                    "exchange %d: rank %d expects %d B (row %d) from %d, which sends no such range" % (k, a, nb, g0, b)
    for lg in logs:
        prev = None
        for o in lg:
            if o["op"] in ("send", "recv"):
                continue
            if prev is not None and o["stream"] != prev:
                assert o["waited"] == 1, "call %d changes stream without the ordering wait" % o["seq"]
            waits += o["waited"]
            prev = o["stream"]
    ops = {}
    for c in calls[0]:
        ops[c["head"][0]] = ops.get(c["head"][0], 0) + 1
    return {"calls": n, "ops": ops, "streams": sorted(streams), "stream_switches": waits}


def partition_plan(n_nodes: int, p, rank: int, nranks: int, coupled=None) -> dict:
    """Host-only row-block partition plan of xfk_problem_create_dist (no device);
    ``coupled``: periodic / air-gap nodes (xfk_partition_plan_coupled)."""
    L = load_library()
    p = np.ascontiguousarray(np.asarray(p, dtype=np.int32).reshape(-1))
    ne = len(p) // 3
    info = DistInfo()
    pp = p.ctypes.data_as(iptr)
    cp = np.ascontiguousarray(np.asarray([] if coupled is None else coupled, dtype=np.int32).reshape(-1))
    nc = len(cp)
    cpp = cp.ctypes.data_as(iptr) if nc else None
    _check(L.xfk_partition_plan_coupled(n_nodes, ne, pp, rank, nranks, nc, cpp, C.byref(info), None, None, None,
                                        None))
    l2g = np.zeros(info.n_own + info.n_halo, np.int32)
    elems = np.zeros(max(1, info.n_elems), np.int32)
    recv = np.zeros(4 * max(1, info.n_recv), np.int32)
    send = np.zeros(4 * max(1, info.n_send), np.int32)
    _check(L.xfk_partition_plan_coupled(n_nodes, ne, pp, rank, nranks, nc, cpp, C.byref(info),
                                        l2g.ctypes.data_as(iptr), elems.ctypes.data_as(iptr),
                                        recv.ctypes.data_as(iptr), send.ctypes.data_as(iptr)))
    d = info.as_dict()
    d["l2g"] = l2g
    d["elems"] = elems[:info.n_elems]
    d["recv"] = recv[:4 * info.n_recv].reshape(-1, 4)   # peer, local offset, length, first global row
    d["send"] = send[:4 * info.n_send].reshape(-1, 4)
    return d
