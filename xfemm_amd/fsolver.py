"""Python view of the file-based FSolver (include/xfemm_fsolver.h).

Mirrors the reference's FSolver surface (cfemm/fsolver/fsolver.h) with the
same names: ``PathName``, ``LoadProblemFile()``, ``runSolver(verbose)``,
``LoadMesh()``, ``Cuthill()``.  The solve itself runs on the GPU; there is no
CPU fallback.
"""
from __future__ import annotations

import ctypes as C
import os

import numpy as np

from . import kernels

FSOLVER_SO = os.path.join(kernels.LIB_DIR, "libxfemm_fsolver.so")

EXPORTED = (
    "xfemm_fsolver_create", "xfemm_fsolver_destroy", "xfemm_fsolver_set_message_handlers",
    "xfemm_fsolver_set_pathname", "xfemm_fsolver_set_device", "xfemm_fsolver_set_delete_mesh_files",
    "xfemm_fsolver_load_problem_file", "xfemm_fsolver_run_solver", "xfemm_fsolver_load_mesh",
    "xfemm_fsolver_cuthill", "xfemm_fsolver_get_nodes", "xfemm_fsolver_get_element_edges",
    "xfemm_fsolver_get_pbcs", "xfemm_fsolver_num_pbcs", "xfemm_fsolver_bandwidth",
    "xfemm_fsolver_get_block_bh", "xfemm_fsolver_num_nodes", "xfemm_fsolver_num_elements",
    "xfemm_fsolver_get_solution", "xfemm_fsolver_get_elements", "xfemm_fsolver_get_stats",
    "xfemm_fsolver_get_times",
    "xfemm_fsolver_last_error", "xfemm_bh_get_slopes", "xfemm_bh_get_slopes_ac",
    "xfemm_fsolver_set_previous_solution_file", "xfemm_fsolver_previous_solution_file", "xfemm_fsolver_ac_solver",
    "xfemm_fsolver_frequency", "xfemm_fsolver_num_line_props", "xfemm_fsolver_num_node_props",
    "xfemm_fsolver_num_block_props", "xfemm_fsolver_num_circ_props", "xfemm_fsolver_num_block_labels",
    "xfemm_fsolver_set_comm", "xfemm_fsolver_num_air_gaps", "xfemm_fsolver_get_air_gap_nodes",
)

_lib = None
dptr = kernels.dptr
iptr = kernels.iptr


def load_library(path: str = FSOLVER_SO):
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(path):
        raise kernels.XfkError("%s not built (run __graft_entry__.build())" % path)
    kernels.load_library()
    L = C.CDLL(path)
    vp = C.c_void_p
    L.xfemm_fsolver_create.restype = vp
    for nm in ("xfemm_fsolver_destroy",):
        getattr(L, nm).argtypes = [vp]
    L.xfemm_fsolver_set_pathname.argtypes = [vp, C.c_char_p]
    L.xfemm_fsolver_set_device.argtypes = [vp, C.c_int]
    L.xfemm_fsolver_set_delete_mesh_files.argtypes = [vp, C.c_int]
    L.xfemm_fsolver_set_comm.argtypes = [vp, vp]
    for nm in ("xfemm_fsolver_load_problem_file", "xfemm_fsolver_load_mesh", "xfemm_fsolver_cuthill",
               "xfemm_fsolver_num_nodes", "xfemm_fsolver_num_elements", "xfemm_fsolver_num_pbcs",
               "xfemm_fsolver_bandwidth", "xfemm_fsolver_num_air_gaps"):
        getattr(L, nm).argtypes = [vp]
        getattr(L, nm).restype = C.c_int
    L.xfemm_fsolver_run_solver.argtypes = [vp, C.c_int]
    L.xfemm_fsolver_get_nodes.argtypes = [vp, dptr, dptr, iptr]
    L.xfemm_fsolver_get_element_edges.argtypes = [vp, iptr]
    L.xfemm_fsolver_get_pbcs.argtypes = [vp, iptr]
    L.xfemm_fsolver_get_air_gap_nodes.argtypes = [vp, iptr, iptr]
    L.xfemm_fsolver_get_air_gap_nodes.restype = C.c_int
    L.xfemm_fsolver_get_block_bh.argtypes = [vp, C.c_int, dptr, dptr, dptr, dptr]
    L.xfemm_fsolver_get_solution.argtypes = [vp, dptr, dptr, dptr]
    L.xfemm_fsolver_get_elements.argtypes = [vp, iptr, iptr]
    L.xfemm_fsolver_get_stats.argtypes = [vp, C.POINTER(kernels.Result)]
    L.xfemm_fsolver_get_times.argtypes = [vp, C.POINTER(C.c_double)]
    L.xfemm_fsolver_last_error.argtypes = [vp]
    L.xfemm_fsolver_set_previous_solution_file.argtypes = [vp, C.c_char_p]
    L.xfemm_fsolver_previous_solution_file.argtypes = [vp]
    L.xfemm_fsolver_previous_solution_file.restype = C.c_char_p
    L.xfemm_fsolver_frequency.argtypes = [vp]
    L.xfemm_fsolver_frequency.restype = C.c_double
    for nm in ("xfemm_fsolver_ac_solver", "xfemm_fsolver_num_line_props", "xfemm_fsolver_num_node_props",
               "xfemm_fsolver_num_block_props", "xfemm_fsolver_num_circ_props", "xfemm_fsolver_num_block_labels"):
        getattr(L, nm).argtypes = [vp]
        getattr(L, nm).restype = C.c_int
    L.xfemm_fsolver_last_error.restype = C.c_char_p
    L.xfemm_bh_get_slopes.argtypes = [C.c_int, dptr, dptr, dptr, C.c_int, C.c_double, dptr]
    L.xfemm_bh_get_slopes_ac.argtypes = [C.c_int, dptr, dptr, dptr, dptr, dptr, C.c_double, C.c_int, C.c_double,
                                         C.c_double, C.c_double, C.c_double, dptr, dptr]
    _lib = L
    return L


def bh_get_slopes(B, H, lam_type=0, lam_fill=1.0):
    """CMMaterialProp::GetSlopes(0) on a B-H table -> (B, H, slope, mu_x)."""
    L = load_library()
    B = np.array(B, dtype=np.float64)
    H = np.array(H, dtype=np.float64)
    S = np.zeros_like(B)
    mu = C.c_double()
    if not L.xfemm_bh_get_slopes(len(B), B.ctypes.data_as(dptr), H.ctypes.data_as(dptr),
                                 S.ctypes.data_as(dptr), lam_type, lam_fill, C.byref(mu)):
        raise ValueError("bad B-H curve")
    return B, H, S, mu.value


def bh_get_slopes_ac(B, H, omega, lam_type=0, lam_fill=1.0, theta_hn=0.0, lam_d=0.0, cduct=0.0):
    """CMMaterialProp::GetSlopes(omega > 0) on a B-H table (the harmonic
    solver's curve: effective sinusoidal-H amplitude, hysteresis lag,
    laminations) -> (B, H complex, slope complex, mu_x, MuMax)."""
    L = load_library()
    B = np.array(B, dtype=np.float64)
    H = np.array(H, dtype=np.float64)
    Hi, S, Si = np.zeros_like(B), np.zeros_like(B), np.zeros_like(B)
    mu, mm = C.c_double(), C.c_double()
    if not L.xfemm_bh_get_slopes_ac(len(B), B.ctypes.data_as(dptr), H.ctypes.data_as(dptr), Hi.ctypes.data_as(dptr),
                                    S.ctypes.data_as(dptr), Si.ctypes.data_as(dptr), omega, lam_type, lam_fill,
                                    theta_hn, lam_d, cduct, C.byref(mu), C.byref(mm)):
        raise ValueError("bad B-H curve")
    return B, H + 1j * Hi, S + 1j * Si, mu.value, mm.value


class FSolver:
    """The reference FSolver workflow over the MI355X hot path."""

    def __init__(self, device: int = 0, delete_mesh_files: bool = True, comm=None):
        L = load_library()
        self._h = C.c_void_p(L.xfemm_fsolver_create())
        L.xfemm_fsolver_set_device(self._h, device)
        L.xfemm_fsolver_set_delete_mesh_files(self._h, int(delete_mesh_files))
        self._path = ""
        self._comm = None
        if comm is not None:
            self.set_comm(comm)

    def set_comm(self, comm):
        """Shard the solve over comm's ranks (xfemm_fsolver_set_comm; a
        kernels.Comm kept alive by this object): every rank runs its own
        FSolver on the same files, rank 0 writes the .ans."""
        self._comm = comm
        _lib.xfemm_fsolver_set_comm(self._h, comm._h if comm is not None else None)

    def __del__(self):
        try:
            if self._h:
                _lib.xfemm_fsolver_destroy(self._h)
                self._h = None
        except Exception:
            pass

    @property
    def PathName(self) -> str:
        return self._path

    @PathName.setter
    def PathName(self, p: str):
        self._path = p
        _lib.xfemm_fsolver_set_pathname(self._h, p.encode())

    @property
    def previousSolutionFile(self) -> str:
        """FSolver::previousSolutionFile; femmcli sets it before LoadProblemFile
        (LuaMagneticsCommands.cpp:824), a [PrevSoln] line of the .fem overrides it."""
        return _lib.xfemm_fsolver_previous_solution_file(self._h).decode()

    @previousSolutionFile.setter
    def previousSolutionFile(self, p: str):
        _lib.xfemm_fsolver_set_previous_solution_file(self._h, p.encode())

    @property
    def ACSolver(self) -> int:
        return _lib.xfemm_fsolver_ac_solver(self._h)

    @property
    def Frequency(self) -> float:
        return _lib.xfemm_fsolver_frequency(self._h)

    def list_sizes(self) -> dict:
        """The property-list sizes femmcli asserts on (LuaMagneticsCommands.cpp:832-838)."""
        h = self._h
        return dict(lineproplist=_lib.xfemm_fsolver_num_line_props(h), nodeproplist=_lib.xfemm_fsolver_num_node_props(h),
                    blockproplist=_lib.xfemm_fsolver_num_block_props(h),
                    circproplist=_lib.xfemm_fsolver_num_circ_props(h), labellist=_lib.xfemm_fsolver_num_block_labels(h))

    def LoadProblemFile(self) -> bool:
        return bool(_lib.xfemm_fsolver_load_problem_file(self._h))

    def LoadMesh(self) -> bool:
        return bool(_lib.xfemm_fsolver_load_mesh(self._h))

    def Cuthill(self) -> bool:
        return bool(_lib.xfemm_fsolver_cuthill(self._h))

    def runSolver(self, verbose: bool = False) -> bool:
        return bool(_lib.xfemm_fsolver_run_solver(self._h, int(verbose)))

    def last_error(self) -> str:
        return _lib.xfemm_fsolver_last_error(self._h).decode()

    @property
    def NumNodes(self) -> int:
        return _lib.xfemm_fsolver_num_nodes(self._h)

    @property
    def NumEls(self) -> int:
        return _lib.xfemm_fsolver_num_elements(self._h)

    @property
    def BandWidth(self) -> int:
        return _lib.xfemm_fsolver_bandwidth(self._h)

    def nodes(self):
        n = self.NumNodes
        x, y = np.zeros(n), np.zeros(n)
        m = np.zeros(n, np.int32)
        _lib.xfemm_fsolver_get_nodes(self._h, x.ctypes.data_as(dptr), y.ctypes.data_as(dptr),
                                     m.ctypes.data_as(iptr))
        return x, y, m

    def elements(self):
        ne = self.NumEls
        p = np.zeros((ne, 3), np.int32)
        lbl = np.zeros(ne, np.int32)
        e = np.zeros((ne, 3), np.int32)
        _lib.xfemm_fsolver_get_elements(self._h, p.ctypes.data_as(iptr), lbl.ctypes.data_as(iptr))
        _lib.xfemm_fsolver_get_element_edges(self._h, e.ctypes.data_as(iptr))
        return p, lbl, e

    def pbcs(self):
        n = _lib.xfemm_fsolver_num_pbcs(self._h)
        a = np.zeros((max(n, 1), 3), np.int32)
        _lib.xfemm_fsolver_get_pbcs(self._h, a.ctypes.data_as(iptr))
        return a[:n]

    def air_gap_nodes(self):
        """(counts, quad) of FEASolver::agelist: quadNodes per air gap and their
        node ids n0..n3, one row per quadNode (renumbered after Cuthill)."""
        na = _lib.xfemm_fsolver_num_air_gaps(self._h)
        counts = np.zeros(max(na, 1), np.int32)
        nq = _lib.xfemm_fsolver_get_air_gap_nodes(self._h, counts.ctypes.data_as(iptr), None)
        quad = np.zeros((max(nq, 1), 4), np.int32)
        _lib.xfemm_fsolver_get_air_gap_nodes(self._h, None, quad.ctypes.data_as(iptr))
        return counts[:na], quad[:nq]

    def block_bh(self, k: int, nmax: int = 4096):
        B, H, S = np.zeros(nmax), np.zeros(nmax), np.zeros(nmax)
        mu = C.c_double()
        n = _lib.xfemm_fsolver_get_block_bh(self._h, k, B.ctypes.data_as(dptr), H.ctypes.data_as(dptr),
                                            S.ctypes.data_as(dptr), C.byref(mu))
        return B[:n], H[:n], S[:n], mu.value

    def solution(self):
        n = self.NumNodes
        x, y, A = np.zeros(n), np.zeros(n), np.zeros(n)
        if not _lib.xfemm_fsolver_get_solution(self._h, x.ctypes.data_as(dptr), y.ctypes.data_as(dptr),
                                               A.ctypes.data_as(dptr)):
            raise RuntimeError("no solution")
        return x, y, A

    def times(self) -> dict:
        """Wall milliseconds of the last runSolver, split as the reference's
        sequence runs: load_mesh, cuthill, create (descriptor + upload),
        solve (device + read-back), write (.ans)."""
        ms = (C.c_double * 5)()
        _lib.xfemm_fsolver_get_times(self._h, ms)
        return dict(zip(("ms_load_mesh", "ms_cuthill", "ms_create", "ms_solve", "ms_write"), list(ms)))

    def stats(self) -> dict:
        r = kernels.Result()
        _lib.xfemm_fsolver_get_stats(self._h, C.byref(r))
        return r.as_dict()
