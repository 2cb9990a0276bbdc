"""fmesher restatement: .fem geometry -> .node / .ele / .edge / .pbc (fixture tool).

TEST INFRASTRUCTURE ONLY.  It makes the meshes of the reference's own machine
models (``test/TorqueBenchmark.fem``, BASELINE.json configs[0]/[1]) so that the
GPU solver and the CPU oracle can be run on them; the meshes it writes are
committed under ``tests/golden/`` and nothing on the product path imports it.

The reference's fmesher cannot be built here: ``writepoly.cpp:39`` includes
``triangle_api.h``, which /root/reference does not ship.  The Triangle library
it drives (``cfemm/fmesher/triangle/triangle.c``, the XFEMM_BUILTIN_TRIANGLE
variant with the 5-argument ``triangulate``) is self-contained and is compiled
from the reference sources into ``oracle/_ref/libtriangle.so`` by
``oracle/Makefile``.  This module restates the driver around it:

  * FMesher::DoPeriodicBCTriangulation       cfemm/fmesher/writepoly.cpp:823-2026
  * FMesher::DoNonPeriodicBCTriangulation    writepoly.cpp:711-811
  * fmesher::discretizeInputSegments         writepoly.cpp:263-399
  * fmesher::discretizeInputArcSegments      writepoly.cpp:401-466
  * fmesher::defaultMeshSizeHeuristics       writepoly.cpp:238-261
  * TriangulateHelper (points, segments, holes/regions, switches, file layout)
                                             writepoly.cpp:543-698, 2067-2404
  * FemmProblem::getCircle                   cfemm/libfemm/FemmProblem.cpp:1523-1547
  * FemmReader geometry sections              cfemm/libfemm/FemmReader.cpp:367-575

Complex arithmetic follows femmcomplex.cpp (product, scaled-reciprocal quotient,
``abs`` as |re| sqrt(1 + (im/re)^2), ``exp`` through sin/cos).

Reference quirks kept on purpose (they shape the mesh the reference produces):
  * AGE arcs: ``totalArcElements += IsSelected`` (writepoly.cpp:1193) adds 0 for
    every arc read from a file, so the AGE spacing is always the
    ``(360/pi)(ro-ri)/(ro+ri)`` limit rounded to 2 significant digits;
  * the ring segments of an AGE carry the boundary name the previous periodic
    arc pair left in the shared ``segm`` (writepoly.cpp:1537, 1663): harmless
    to the solver (periodic markers add no element terms).

Parity of the mesh with the reference's fmesher is **unpinned** (no reference
mesh of these models exists); what is pinned is the physics the reference's
own test asserts on the result (femmcli/test/femmcli_TorqueBenchmark.lua:
torque = sin(rotor angle) N m), see oracle/gaptorque.py.
"""
from __future__ import annotations

import ctypes
import math
import os
from dataclasses import dataclass, field
from typing import List, Optional

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
PI = 3.141592653589793238462643383       # femmconstants.h
DEGREE = 0.01745329251994329576923690768
LINE_FRACTION = 500.0                     # writepoly.cpp:58
BOUNDING_BOX_FRACTION = 100.0             # writepoly.cpp:64
MINANGLE_BUMP = 3.0                       # femmconstants.h:32
MINANGLE_MAX = 33.8


# --------------------------------------------------------------------------
# femmcomplex.cpp arithmetic
# --------------------------------------------------------------------------

def c_abs(z: complex) -> float:             # femmcomplex.cpp:749-757
    re, im = z.real, z.imag
    if re == 0 and im == 0:
        return 0.0
    if abs(re) > abs(im):
        return abs(re) * math.sqrt(1. + (im / re) * (im / re))
    return abs(im) * math.sqrt(1. + (re / im) * (re / im))


def c_div(x: complex, z: complex) -> complex:   # femmcomplex.cpp:362-381
    if abs(z.real) > abs(z.imag):
        c = z.imag / z.real
        yre = 1. / (z.real * (1. + c * c))
        yim = (-c) * yre
    else:
        c = z.real / z.imag
        yim = (-1.) / (z.imag * (1. + c * c))
        yre = (-c) * yim
    return c_mul(x, complex(yre, yim))


def c_mul(x: complex, y: complex) -> complex:   # femmcomplex.cpp:355-358
    return complex(x.real * y.real - x.imag * y.imag, x.real * y.imag + x.imag * y.real)


def c_divd(x: complex, d: float) -> complex:    # femmcomplex.cpp:388-391
    return complex(x.real / d, x.imag / d)


def c_expi(phi: float) -> complex:              # exp(I*phi), femmcomplex.cpp:622-632
    return complex(math.cos(phi) * 1.0, math.sin(phi) * 1.0)


def c_arg(z: complex) -> float:                 # femmcomplex.cpp:764-769
    if z.real == 0 and z.imag == 0:
        return 0.0
    return math.atan2(z.imag, z.real)


def to_degrees(z: complex) -> float:           # writepoly.cpp:69
    a = c_arg(z) if z.imag >= 0 else c_arg(z) + 2. * PI
    return a * (180. / PI)


def c_round(v: float) -> int:                  # C round(): half away from zero
    return int(math.floor(abs(v) + 0.5)) * (1 if v >= 0 else -1)


def fmt_1e(v: float) -> float:                 # sprintf("%.1e") + sscanf("%lf")
    return float("%.1e" % v)


# --------------------------------------------------------------------------
# .fem geometry (FemmReader.cpp) -- only what the mesher reads
# --------------------------------------------------------------------------

@dataclass
class Node:
    x: float
    y: float
    marker: str = "<None>"      # BoundaryMarkerName

    def cc(self) -> complex:
        return complex(self.x, self.y)


@dataclass
class Segment:
    n0: int
    n1: int
    MaxSideLength: float = -1.0
    marker: str = "<None>"
    cnt: int = 0
    IsSelected: bool = False


@dataclass
class Arc(Segment):
    ArcLength: float = 90.0
    NormalDirection: bool = True


@dataclass
class Label:
    x: float
    y: float
    BlockType: int          # -1: hole
    MaxArea: float = 0.0


@dataclass
class BdryProp:
    name: str
    BdryFormat: int
    InnerAngle: float = 0.0
    OuterAngle: float = 0.0


@dataclass
class Geometry:
    nodes: List[Node] = field(default_factory=list)
    lines: List[Segment] = field(default_factory=list)
    arcs: List[Arc] = field(default_factory=list)
    labels: List[Label] = field(default_factory=list)
    bdrys: List[BdryProp] = field(default_factory=list)
    points: List[str] = field(default_factory=list)
    MinAngle: float = 30.0
    DoSmartMesh: bool = True

    def length_of_line(self, s: Segment) -> float:      # FemmProblem.cpp:1656-1660
        return c_abs(self.nodes[s.n0].cc() - self.nodes[s.n1].cc())

    def get_circle(self, arc: Arc):                      # FemmProblem.cpp:1523-1547
        a0 = self.nodes[arc.n0].cc()
        a1 = self.nodes[arc.n1].cc()
        d = c_abs(a1 - a0)
        t = c_divd(a1 - a0, d)
        tta = arc.ArcLength * PI / 180.
        R = d / (2. * math.sin(tta / 2.))
        c = a0 + c_mul(complex(d / 2., math.sqrt(R * R - d * d / 4.)), t)
        return c, R


def _val(tok: str) -> str:
    return tok.split("=", 1)[1].strip()


def parse_geometry(path: str) -> Geometry:
    """The geometry part of FemmReader::parse (FemmReader.cpp:367-575) plus the
    boundary / point property names, MinAngle and DoSmartMesh."""
    g = Geometry()
    with open(path, "r") as fh:
        lines = [ln.rstrip("\r\n") for ln in fh]
    i = 0
    cur_bdry: Optional[dict] = None
    while i < len(lines):
        ln = lines[i].strip()
        i += 1
        low = ln.lower()
        if low.startswith("[minangle]"):
            g.MinAngle = float(_val(ln))
        elif low.startswith("[dosmartmesh]"):
            g.DoSmartMesh = int(float(_val(ln))) != 0
        elif low.startswith("<beginbdry>"):
            cur_bdry = {"name": "", "fmt": 0, "inner": 0.0, "outer": 0.0}
        elif low.startswith("<endbdry>"):
            g.bdrys.append(BdryProp(cur_bdry["name"], cur_bdry["fmt"], cur_bdry["inner"], cur_bdry["outer"]))
            cur_bdry = None
        elif cur_bdry is not None and low.startswith("<bdryname>"):
            cur_bdry["name"] = _val(ln).strip().strip('"')
        elif cur_bdry is not None and low.startswith("<bdrytype>"):
            cur_bdry["fmt"] = int(float(_val(ln)))
        elif cur_bdry is not None and low.startswith("<innerangle>"):
            cur_bdry["inner"] = float(_val(ln))
        elif cur_bdry is not None and low.startswith("<outerangle>"):
            cur_bdry["outer"] = float(_val(ln))
        elif low.startswith("<pointname>"):
            g.points.append(_val(ln).strip().strip('"'))
        elif low.startswith("[numpoints]"):
            for _ in range(int(_val(ln))):
                f = lines[i].split()
                i += 1
                m = int(f[2]) - 1
                g.nodes.append(Node(float(f[0]), float(f[1]), m))   # resolved below
        elif low.startswith("[numsegments]"):
            for _ in range(int(_val(ln))):
                f = lines[i].split()
                i += 1
                g.lines.append(Segment(int(f[0]), int(f[1]), float(f[2]), int(f[3]) - 1))
        elif low.startswith("[numarcsegments]"):
            for _ in range(int(_val(ln))):
                f = lines[i].split()
                i += 1
                g.arcs.append(Arc(int(f[0]), int(f[1]), float(f[3]), int(f[4]) - 1, ArcLength=float(f[2])))
        elif low.startswith("[numholes]"):
            for _ in range(int(_val(ln))):
                f = lines[i].split()
                i += 1
                g.labels.append(Label(float(f[0]), float(f[1]), -1, 0.0))
        elif low.startswith("[numblocklabels]"):
            for _ in range(int(_val(ln))):
                f = lines[i].split()
                i += 1
                ma = float(f[3])
                ma = 0.0 if ma <= 0 else ma * (PI * ma / 4.)        # CBlockLabel.cpp:131-135
                g.labels.append(Label(float(f[0]), float(f[1]), int(f[2]) - 1, ma))
    # FemmProblem::updateLabelsFromIndex (FemmProblem.cpp:254-290)
    for n in g.nodes:
        n.marker = g.points[n.marker] if 0 <= n.marker < len(g.points) else "<None>"
    for s in g.lines + g.arcs:
        s.marker = g.bdrys[s.marker].name if 0 <= s.marker < len(g.bdrys) else "<None>"
    return g


# --------------------------------------------------------------------------
# Triangle (the reference's cfemm/fmesher/triangle/triangle.c, oracle/_ref)
# --------------------------------------------------------------------------

class _TriIO(ctypes.Structure):     # triangle.h:384-413
    _fields_ = [
        ("pointlist", ctypes.POINTER(ctypes.c_double)),
        ("pointattributelist", ctypes.POINTER(ctypes.c_double)),
        ("pointmarkerlist", ctypes.POINTER(ctypes.c_int)),
        ("numberofpoints", ctypes.c_int),
        ("numberofpointattributes", ctypes.c_int),
        ("trianglelist", ctypes.POINTER(ctypes.c_int)),
        ("triangleattributelist", ctypes.POINTER(ctypes.c_double)),
        ("trianglearealist", ctypes.POINTER(ctypes.c_double)),
        ("neighborlist", ctypes.POINTER(ctypes.c_int)),
        ("numberoftriangles", ctypes.c_int),
        ("numberofcorners", ctypes.c_int),
        ("numberoftriangleattributes", ctypes.c_int),
        ("segmentlist", ctypes.POINTER(ctypes.c_int)),
        ("segmentmarkerlist", ctypes.POINTER(ctypes.c_int)),
        ("numberofsegments", ctypes.c_int),
        ("holelist", ctypes.POINTER(ctypes.c_double)),
        ("numberofholes", ctypes.c_int),
        ("regionlist", ctypes.POINTER(ctypes.c_double)),
        ("numberofregions", ctypes.c_int),
        ("edgelist", ctypes.POINTER(ctypes.c_int)),
        ("edgemarkerlist", ctypes.POINTER(ctypes.c_int)),
        ("normlist", ctypes.POINTER(ctypes.c_double)),
        ("numberofedges", ctypes.c_int),
    ]


_TRI = None


def triangle_library():
    global _TRI
    if _TRI is None:
        path = os.path.join(_HERE, "_ref", "libtriangle.so")
        if not os.path.exists(path):
            raise RuntimeError("oracle/_ref/libtriangle.so missing: `make -C oracle ref` "
                               "(needs /root/reference/cfemm/fmesher/triangle)")
        lib = ctypes.CDLL(path)
        lib.triangulate.restype = ctypes.c_int
        lib.triangulate.argtypes = [ctypes.c_char_p, ctypes.POINTER(_TriIO), ctypes.POINTER(_TriIO),
                                    ctypes.POINTER(_TriIO), ctypes.c_void_p]
        lib.trifree.argtypes = [ctypes.c_void_p]
        _TRI = lib
    return _TRI


@dataclass
class TriMesh:
    x: np.ndarray
    y: np.ndarray
    pmark: np.ndarray
    tri: np.ndarray        # (nt, 3)
    attr: np.ndarray       # (nt,) regional attribute
    edges: np.ndarray      # (ne, 2)
    emark: np.ndarray      # (ne,)


def _arr(ptr, n, dtype):
    if n == 0 or not ptr:
        return np.zeros(0, dtype=dtype)
    return np.ctypeslib.as_array(ptr, shape=(n,)).astype(dtype, copy=True)


def triangulate(switches: str, pts, pmark, segs, smark, holes, regions) -> TriMesh:
    """TriangulateHelper::triangulate (writepoly.cpp:2288-2322), XFEMM_BUILTIN_TRIANGLE path."""
    lib = triangle_library()
    keep = []

    def dbuf(a):
        a = np.ascontiguousarray(a, dtype=np.float64)
        keep.append(a)
        return a.ctypes.data_as(ctypes.POINTER(ctypes.c_double))

    def ibuf(a):
        a = np.ascontiguousarray(a, dtype=np.int32)
        keep.append(a)
        return a.ctypes.data_as(ctypes.POINTER(ctypes.c_int))

    inp = _TriIO()
    out = _TriIO()
    inp.numberofpoints = len(pmark)
    inp.pointlist = dbuf(np.asarray(pts, dtype=np.float64).reshape(-1))
    inp.pointmarkerlist = ibuf(pmark)
    inp.numberofsegments = len(smark)
    inp.segmentlist = ibuf(np.asarray(segs, dtype=np.int32).reshape(-1))
    inp.segmentmarkerlist = ibuf(smark)
    inp.numberofholes = len(holes)
    if holes:
        inp.holelist = dbuf(np.asarray(holes, dtype=np.float64).reshape(-1))
    inp.numberofregions = len(regions)
    inp.regionlist = dbuf(np.asarray(regions, dtype=np.float64).reshape(-1))
    libc = ctypes.CDLL(None)
    st = lib.triangulate(switches.encode(), ctypes.byref(inp), ctypes.byref(out), None,
                         ctypes.cast(libc.printf, ctypes.c_void_p))
    if st != 0:
        raise RuntimeError("triangulate failed with status %d" % st)
    npnt, nt, ne = out.numberofpoints, out.numberoftriangles, out.numberofedges
    pl = _arr(out.pointlist, 2 * npnt, np.float64)
    m = TriMesh(x=pl[0::2].copy(), y=pl[1::2].copy(),
                pmark=_arr(out.pointmarkerlist, npnt, np.int32),
                tri=_arr(out.trianglelist, 3 * nt, np.int32).reshape(nt, 3),
                attr=_arr(out.triangleattributelist, nt * out.numberoftriangleattributes, np.float64)
                .reshape(nt, -1)[:, 0] if out.numberoftriangleattributes else np.zeros(nt),
                edges=_arr(out.edgelist, 2 * ne, np.int32).reshape(ne, 2),
                emark=_arr(out.edgemarkerlist, ne, np.int32))
    for name in ("pointlist", "pointattributelist", "pointmarkerlist", "trianglelist",
                 "triangleattributelist", "neighborlist", "segmentlist", "segmentmarkerlist",
                 "edgelist", "edgemarkerlist", "normlist"):
        p = getattr(out, name)
        if p:
            lib.trifree(ctypes.cast(p, ctypes.c_void_p))
    return m


def _switches(min_angle: float, suppress_unused=False, suppress_exterior=False) -> str:
    # TriangulateHelper::triangulateParams (writepoly.cpp:2324-2350); std::to_string(double) = "%f"
    s = "-pPq" + ("%f" % min_angle) + "eAaz" + "Q" + "I"
    if suppress_unused:
        s += "j"
    if suppress_exterior:
        s += "Y"
    return s


def _point_markers(g: Geometry, nodelst: List[Node], from_problem: bool):
    # TriangulateHelper::initPointsWithMarkers (writepoly.cpp:2067-2122), magnetics
    out = np.zeros(len(nodelst), dtype=np.int32)
    if from_problem:
        for i, n in enumerate(nodelst):
            t = 0
            for j, name in enumerate(g.points):
                if name == n.marker:
                    t = j + 2
            out[i] = t
    return out


def _segment_markers(g: Geometry, linelst: List[Segment], from_problem: bool):
    # TriangulateHelper::initSegmentsWithMarkers (writepoly.cpp:2124-2187), magnetics
    out = np.zeros(len(linelst), dtype=np.int32)
    for i, s in enumerate(linelst):
        if from_problem:
            t = 0
            for j, b in enumerate(g.bdrys):
                if b.name == s.marker:
                    t = -(j + 2)
        else:
            t = -(s.cnt + 2)
        out[i] = t
    return out


def _holes_regions(g: Geometry, force_max: bool, default_size: float):
    # TriangulateHelper::initHolesAndRegions (writepoly.cpp:2189-2286)
    holes = [(lb.x, lb.y) for lb in g.labels if lb.BlockType == -1]
    regions = []
    k = 0
    for lb in g.labels:
        if lb.BlockType == -1:
            continue
        if lb.MaxArea <= 0:
            a = default_size
        elif lb.MaxArea > default_size and force_max:
            a = default_size
        else:
            a = lb.MaxArea
        regions.append((lb.x, lb.y, float(k + 1), a))
        k += 1
    return holes, regions


def _copy_seg(s: Segment, **kw) -> Segment:
    d = dict(n0=s.n0, n1=s.n1, MaxSideLength=s.MaxSideLength, marker=s.marker, cnt=s.cnt,
             IsSelected=s.IsSelected)
    d.update(kw)
    return Segment(**d)


def discretize_segments(g: Geometry, nodelst, linelst, dL, only_unselected=False):
    """fmesher::discretizeInputSegments (writepoly.cpp:263-399)."""
    for i, line in enumerate(g.lines):
        if only_unselected and line.IsSelected:
            continue
        a0 = g.nodes[line.n0].cc()
        a1 = g.nodes[line.n1].cc()
        segm = _copy_seg(line, cnt=i)
        L = g.length_of_line(line)
        num = 1 if line.MaxSideLength == -1 else int(math.ceil(L / line.MaxSideLength))
        if num == 1:
            if L < 3. * dL or not g.DoSmartMesh:
                linelst.append(_copy_seg(segm))
            else:
                # three parts, extra points dL from the ends (writepoly.cpp:327-365)
                a2 = a0 + c_divd(dL * (a1 - a0), c_abs(a1 - a0))
                l = len(nodelst)
                nodelst.append(Node(a2.real, a2.imag))
                linelst.append(_copy_seg(segm, n0=line.n0, n1=l))
                a2 = a1 + c_divd(dL * (a0 - a1), c_abs(a1 - a0))
                l = len(nodelst)
                nodelst.append(Node(a2.real, a2.imag))
                linelst.append(_copy_seg(segm, n0=l - 1, n1=l))
                l = len(nodelst) - 1
                linelst.append(_copy_seg(segm, n0=l, n1=line.n1))
        else:
            for j in range(num):
                a2 = a0 + c_divd((a1 - a0) * float(j + 1), float(num))
                if j == 0:
                    l = len(nodelst)
                    nodelst.append(Node(a2.real, a2.imag))
                    linelst.append(_copy_seg(segm, n0=line.n0, n1=l))
                elif j == num - 1:
                    l = len(nodelst) - 1
                    linelst.append(_copy_seg(segm, n0=l, n1=line.n1))
                else:
                    l = len(nodelst)
                    nodelst.append(Node(a2.real, a2.imag))
                    linelst.append(_copy_seg(segm, n0=l - 1, n1=l))


def discretize_arcs(g: Geometry, nodelst, linelst, only_unselected=False):
    """fmesher::discretizeInputArcSegments (writepoly.cpp:401-466)."""
    for i, arc in enumerate(g.arcs):
        if only_unselected and arc.IsSelected:
            continue
        segm = _copy_seg(arc, cnt=i + len(g.lines))
        num = int(math.ceil(arc.ArcLength / arc.MaxSideLength))
        c, R = g.get_circle(arc)
        a1 = c_expi(arc.ArcLength * PI / (float(num) * 180.))
        a2 = g.nodes[arc.n0].cc()
        if num == 1:
            linelst.append(_copy_seg(segm))
            continue
        for j in range(num):
            a2 = c_mul(a2 - c, a1) + c
            l = len(nodelst)
            if j == 0:
                nodelst.append(Node(a2.real, a2.imag))
                linelst.append(_copy_seg(segm, n0=arc.n0, n1=l))
            elif j == num - 1:
                linelst.append(_copy_seg(segm, n0=l - 1, n1=arc.n1))
            else:
                nodelst.append(Node(a2.real, a2.imag))
                linelst.append(_copy_seg(segm, n0=l - 1, n1=l))


def default_mesh_size(nodelst, smart: bool) -> float:
    """fmesher::defaultMeshSizeHeuristics (writepoly.cpp:238-261)."""
    mn = complex(nodelst[0].x, nodelst[0].y)
    mx = mn
    for n in nodelst:
        if n.x < mn.real:
            mn = complex(n.x, mn.imag)
        if n.y < mn.imag:
            mn = complex(mn.real, n.y)
        if n.x > mx.real:
            mx = complex(n.x, mx.imag)
        if n.y > mx.imag:
            mx = complex(mx.real, n.y)
    if smart:
        d = c_abs(mx - mn) / BOUNDING_BOX_FRACTION
        return d * d
    return c_abs(mx - mn)


def average_line_length(g: Geometry) -> float:      # writepoly.cpp:227-236
    z = 0.0
    n = float(len(g.lines))
    for s in g.lines:
        z += g.length_of_line(s) / n
    return z


@dataclass
class AirGap:
    name: str
    BdryFormat: int
    InnerAngle: float
    OuterAngle: float
    totalArcLength: float = 0.0
    totalArcElements: int = 0
    ri: float = 0.0
    ro: float = 0.0
    agc: complex = 0j
    nodeNums: List[int] = field(default_factory=list)


@dataclass
class MeshResult:
    mesh: TriMesh
    pbc: List[tuple]                    # (x, y, t) node pairs of the .pbc
    ages: List[AirGap]
    nodelst: List[Node]                 # the pre-triangulation node list (AGE ring positions)
    switches: str


def _is_periodic(g: Geometry) -> bool:              # FMesher::HasPeriodicBC (writepoly.cpp:477-540)
    if not any(b.BdryFormat in (4, 5, 6, 7) for b in g.bdrys):
        return False
    names = {b.name for b in g.bdrys if b.BdryFormat in (4, 5, 6, 7)}
    return any(s.marker in names for s in g.lines + g.arcs)


def mesh_problem(g: Geometry) -> MeshResult:
    """FMesher::DoPeriodicBCTriangulation (writepoly.cpp:823-2026) when the
    problem has periodic / air-gap boundaries, else DoNonPeriodicBCTriangulation."""
    if not _is_periodic(g):
        return _mesh_nonperiodic(g)
    dL = average_line_length(g) / LINE_FRACTION
    nodelst = [Node(n.x, n.y, n.marker) for n in g.nodes]
    for s in g.lines + g.arcs:
        s.cnt = 0
    linelst: List[Segment] = []
    discretize_segments(g, nodelst, linelst, dL)
    discretize_arcs(g, nodelst, linelst)
    default_size = default_mesh_size(nodelst, g.DoSmartMesh)

    # first call: segment markers carry the input entity index (writepoly.cpp:884-907)
    holes, regions = _holes_regions(g, True, default_size)
    m0 = triangulate(_switches(g.MinAngle), [(n.x, n.y) for n in nodelst],
                     _point_markers(g, nodelst, False), [(s.n0, s.n1) for s in linelst],
                     _segment_markers(g, linelst, False), holes, regions)

    # orient the input entities along the mesh (writepoly.cpp:953-1010)
    nl = len(g.lines)
    npt = nl + len(g.arcs)
    pt_t = [0] * npt
    pt_xy = [(0, 0)] * npt
    for s in g.lines + g.arcs:
        s.cnt = 0
    for (n0, n1), j in zip(m0.edges.tolist(), m0.emark.tolist()):
        if j == 0:
            continue
        j = -(j + 2)
        assert j >= 0
        if pt_t[j] == 0:
            pt_t[j] = 1
            pt_xy[j] = (min(n0, n1), max(n0, n1))
        if j < nl:
            s = g.lines[j]
            s.cnt += 1
            if s.n0 == n1 or s.n1 == n0:
                s.n0, s.n1 = s.n1, s.n0
        else:
            a = g.arcs[j - nl]
            a.cnt += 1
            if a.n0 == n1 or a.n1 == n0:
                a.NormalDirection = False
            if a.n0 == n0 or a.n1 == n1:
                a.NormalDirection = True
    # boundary entities appear in one element only (writepoly.cpp:1039-1058)
    ref = {}
    for j in range(npt):
        ref.setdefault(pt_xy[j], []).append(j)
    srt = np.sort(m0.tri, axis=1)
    for a, b, c in srt.tolist():
        for key in ((a, b), (a, c), (b, c)):
            for j in ref.get(key, ()):
                pt_t[j] -= 1
    for i, s in enumerate(g.lines):                                 # writepoly.cpp:1065-1075
        if pt_t[i] == 0:
            s.MaxSideLength = g.length_of_line(s) / float(s.cnt)
    for i, a in enumerate(g.arcs):                                  # writepoly.cpp:1077-1095
        if pt_t[i + nl] == 0:
            a.MaxSideLength = fmt_1e(a.ArcLength / float(a.cnt))

    # periodic boundaries and air gaps in play (writepoly.cpp:1110-1169)
    pbcs = []
    ages: List[AirGap] = []
    for b in g.bdrys:
        if b.BdryFormat in (4, 5):
            pbcs.append({"name": b.name, "anti": 1 if b.BdryFormat == 5 else 0,
                         "nseg": 0, "narc": 0, "seg": [0, 0]})
        if b.BdryFormat in (6, 7):
            if sum(1 for a in g.arcs if a.marker == b.name) > 1:
                ages.append(AirGap(b.name, b.BdryFormat - 6, b.InnerAngle, b.OuterAngle))
    for a in g.arcs:                                                # writepoly.cpp:1183-1208
        if a.marker == "<None>":
            continue
        for age in ages:
            if a.marker == age.name:
                age.totalArcLength += a.ArcLength
                age.totalArcElements += int(a.IsSelected)
                age.agc, R = g.get_circle(a)
                if age.ro == 0:
                    age.ri = R
                    age.ro = R
                if R > age.ro:
                    age.ro = R
                if R < age.ri:
                    age.ri = R
                break
    for age in ages:                                                # writepoly.cpp:1211-1233
        if age.totalArcLength > 0:
            my = age.totalArcLength / age.totalArcElements if age.totalArcElements else math.inf
            age.totalArcLength /= 2
            alt = (360. / PI) * (age.ro - age.ri) / (age.ro + age.ri)
            if alt < my:
                my = alt
            my = fmt_1e(my)
            for a in g.arcs:
                if a.marker == age.name:
                    a.MaxSideLength = my
    for s in g.lines:
        if s.marker != "<None>" and any(s.marker == age.name for age in ages):
            raise ValueError("Can't apply Air Gap Element BCs to line segments")
    for i, s in enumerate(g.lines):                                 # writepoly.cpp:1279-1300
        for p in pbcs:
            if p["name"] == s.marker:
                if p["nseg"] == 2:
                    raise ValueError("periodic BC %s on more than two segments" % p["name"])
                p["seg"][p["nseg"]] = i
                p["nseg"] += 1
    for i, a in enumerate(g.arcs):                                  # writepoly.cpp:1302-1323
        for p in pbcs:
            if p["name"] == a.marker:
                if p["narc"] == 2:
                    raise ValueError("periodic BC %s on more than two arcs" % p["name"])
                p["seg"][p["narc"]] = i
                p["narc"] += 1
    kept = []
    for p in pbcs:                                                  # writepoly.cpp:1325-1341
        if p["nseg"] > 0 and p["narc"] > 0:
            raise ValueError("Can't mix arcs and segments for (anti)periodic BCs")
        if p["nseg"] < 2 and p["narc"] < 2:
            continue
        kept.append(p)
    pbcs = kept
    for p in pbcs:                                                  # writepoly.cpp:1343-1397
        if p["nseg"] > 0:
            s0, s1 = g.lines[p["seg"][0]], g.lines[p["seg"][1]]
            if abs(g.length_of_line(s0) - g.length_of_line(s1)) > 1e-6:
                raise ValueError("(anti)periodic BCs applied to dissimilar segments")
            l1, l2 = s0.MaxSideLength, s1.MaxSideLength
            if l1 <= 0:
                l1 = l2
            if l2 <= 0:
                l2 = l1
            s0.MaxSideLength = s1.MaxSideLength = min(l1, l2)
        if p["narc"] > 0:
            a0, a1 = g.arcs[p["seg"][0]], g.arcs[p["seg"][1]]
            if abs(a0.ArcLength - a1.ArcLength) > 1e-6:
                raise ValueError("(anti)periodic BCs applied to dissimilar arc segments")
            a0.MaxSideLength = a1.MaxSideLength = min(a0.MaxSideLength, a1.MaxSideLength)

    # second pass: paired discretisation + .pbc node pairs (writepoly.cpp:1404-1648)
    for s in g.lines + g.arcs:
        s.cnt = 0
        s.IsSelected = False
    nodelst = [Node(n.x, n.y, n.marker) for n in g.nodes]
    linelst = []
    ptlst: List[list] = []
    segm_name = "<None>"          # the shared `segm` of writepoly.cpp:845
    for p in pbcs:
        anti = p["anti"]
        if p["nseg"] != 0:
            s0, s1 = g.lines[p["seg"][0]], g.lines[p["seg"][1]]
            s0.IsSelected = s1.IsSelected = True
            s1.n0, s1.n1 = s1.n1, s1.n0
            if s0.MaxSideLength == -1:
                k = 1
            else:
                a0 = g.nodes[s0.n0].cc()
                a1 = g.nodes[s0.n1].cc()
                b0 = g.nodes[s1.n0].cc()
                b1 = g.nodes[s1.n1].cc()
                k = int(math.ceil(c_abs(a1 - a0) / s0.MaxSideLength))
            ptlst.append([s0.n0, s1.n0, anti])
            ptlst.append([s0.n1, s1.n1, anti])
            if k == 1:
                linelst.append(_copy_seg(s0))
                linelst.append(_copy_seg(s1))
            else:
                segm = _copy_seg(s0)
                segm_name = s0.marker
                for j in range(k):
                    a2 = a0 + c_divd((a1 - a0) * float(j + 1), float(k))
                    b2 = b0 + c_divd((b1 - b0) * float(j + 1), float(k))
                    if j == 0:
                        l = len(nodelst)
                        nodelst.append(Node(a2.real, a2.imag))
                        linelst.append(_copy_seg(segm, n0=s0.n0, n1=l))
                        px = l
                        l = len(nodelst)
                        nodelst.append(Node(b2.real, b2.imag))
                        linelst.append(_copy_seg(segm, n0=s1.n0, n1=l))
                        ptlst.append([px, l, anti])
                    elif j == k - 1:
                        l = len(nodelst) - 2
                        linelst.append(_copy_seg(segm, n0=l, n1=s0.n1))
                        l = len(nodelst) - 1
                        linelst.append(_copy_seg(segm, n0=l, n1=s1.n1))
                    else:
                        l = len(nodelst)
                        nodelst.append(Node(a2.real, a2.imag))
                        nodelst.append(Node(b2.real, b2.imag))
                        linelst.append(_copy_seg(segm, n0=l - 2, n1=l))
                        linelst.append(_copy_seg(segm, n0=l - 1, n1=l + 1))
                        ptlst.append([l, l + 1, anti])
        else:
            s0, s1 = g.arcs[p["seg"][0]], g.arcs[p["seg"][1]]
            s0.IsSelected = s1.IsSelected = True
            k = int(math.ceil(s0.ArcLength / s0.MaxSideLength))
            segm_name = s0.marker
            c0, r0 = g.get_circle(s0)
            c1, r1 = g.get_circle(s1)
            if not s0.NormalDirection:
                bgn0 = g.nodes[s0.n0].cc()
                d0 = c_expi(s0.ArcLength * PI / (float(k) * 180.))
                p0 = (s0.n0, s0.n1)
            else:
                bgn0 = g.nodes[s0.n1].cc()
                d0 = c_expi(-(s0.ArcLength * PI) / (float(k) * 180.))
                p0 = (s0.n1, s0.n0)
            if s1.NormalDirection:
                bgn1 = g.nodes[s1.n0].cc()
                d1 = c_expi(s1.ArcLength * PI / (float(k) * 180.))
                p1 = (s1.n0, s1.n1)
            else:
                bgn1 = g.nodes[s1.n1].cc()
                d1 = c_expi(-(s1.ArcLength * PI) / (float(k) * 180.))
                p1 = (s1.n1, s1.n0)
            ptlst.append([p0[0], p1[0], anti])
            ptlst.append([p0[1], p1[1], anti])
            segm = Segment(0, 0, marker=segm_name)
            if k == 1:
                linelst.append(_copy_seg(segm, n0=p0[0], n1=p0[1]))
                linelst.append(_copy_seg(segm, n0=p1[0], n1=p1[1]))
            else:
                for j in range(k):
                    bgn0 = c_mul(bgn0 - c0, d0) + c0
                    bgn1 = c_mul(bgn1 - c1, d1) + c1
                    if j == 0:
                        l = len(nodelst)
                        nodelst.append(Node(bgn0.real, bgn0.imag))
                        linelst.append(_copy_seg(segm, n0=p0[0], n1=l))
                        px = l
                        l = len(nodelst)
                        nodelst.append(Node(bgn1.real, bgn1.imag))
                        linelst.append(_copy_seg(segm, n0=p1[0], n1=l))
                        ptlst.append([px, l, anti])
                    elif j == k - 1:
                        l = len(nodelst) - 2
                        linelst.append(_copy_seg(segm, n0=l, n1=p0[1]))
                        l = len(nodelst) - 1
                        linelst.append(_copy_seg(segm, n0=l, n1=p1[1]))
                    else:
                        l = len(nodelst)
                        nodelst.append(Node(bgn0.real, bgn0.imag))
                        nodelst.append(Node(bgn1.real, bgn1.imag))
                        linelst.append(_copy_seg(segm, n0=l - 2, n1=l))
                        linelst.append(_copy_seg(segm, n0=l - 1, n1=l + 1))
                        ptlst.append([l, l + 1, anti])

    # air-gap rings (writepoly.cpp:1652-1723); segments keep segm_name (quirk, see header)
    for age in ages:
        vec: List[int] = []
        z = (age.ro + age.ri) / 2.
        for a in g.arcs:
            if a.IsSelected or a.marker != age.name:
                continue
            a.IsSelected = True
            a2 = g.nodes[a.n0].cc()
            k = int(math.ceil(a.ArcLength / a.MaxSideLength))
            c, R = g.get_circle(a)
            a1 = c_expi(a.ArcLength * PI / (float(k) * 180.))
            if R > z:
                vec.append(a.n0)
            else:
                vec.insert(0, a.n0)
            segm = Segment(0, 0, marker=segm_name)
            if k == 1:
                linelst.append(_copy_seg(segm, n0=a.n0, n1=a.n1))
                continue
            for j in range(k):
                a2 = c_mul(a2 - c, a1) + c
                if j == 0:
                    l = len(nodelst)
                    nodelst.append(Node(a2.real, a2.imag))
                    linelst.append(_copy_seg(segm, n0=a.n0, n1=l))
                    if R > z:
                        vec.append(l)
                    else:
                        vec.insert(0, l)
                elif j == k - 1:
                    l = len(nodelst) - 1
                    linelst.append(_copy_seg(segm, n0=l, n1=a.n1))
                else:
                    l = len(nodelst)
                    nodelst.append(Node(a2.real, a2.imag))
                    linelst.append(_copy_seg(segm, n0=l - 1, n1=l))
                    if R > z:
                        vec.append(l)
                    else:
                        vec.insert(0, l)
        age.nodeNums = [len(vec)] + vec

    # the rest in the normal way (writepoly.cpp:1730-1733)
    discretize_segments(g, nodelst, linelst, dL, only_unselected=True)
    discretize_arcs(g, nodelst, linelst, only_unselected=True)

    # prune duplicated pairs (writepoly.cpp:1789-1801)
    for p in ptlst:
        if p[0] > p[1]:
            p[0], p[1] = p[1], p[0]
    k = 0
    while k + 1 < len(ptlst):
        j = k + 1
        while j < len(ptlst):
            if ptlst[k][0] == ptlst[j][0] and ptlst[k][1] == ptlst[j][1]:
                del ptlst[j]
            else:
                j += 1
        k += 1

    # final call with -Y (writepoly.cpp:1986-2010)
    sw = _switches(min(g.MinAngle + MINANGLE_BUMP, MINANGLE_MAX), suppress_exterior=True)
    holes, regions = _holes_regions(g, True, default_size)
    m1 = triangulate(sw, [(n.x, n.y) for n in nodelst], _point_markers(g, nodelst, True),
                     [(s.n0, s.n1) for s in linelst], _segment_markers(g, linelst, True), holes, regions)
    return MeshResult(m1, [tuple(p) for p in ptlst], ages, nodelst, sw)


def _mesh_nonperiodic(g: Geometry) -> MeshResult:
    """FMesher::DoNonPeriodicBCTriangulation (writepoly.cpp:711-811)."""
    dL = average_line_length(g) / LINE_FRACTION
    nodelst = [Node(n.x, n.y, n.marker) for n in g.nodes]
    linelst: List[Segment] = []
    discretize_segments(g, nodelst, linelst, dL)
    discretize_arcs(g, nodelst, linelst)
    default_size = default_mesh_size(nodelst, g.DoSmartMesh)
    holes, regions = _holes_regions(g, False, default_size)    # DoForceMaxMeshArea: off
    sw = _switches(min(g.MinAngle + MINANGLE_BUMP, MINANGLE_MAX), suppress_unused=True)
    m = triangulate(sw, [(n.x, n.y) for n in nodelst], _point_markers(g, nodelst, True),
                    [(s.n0, s.n1) for s in linelst], _segment_markers(g, linelst, True), holes, regions)
    return MeshResult(m, [], [], nodelst, sw)


def age_section(res: MeshResult, age: AirGap, inner_angle: Optional[float] = None,
                outer_angle: Optional[float] = None) -> str:
    """One AGE block of the .pbc file (writepoly.cpp:1853-1980) at the given
    rotor angles (the mesh itself does not depend on them)."""
    ia = age.InnerAngle if inner_angle is None else inner_angle
    oa = age.OuterAngle if outer_angle is None else outer_angle
    n = age.nodeNums[0] // 2
    dtta = age.totalArcLength / n
    n0 = c_round(360. / dtta)
    n1 = c_round(360. / age.totalArcLength)
    inner, outer = [], []
    for j in range(n1):
        dl = -1.0 if (age.BdryFormat == 1 and j % 2 != 0) else 1.0
        a1 = c_expi((j * age.totalArcLength + ia) * DEGREE)
        a2 = c_expi((j * age.totalArcLength + oa) * DEGREE)
        for i in range(1, n + 1):
            ni = age.nodeNums[i]
            a0 = c_mul(a1, res.nodelst[ni].cc() - age.agc)
            inner.append([ni, to_degrees(a0) / dtta, dl])
            no = age.nodeNums[i + n]
            a0 = c_mul(a2, res.nodelst[no].cc() - age.agc)
            outer.append([no, to_degrees(a0) / dtta, dl])
    for ring in (inner, outer):                    # bubble sort by w0 (writepoly.cpp:1908-1942)
        for _ in range(n0):
            done = True
            for jj in range(n0 - 1):
                if ring[jj][1] > ring[jj + 1][1]:
                    ring[jj], ring[jj + 1] = ring[jj + 1], ring[jj]
                    done = False
            if done:
                break
    out = ['"%s"\n' % age.name,
           "%i %.17g %.17g %.17g %.17g %.17g %.17g %.17g %i %.17g %.17g\n" % (
               age.BdryFormat, ia, oa, age.ri, age.ro, age.totalArcLength,
               age.agc.real, age.agc.imag, n, inner[0][1], outer[0][1])]
    for i in range(n + 1):
        p1 = 0 if i == n0 else i
        p0 = p1 - 1
        if p0 < 0:
            p0 = n0 + p0
        out.append("%i %g %i %g %i %g %i %g\n" % (inner[p0][0], inner[p0][2], inner[p1][0], inner[p1][2],
                                                  outer[p0][0], outer[p0][2], outer[p1][0], outer[p1][2]))
    return "".join(out)


def pbc_text(res: MeshResult, angles: Optional[dict] = None) -> str:
    """The .pbc file (writepoly.cpp:1838-1852): node pairs then the AGE blocks.
    ``angles`` maps an AGE name to (inner_angle, outer_angle)."""
    out = ["%i\n" % len(res.pbc)]
    for k, (x, y, t) in enumerate(res.pbc):
        out.append("%i    %i    %i    %i\n" % (k, x, y, t))
    out.append("%i\n" % len(res.ages))
    for age in res.ages:
        ia, oa = (angles or {}).get(age.name, (None, None))
        out.append(age_section(res, age, ia, oa))
    return "".join(out)


def write_mesh(res: MeshResult, base: str, angles: Optional[dict] = None) -> None:
    """TriangulateHelper::writeTriangulationFiles (writepoly.cpp:543-698) + the .pbc."""
    m = res.mesh
    with open(base + ".node", "w") as fh:
        fh.write("%i\t%i\t%i\t%i\n" % (len(m.x), 2, 0, 1))
        fh.writelines("%i\t%.17g\t%.17g\t%i\n" % (i, m.x[i], m.y[i], m.pmark[i]) for i in range(len(m.x)))
    with open(base + ".edge", "w") as fh:
        fh.write("%i\t%i\n" % (len(m.edges), 1))
        fh.writelines("%i\t%i\t%i\t%i\n" % (i, m.edges[i, 0], m.edges[i, 1], m.emark[i])
                      for i in range(len(m.edges)))
    with open(base + ".ele", "w") as fh:
        fh.write("%i\t%i\t%i\n" % (len(m.tri), 3, 1))
        fh.writelines("%i\t%i\t%i\t%i\t%.17g\t\n" % (i, m.tri[i, 0], m.tri[i, 1], m.tri[i, 2], m.attr[i])
                      for i in range(len(m.tri)))
    with open(base + ".pbc", "w") as fh:
        fh.write(pbc_text(res, angles) if (res.pbc or res.ages) else "0\n0\n")


def refine_fem_text(text: str, factor: float) -> str:
    """A finer variant of a .fem, as a user would ask fmesher for one: block
    label mesh sizes and the side lengths of non-air-gap arcs divided by
    ``factor``, smart meshing off (so the bounding-box default does not cap
    the label sizes).  Used for BASELINE configs[1] (TorqueBenchmark refined)."""
    g = parse_geometry_text(text)
    age_names = {b.name for b in g.bdrys if b.BdryFormat in (6, 7)}
    nl = "\r\n" if "\r\n" in text else "\n"
    out, mode, k = [], None, 0
    for ln in text.split(nl):
        s = ln.strip()
        low = s.lower()
        if low.startswith("[dosmartmesh]"):
            out.append("[DoSmartMesh] =  0")
            continue
        if low.startswith("[numarcsegments]"):
            mode, k = "arc", 0
            out.append(ln)
            continue
        if low.startswith("[numblocklabels]"):
            mode = "lbl"
            out.append(ln)
            continue
        if low.startswith("[") or not s:
            mode = None if not low.startswith("[num") or low.startswith("[numholes]") else mode
        if mode == "arc" and s and not low.startswith("["):
            f = s.split()
            if g.arcs[k].marker not in age_names:
                f[3] = repr(float(f[3]) / factor)
            k += 1
            ln = "\t".join(f)
        elif mode == "lbl" and s and not low.startswith("["):
            f = s.split()
            if float(f[3]) > 0:
                f[3] = repr(float(f[3]) / factor)
            ln = "\t".join(f)
        out.append(ln)
    return nl.join(out)


def parse_geometry_text(text: str) -> Geometry:
    import tempfile
    with tempfile.NamedTemporaryFile("w", suffix=".fem", delete=False) as fh:
        fh.write(text)
        path = fh.name
    try:
        return parse_geometry(path)
    finally:
        os.unlink(path)
