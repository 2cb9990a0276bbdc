"""CPU oracle front-end: .fem parsing, circuit expansion, B-H slopes, mesh loading.

TEST INFRASTRUCTURE ONLY.  This module is the checker, never the thing measured
or shipped: only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s
``cpu_baseline`` leg may import it.  The product path (``xfemm_amd``) has its
own C++ host code and fails loudly when the HIP library is missing.

It restates, in plain Python/numpy, the reference behaviour of:
  * FEASolver::LoadProblemFile        cfemm/libfemm/feasolver.cpp:223-520
  * CMSolverMaterialProp::fromStream  cfemm/libfemm/CMaterialProp.cpp:1173-1328
  * CMBoundaryProp / CMPointProp / CMCircuit / CMBlockLabel ::fromStream
                                      cfemm/libfemm/CBoundaryProp.cpp:98-200,
                                      CPointProp.cpp, CCircuit.cpp:67-130,
                                      CBlockLabel.cpp:110-154
  * FSolver::LoadProblemFile          cfemm/fsolver/fsolver.cpp:202-348
  * CMMaterialProp::GetSlopes(0)      cfemm/libfemm/CMaterialProp.cpp:127-348
  * CComplexFullMatrix::GaussSolve    cfemm/libfemm/fullmatrix.cpp:183-218
  * FSolver::LoadMesh                 cfemm/fsolver/fsolver.cpp:350-718
  * FEASolver::Cuthill / SortElements cfemm/libfemm/cuthill.cpp
  * FSolver::GetFillFactor (static)   cfemm/fsolver/fsolver.cpp:1083-1105

Complex arithmetic of the reference (femmcomplex.cpp) is restated on the real
axis with the same rounding: ``a / z`` for a complex ``z`` is ``a * (1/z)``
(femmcomplex.cpp:362-381), ``abs`` of a real-valued complex is ``fabs``.
"""
from __future__ import annotations

import math
import os
from dataclasses import dataclass, field
from typing import List, Optional

import dataclasses

import numpy as np

MUO = 1.2566370614359173e-6          # femmconstants.h
PI = 3.141592653589793238462643383
DEG = 0.01745329251994329576923690768
LENGTH_CONV_METERS = [0.0254, 0.001, 0.01, 1.0, 2.54e-05, 1.0e-06]  # femmenums.h:51
LENGTH_UNITS = {"inches": 0, "millimeters": 1, "centimeters": 2, "meters": 3,
                "mils": 4, "microns": 5}


@dataclass
class PointProp:                 # CPointProp.h (CMPointProp)
    name: str = ""
    A_re: float = 0.0
    A_im: float = 0.0
    J_re: float = 0.0
    J_im: float = 0.0


@dataclass
class BdryProp:                  # CBoundaryProp.cpp:51-75
    name: str = "New Boundary"
    BdryFormat: int = 0
    A0: float = 0.0
    A1: float = 0.0
    A2: float = 0.0
    phi: float = 0.0
    c0: float = 0.0
    c0i: float = 0.0
    c1: float = 0.0
    c1i: float = 0.0
    Mu: float = 0.0
    Sig: float = 0.0
    InnerAngle: float = 0.0
    OuterAngle: float = 0.0


@dataclass
class BlockProp:                 # CMaterialProp.cpp:65-89
    name: str = "New Material"
    mu_x: float = 1.0
    mu_y: float = 1.0
    H_c: float = 0.0
    Theta_m: float = 0.0
    J_re: float = 0.0
    J_im: float = 0.0
    Cduct: float = 0.0
    Lam_d: float = 0.0
    Theta_hn: float = 0.0
    Theta_hx: float = 0.0
    Theta_hy: float = 0.0
    LamType: int = 0
    LamFill: float = 1.0
    NStrands: int = 0
    WireD: float = 0.0
    BHpoints: int = 0
    Bdata: List[float] = field(default_factory=list)
    Hdata: List[float] = field(default_factory=list)   # real parts (static problems)
    slope: List[float] = field(default_factory=list)
    MuMax: float = 0.0


@dataclass
class Circuit:                   # CCircuit.cpp:50-65
    name: str = "New Circuit"
    CircType: int = 0
    Amps_re: float = 0.0
    Amps_im: float = 0.0
    dVolts_re: float = 0.0
    dVolts_im: float = 0.0
    OrigCirc: int = 0
    Case: int = 0
    J: float = 0.0
    dV: float = 0.0


@dataclass
class BlockLabel:                # CBlockLabel.cpp:42-109
    x: float = 0.0
    y: float = 0.0
    BlockType: int = -1
    MaxArea: float = 0.0
    InCircuit: int = -1
    MagDir: float = 0.0
    InGroup: int = 0
    Turns: int = 1
    IsDefault: bool = False
    IsExternal: bool = False
    MagDirFctn: str = ""
    bIsWound: bool = False
    ProximityMu: complex = 1.0


@dataclass
class FemProblem:
    FileFormat: float = -1.0
    Frequency: float = 0.0
    Precision: float = 1.0e-8
    MinAngle: float = 0.0
    Depth: float = -1.0
    LengthUnits: int = 0
    Coords: int = 0            # 0 cartesian, 1 polar
    ProblemType: int = 0       # 0 planar, 1 axisymmetric
    ACSolver: int = 0
    PrevType: int = 0
    PrevSoln: str = ""
    Comment: str = ""
    points: List[PointProp] = field(default_factory=list)
    bdrys: List[BdryProp] = field(default_factory=list)
    blocks: List[BlockProp] = field(default_factory=list)
    circuits: List[Circuit] = field(default_factory=list)
    labels: List[BlockLabel] = field(default_factory=list)
    NumCircPropsOrig: int = 0
    Relax: float = 1.0
    extZo: float = 0.0          # axisymmetric exterior region (feasolver.cpp:306-326)
    extRo: float = 0.0
    extRi: float = 0.0


# --------------------------------------------------------------------------
# tokenizer helpers mirroring fparse.cpp (nextToken / expectChar / parseValue)
# --------------------------------------------------------------------------

def _rest_after_eq(line: str) -> str:
    s = line.split("=", 1)
    if len(s) != 2:
        raise ValueError("expected '=' in line: %r" % line)
    return s[1].strip()


def _parse_string(rest: str) -> str:
    # fparse.cpp parseString: opening '"', terminated by the LAST '"' of the line
    rest = rest.strip()
    if not rest.startswith('"'):
        raise ValueError("invalid begin of string literal: %r" % rest)
    body = rest[1:]
    pos = body.rfind('"')
    if pos < 0:
        raise ValueError("unterminated string literal: %r" % rest)
    return body[:pos]


def _stod(s: str) -> float:
    # std::stod accepts a leading numeric prefix; the reference warns on trailing chars
    s = s.strip()
    i = len(s)
    while i > 0:
        try:
            return float(s[:i])
        except ValueError:
            i -= 1
    raise ValueError("could not convert %r to double" % s)


def _stoi(s: str) -> int:
    s = s.strip()
    i = len(s)
    while i > 0:
        try:
            return int(s[:i])
        except ValueError:
            i -= 1
    raise ValueError("could not convert %r to int" % s)


class _Lines:
    def __init__(self, text: str):
        self.lines = text.splitlines()
        self.i = 0

    def good(self) -> bool:
        return self.i < len(self.lines)

    def next(self) -> str:
        ln = self.lines[self.i]
        self.i += 1
        return ln


def _read_block(lines: _Lines, begin: str, end: str):
    """Yield (token, rest-of-line) pairs of one <Begin...> ... <End...> block."""
    # expectToken(input, "<beginxxx>")
    while lines.good():
        ln = lines.next().strip()
        if not ln:
            continue
        if ln.split()[0].lower() != begin:
            raise ValueError("expected %s, got %r" % (begin, ln))
        break
    while lines.good():
        ln = lines.next().strip()
        if not ln:
            continue
        tok = ln.split()[0].lower()
        if tok == end:
            return
        yield tok, ln, lines


def _parse_point(lines):  # CPointProp.cpp CMPointProp::fromStream
    p = PointProp()
    for tok, ln, _ in _read_block(lines, "<beginpoint>", "<endpoint>"):
        r = _rest_after_eq(ln)
        if tok == "<pointname>":
            p.name = _parse_string(r)
        elif tok == "<a_re>":
            p.A_re = _stod(r)
        elif tok == "<a_im>":
            p.A_im = _stod(r)
        elif tok == "<i_re>":
            p.J_re = _stod(r)
        elif tok == "<i_im>":
            p.J_im = _stod(r)
    return p


def _parse_bdry(lines):  # CBoundaryProp.cpp:98-200
    b = BdryProp()
    for tok, ln, _ in _read_block(lines, "<beginbdry>", "<endbdry>"):
        r = _rest_after_eq(ln)
        if tok == "<bdryname>":
            b.name = _parse_string(r)
        elif tok == "<bdrytype>":
            b.BdryFormat = _stoi(r)
        elif tok == "<mu_ssd>":
            b.Mu = _stod(r)
        elif tok == "<sigma_ssd>":
            b.Sig = _stod(r)
        elif tok == "<a_0>":
            b.A0 = _stod(r)
        elif tok == "<a_1>":
            b.A1 = _stod(r)
        elif tok == "<a_2>":
            b.A2 = _stod(r)
        elif tok == "<phi>":
            b.phi = _stod(r)
        elif tok == "<c0>":
            b.c0 = _stod(r)
        elif tok == "<c1>":
            b.c1 = _stod(r)
        elif tok == "<c0i>":
            b.c0i = _stod(r)
        elif tok == "<c1i>":
            b.c1i = _stod(r)
        elif tok == "<innerangle>":
            b.InnerAngle = _stod(r)
        elif tok == "<outerangle>":
            b.OuterAngle = _stod(r)
    return b


def _parse_block(lines):  # CMaterialProp.cpp:1173-1328
    m = BlockProp()
    for tok, ln, ls in _read_block(lines, "<beginblock>", "<endblock>"):
        r = _rest_after_eq(ln)
        if tok == "<blockname>":
            m.name = _parse_string(r)
        elif tok == "<mu_x>":
            m.mu_x = _stod(r)
        elif tok == "<mu_y>":
            m.mu_y = _stod(r)
        elif tok == "<h_c>":
            m.H_c = _stod(r)
        elif tok == "<h_cangle>":
            m.Theta_m = _stod(r)
        elif tok == "<j_re>":
            m.J_re = _stod(r)
        elif tok == "<j_im>":
            m.J_im = _stod(r)
        elif tok == "<sigma>":
            m.Cduct = _stod(r)
        elif tok == "<phi_h>":
            m.Theta_hn = _stod(r)
        elif tok == "<phi_hx>":
            m.Theta_hx = _stod(r)
        elif tok == "<phi_hy>":
            m.Theta_hy = _stod(r)
        elif tok == "<d_lam>":
            m.Lam_d = _stod(r)
        elif tok == "<lamfill>":
            m.LamFill = _stod(r)
        elif tok == "<wired>":
            m.WireD = _stod(r)
        elif tok == "<lamtype>":
            m.LamType = _stoi(r)
        elif tok == "<nstrands>":
            m.NStrands = _stoi(r)
        elif tok == "<bhpoints>":
            m.BHpoints = _stoi(r)
            vals: List[float] = []
            while len(vals) < 2 * m.BHpoints:
                vals.extend(float(v) for v in ls.next().split())
            m.Bdata = vals[0::2]
            m.Hdata = vals[1::2]
    return m


def _parse_circuit(lines):  # CCircuit.cpp:67-130
    c = Circuit()
    for tok, ln, _ in _read_block(lines, "<begincircuit>", "<endcircuit>"):
        r = _rest_after_eq(ln)
        if tok == "<circuitname>":
            c.name = _parse_string(r)
        elif tok == "<voltgradient_re>":
            c.dVolts_re = _stod(r)
        elif tok == "<voltgradient_im>":
            c.dVolts_im = _stod(r)
        elif tok == "<totalamps_re>":
            c.Amps_re = _stod(r)
        elif tok == "<totalamps_im>":
            c.Amps_im = _stod(r)
        elif tok == "<circuittype>":
            c.CircType = _stoi(r)
    return c


def _parse_label(line: str) -> BlockLabel:  # CBlockLabel.cpp:110-154
    lb = BlockLabel()
    # the optional trailing MagDirFctn is a quoted string
    q = line.find('"')
    head = line if q < 0 else line[:q]
    tail = "" if q < 0 else line[q:]
    f = head.split()
    conv = [float, float, int, float, int, float, int, int, int]
    vals = []
    for i, c in enumerate(conv):
        if i < len(f):
            vals.append(c(float(f[i])) if c is int else c(f[i]))
        else:
            vals.append(None)
    if vals[0] is not None:
        lb.x = vals[0]
    if vals[1] is not None:
        lb.y = vals[1]
    if vals[2] is not None:
        lb.BlockType = vals[2] - 1
    if vals[3] is not None:
        ma = vals[3]
        lb.MaxArea = 0.0 if ma <= 0 else ma * (PI * ma / 4.0)
    if vals[4] is not None:
        lb.InCircuit = vals[4] - 1
    if vals[5] is not None:
        lb.MagDir = vals[5]
    if vals[6] is not None:
        lb.InGroup = vals[6]
    if vals[7] is not None:
        lb.Turns = vals[7]
    ext = vals[8] or 0
    lb.IsDefault = bool(ext & 2)
    lb.IsExternal = bool(ext & 1)
    if tail:
        lb.MagDirFctn = _parse_string(tail)
    return lb


def parse_fem(path: str) -> FemProblem:
    """FEASolver::LoadProblemFile (feasolver.cpp:223-520) + FSolver::handleToken."""
    with open(path, "r") as fh:
        lines = _Lines(fh.read())
    pr = FemProblem()
    while lines.good():
        ln = lines.next().strip()
        if not ln:
            continue
        tok = ln.split()[0].lower()
        if tok in ("[numpoints]", "[numsegments]", "[numarcsegments]", "[numholes]"):
            n = _stoi(_rest_after_eq(ln))
            for _ in range(n):
                lines.next()
            continue
        r = _rest_after_eq(ln)
        if tok == "[format]":
            pr.FileFormat = _stod(r)
        elif tok == "[frequency]":
            pr.Frequency = _stod(r)
        elif tok == "[precision]":
            pr.Precision = _stod(r)
        elif tok == "[minangle]":
            pr.MinAngle = _stod(r)
        elif tok == "[depth]":
            pr.Depth = _stod(r)
        elif tok == "[lengthunits]":
            u = r.split()[0].lower() if r.split() else ""
            if u in LENGTH_UNITS:
                pr.LengthUnits = LENGTH_UNITS[u]
        elif tok == "[coordinates]":
            u = r.split()[0].lower()
            if u == "cartesian":
                pr.Coords = 0
            if u == "polar":
                pr.Coords = 1
        elif tok == "[problemtype]":
            u = r.split()[0].lower()
            if u == "planar":
                pr.ProblemType = 0
            if u == "axisymmetric":
                pr.ProblemType = 1
        elif tok == "[extzo]":
            pr.extZo = _stod(r)
        elif tok == "[extro]":
            pr.extRo = _stod(r)
        elif tok == "[extri]":
            pr.extRi = _stod(r)
        elif tok in ("[forcemaxmesh]", "[dosmartmesh]"):
            pass
        elif tok == "[comment]":
            pr.Comment = _parse_string(r)
        elif tok == "[acsolver]":
            pr.ACSolver = _stoi(r)
        elif tok == "[prevtype]":
            pr.PrevType = _stoi(r)
        elif tok == "[prevsoln]":
            pr.PrevSoln = _parse_string(r)
        elif tok == "[pointprops]":
            for _ in range(_stoi(r)):
                pr.points.append(_parse_point(lines))
        elif tok == "[bdryprops]":
            for _ in range(_stoi(r)):
                pr.bdrys.append(_parse_bdry(lines))
        elif tok == "[blockprops]":
            for _ in range(_stoi(r)):
                pr.blocks.append(_parse_block(lines))
        elif tok in ("[circuitprops]", "[conductorprops]"):
            for _ in range(_stoi(r)):
                pr.circuits.append(_parse_circuit(lines))
        elif tok == "[numblocklabels]":
            for _ in range(_stoi(r)):
                pr.labels.append(_parse_label(lines.next().strip()))
        else:
            raise ValueError("Unknown token: %s" % tok)
    return pr


# --------------------------------------------------------------------------
# B-H curve preprocessing: CMMaterialProp::GetSlopes(omega=0)
# --------------------------------------------------------------------------

def _recip(z: float) -> float:
    # femmcomplex.cpp:367-372 on the real axis: y.re = 1./(z.re*(1.+c*c)), c = 0
    return 1.0 / (z * (1.0 + 0.0 * 0.0))


def _gauss_solve(M: List[List[float]], b: List[float]) -> List[float]:
    """CComplexFullMatrix::GaussSolve (fullmatrix.cpp:183-218), real axis."""
    n = len(b)
    M = [row[:] for row in M]
    b = b[:]
    q = 0
    for i in range(n):
        mx = 0.0
        for j in range(i, n):
            if abs(M[j][i]) > abs(mx):
                mx = M[j][i]
                q = j
        if mx == 0:
            raise ZeroDivisionError("singular B-H slope system")
        M[i], M[q] = M[q], M[i]
        b[i], b[q] = b[q], b[i]
        for j in range(i + 1, n):
            f = M[j][i] * _recip(M[i][i])
            b[j] = b[j] - f * b[i]
            for k in range(i, n):
                M[j][k] -= f * M[i][k]
    for i in range(n - 1, -1, -1):
        f = 0.0
        for j in range(n - 1, i, -1):
            f += M[i][j] * b[j]
        b[i] = (b[i] - f) * _recip(M[i][i])
    return b


def get_slopes(m: BlockProp) -> None:
    """CMMaterialProp::GetSlopes(0) (CMaterialProp.cpp:127-348), static case."""
    if m.BHpoints == 0 or m.slope:
        return
    n = m.BHpoints
    B = list(m.Bdata)
    H = list(m.Hdata)
    m.mu_x = B[1] / (MUO * abs(H[1]))
    m.mu_y = m.mu_x
    m.Theta_hx = m.Theta_hn
    m.Theta_hy = m.Theta_hn
    curve_ok = False
    processed_lams = False
    bn = [0.0] * n
    hn = [0.0] * n
    slope: List[float] = []
    while not curve_ok:
        M = [[0.0] * n for _ in range(n)]
        rhs = [0.0] * n
        l1 = B[1] - B[0]
        M[0][0] = 4.0 / l1
        M[0][1] = 2.0 / l1
        rhs[0] = 6.0 * (H[1] - H[0]) / (l1 * l1)
        l1 = B[n - 1] - B[n - 2]
        M[n - 1][n - 1] = 4.0 / l1
        M[n - 1][n - 2] = 2.0 / l1
        rhs[n - 1] = 6.0 * (H[n - 1] - H[n - 2]) / (l1 * l1)
        for i in range(1, n - 1):
            l1 = B[i] - B[i - 1]
            l2 = B[i + 1] - B[i]
            M[i][i - 1] = 2.0 / l1
            M[i][i] = 4.0 * (l1 + l2) / (l1 * l2)
            M[i][i + 1] = 2.0 / l2
            rhs[i] = 6.0 * (H[i] - H[i - 1]) / (l1 * l1) + 6.0 * (H[i + 1] - H[i]) / (l2 * l2)
        slope = _gauss_solve(M, rhs)
        curve_ok = True
        for i in range(1, n):
            d0 = slope[i - 1]
            d1 = slope[i]
            u0 = H[i - 1]
            u1 = H[i]
            L = B[i] - B[i - 1]
            c0 = d0
            c1 = -(2.0 * (2.0 * d0 * L + d1 * L + 3.0 * u0 - 3.0 * u1)) / (L * L)
            c2 = (3.0 * (d0 * L + d1 * L + 2.0 * u0 - 2.0 * u1)) / (L * L * L)
            X0 = -1.0
            X1 = -1.0
            u0 = c1 * c1 - 4.0 * c0 * c2
            if c2 == 0:
                if c1 != 0:
                    X0 = -c0 / c1
            elif u0 > 0:
                u0 = math.sqrt(u0)
                X0 = -(c1 + u0) / (2.0 * c2)
                X1 = (-c1 + u0) / (2.0 * c2)
            if (0.0 <= X0 <= L) or (0.0 <= X1 <= L):
                curve_ok = False
        if not curve_ok:
            for i in range(1, n - 1):
                bn[i] = (B[i - 1] + B[i] + B[i + 1]) / 3.0
                hn[i] = (H[i - 1] + H[i] + H[i + 1]) / 3.0
            for i in range(1, n - 1):
                H[i] = hn[i]
                B[i] = bn[i]
        if curve_ok and not processed_lams:
            # omega == 0: the lamination eddy-current branch never runs
            if m.LamType == 0 and m.LamFill != 1:
                for i in range(1, n):
                    # mu = LamFill*B/H + (1-LamFill)*muo  (double / CComplex)
                    mu = (_recip(H[i]) * (m.LamFill * B[i])) + (1.0 - m.LamFill) * MUO
                    B[i] = abs(mu * H[i])
                    H[i] = B[i] * _recip(mu)
                curve_ok = False
            processed_lams = True
    m.Bdata = B
    m.Hdata = H
    m.slope = slope


# --------------------------------------------------------------------------
# FSolver::LoadProblemFile post-processing (fsolver.cpp:202-348)
# --------------------------------------------------------------------------

class PrevSolnError(ValueError):
    """A previous-solution problem the reference refuses, or on which its
    behaviour is undefined (message says which)."""


def prepare_problem(pr: FemProblem) -> FemProblem:
    pr.Relax = 1.0
    if pr.PrevSoln:
        # fsolver.cpp:224-238: with a previous solution LoadProblemFile returns
        # right after loadPreviousSolution, before the B-H precomputation
        # (GetSlopes) and the serial-circuit expansion.  A B-H block then has
        # no slopes (Get_v / GetdHdB index empty vectors) and a serial circuit
        # keeps CircType 1: undefined in the reference, refused here.
        if any(m.BHpoints > 0 for m in pr.blocks):
            raise PrevSolnError("B-H curves with a previous solution: the reference never computes their "
                                "slopes (fsolver.cpp:224-238)")
        if any(c.CircType == 1 for c in pr.circuits):
            raise PrevSolnError("serial circuits with a previous solution: the reference skips their "
                                "expansion (fsolver.cpp:224-238)")
        return pr
    for m in pr.blocks:
        if m.BHpoints > 0:
            get_slopes(m)
            m.MuMax = 0.0
    if not pr.circuits:
        return pr
    ncirc = len(pr.circuits)
    for c in pr.circuits:
        c.OrigCirc = -1
    pr.NumCircPropsOrig = ncirc
    for k, lb in enumerate(pr.labels):
        if lb.InCircuit >= 0:
            ic = lb.InCircuit
            if pr.circuits[ic].CircType == 1:
                src = pr.circuits[ic]
                nc = Circuit(**{**src.__dict__})
                nc.OrigCirc = ic
                nc.Amps_im = nc.Amps_im * lb.Turns
                nc.Amps_re = nc.Amps_re * lb.Turns
                pr.circuits.append(nc)
                lb.InCircuit = len(pr.circuits) - 1
    for c in pr.circuits:
        if c.CircType == 1:
            c.CircType = 0
    return pr


def get_fill_factor(pr: FemProblem, mesh=None) -> None:
    """FSolver::GetFillFactor (fsolver.cpp:1083-1193): bIsWound, and the
    proximity-effect permeability ProximityMu of AC wound regions (blocks of
    LamType > 2; wiretype = LamType - 3): for rectangular wire (3) an
    equivalent foil of pitch d / sqrt(fill) (:1128-1141), for round wire the
    fitted ufd = c2 tanh(sqrt(c1 I W)) / sqrt(c1 I W) + 1 - c2 with
    W = omega sigma muo R^2 / 2 (:1143-1192).  The region's area comes from
    the mesh (ElmArea, :1196-1210, nodes in cm); without a mesh ProximityMu
    stays 1.  Copper-clad aluminium (wiretypes 4, 5) leaves R = 0 in the
    reference and gives 0/0 (NaN) here too."""
    import cmath
    muo = 4e-7 * math.pi
    for li, lb in enumerate(pr.labels):
        bp = pr.blocks[lb.BlockType] if lb.BlockType >= 0 else None
        bt = bp.LamType if bp is not None else 0
        lb.bIsWound = (abs(lb.Turns) > 1) or (bt > 2)
        lb.ProximityMu = 1.0
        if pr.Frequency == 0 or bt < 3 or mesh is None:
            continue
        sel = np.asarray(mesh.lbl) == li
        p = np.asarray(mesh.p)[sel]
        x, y = np.asarray(mesh.x), np.asarray(mesh.y)
        atot = 0.0
        for n0, n1, n2 in p:   # element order, as the reference sums
            b0, b1 = y[n1] - y[n2], y[n2] - y[n0]
            c0, c1 = x[n2] - x[n1], x[n0] - x[n2]
            atot += 0.0001 * (b0 * c1 - b1 * c0) / 2.
        if atot == 0 or bp.Cduct == 0:
            continue
        wt = bt - 3
        if wt == 3:
            W = 2. * math.pi * pr.Frequency
            d = bp.WireD * 0.001
            fill = abs(d * d * lb.Turns / atot)
            dd = d / math.sqrt(fill)
            fill = d / dd
            o = bp.Cduct * (d / dd) * 1.e6
            k = cmath.sqrt(1j * W * o * muo) * d / 2.
            ufd = muo * cmath.tanh(k) / k
            lb.ProximityMu = (fill * ufd + (1. - fill) * muo) / muo
            continue
        R = awire = 0.0
        if wt in (0, 2):
            R = bp.WireD * 0.0005
            awire = math.pi * R * R * bp.NStrands * lb.Turns
        elif wt == 1:
            R = bp.WireD * 0.0005 * math.sqrt(bp.NStrands)
            awire = math.pi * R * R * lb.Turns
        fill = abs(awire / atot)
        W = 2. * math.pi * pr.Frequency * bp.Cduct * 1.e6 * muo * R * R / 2.
        if wt <= 2:
            c1 = 0.7756067409818643 + fill * (0.6873854335408803 + fill * (0.06841584481674128
                                                                          - 0.07143732702512284 * fill))
            c2 = 1.5 * fill / c1
        elif wt == 4:
            c1 = (0.7270741505617485 + 0.8902950067721367 * fill + 0.11894736885885195 * fill ** 2
                  - 0.12247276254503957 * fill ** 3)
            c2 = (0.006784920229549677 + 1.8942880489198526 * fill - 1.3631438759519217 * fill ** 2
                  + 0.504431701685587 * fill ** 3)
        else:
            c1 = (0.7486913529860821 + 0.9042845510838825 * fill + 0.1361040321433224 * fill ** 2
                  - 0.10652380745682069 * fill ** 3)
            c2 = (0.006790468527313965 + 1.8945509985370095 * fill - 1.3643501010185972 * fill ** 2
                  + 0.5036765577982594 * fill ** 3)
        z = cmath.sqrt(c1 * 1j * W)
        lb.ProximityMu = c2 * (cmath.tanh(z) / z) + (1. - c2) if z != 0 else complex("nan+nanj")


# --------------------------------------------------------------------------
# Mesh
# --------------------------------------------------------------------------

@dataclass
class Mesh:
    x: np.ndarray            # cm
    y: np.ndarray            # cm
    marker: np.ndarray       # point-prop index or -1
    p: np.ndarray            # (ne,3) int32
    e: np.ndarray            # (ne,3) boundary prop index or -1
    lbl: np.ndarray          # (ne,)
    blk: np.ndarray          # (ne,)
    pbc: np.ndarray          # (npbc,3) x,y,t
    bandwidth: int = 0
    edges: Optional[np.ndarray] = None   # (nedge,3) n0,n1,marker (raw .edge content)
    # air-gap elements (CAirGapElement): dicts format, ri, ro, total_arc_length,
    # inner_shift, outer_shift, qn / qw ((n_arc + 1) x 4)
    ages: list = dataclasses.field(default_factory=list)


def _read_ints_floats(path):
    with open(path, "r") as fh:
        return fh.read().split()


def load_mesh(base: str, pr: FemProblem) -> Mesh:
    """FSolver::LoadMesh (fsolver.cpp:350-718): .node .pbc .ele .edge."""
    conv = 100.0 * LENGTH_CONV_METERS[pr.LengthUnits]
    tok = _read_ints_floats(base + ".node")
    nn = int(tok[0])
    hdr = 4
    body = np.array(tok[hdr:hdr + 4 * nn], dtype=object).reshape(nn, 4)
    x = np.array([float(v) for v in body[:, 1]]) * conv
    y = np.array([float(v) for v in body[:, 2]]) * conv
    mk = np.array([int(v) for v in body[:, 3]], dtype=np.int64)
    marker = np.where(mk > 1, mk - 2, -1).astype(np.int32)

    with open(base + ".pbc", "r") as fh:
        plines = fh.read().splitlines()
    npbc = int(plines[0].split()[0])
    pbc = np.zeros((npbc, 3), dtype=np.int32)
    for i in range(npbc):
        f = plines[1 + i].split()
        pbc[i] = (int(f[1]), int(f[2]), int(f[3]))
    # air-gap elements (fsolver.cpp:425-515): name line, parameter line,
    # totalArcElements + 1 quadNode lines
    nage = int(plines[1 + npbc].split()[0]) if len(plines) > 1 + npbc else 0
    ages, _ = _parse_age_blocks(plines, 2 + npbc, nage)

    tok = _read_ints_floats(base + ".ele")
    ne = int(tok[0])
    body = np.array(tok[3:3 + 5 * ne], dtype=np.int64).reshape(ne, 5)
    p = body[:, 1:4].astype(np.int32)
    lbl = body[:, 4] - 1
    default_label = -1
    for i, lb in enumerate(pr.labels):
        if lb.IsDefault:
            default_label = i
    lbl = np.where(lbl < 0, default_label, lbl)
    if (lbl < 0).any():
        raise ValueError("Material properties have not been defined for all regions.")
    if (lbl >= len(pr.labels)).any():
        raise ValueError("element label number greater than the number of labels")
    lbl = lbl.astype(np.int32)
    blk = np.array([pr.labels[l].BlockType for l in lbl], dtype=np.int32)

    tok = _read_ints_floats(base + ".edge")
    ned = int(tok[0])
    ebody = np.array(tok[2:2 + 4 * ned], dtype=np.int64).reshape(ned, 4)
    edges = ebody[:, 1:4].astype(np.int64)
    e = -np.ones((ne, 3), dtype=np.int32)
    # node -> element membership lists (fsolver.cpp:633-657)
    mbr: List[List[int]] = [[] for _ in range(nn)]
    for i in range(ne):
        for j in range(3):
            mbr[p[i, j]].append(i)
    for n0, n1, j in edges:
        if j < 0:
            j = -(j + 2)
            for el in mbr[n0]:
                a, b, c = p[el]
                if (a == n0 and b == n1) or (a == n1 and b == n0):
                    e[el, 0] = j
                if (b == n0 and c == n1) or (b == n1 and c == n0):
                    e[el, 1] = j
                if (c == n0 and a == n1) or (c == n1 and a == n0):
                    e[el, 2] = j
    return Mesh(x=x, y=y, marker=marker, p=p, e=e, lbl=lbl, blk=blk, pbc=pbc, edges=edges, ages=ages)


def cuthill(mesh: Mesh) -> np.ndarray:
    """FEASolver::Cuthill + SortNodes + SortElements (cuthill.cpp).  Modifies mesh
    in place and returns newnum (old -> new node number)."""
    nn = len(mesh.x)
    edges = mesh.edges
    numcon = [0] * nn
    for n0, n1, _ in edges:
        numcon[n0] += 1
        numcon[n1] += 1
    ocon: List[List[int]] = [[] for _ in range(nn)]
    for n0, n1, _ in edges:
        ocon[n0].append(int(n1))
        ocon[n1].append(int(n0))
    # bubble sort by increasing connectivity (cuthill.cpp: "I'm lazy")
    for n0 in range(nn):
        lst = ocon[n0]
        m = len(lst)
        for _ in range(1, m):
            for j in range(1, m):
                if numcon[lst[j]] < numcon[lst[j - 1]]:
                    lst[j], lst[j - 1] = lst[j - 1], lst[j]
    # starting node
    j = numcon[0]
    n0 = 0
    i = 1
    n_lines = len(edges)
    while i < nn:
        if numcon[i] < j:
            j = numcon[i]
            n0 = i
        if j == 2:
            i = n_lines
        i += 1
    newnum = [-1] * nn
    nxtnum = [-1] * nn
    newnum[n0] = 0
    n = 1
    nxtnum[0] = n0
    while True:
        for k in ocon[n0]:
            if newnum[k] < 0:
                newnum[k] = n
                nxtnum[n] = k
                n += 1
        if nxtnum[newnum[n0] + 1] < 0:
            jj = 0
            for ii in range(nn):
                if newnum[ii] < 0:
                    jj = numcon[ii]
                    n0 = ii
                    break
            for ii in range(nn):
                if newnum[ii] < 0 and numcon[ii] < jj:
                    jj = numcon[ii]
                    n0 = ii
                if jj == 2:
                    break
            newnum[n0] = n
            nxtnum[n] = n0
            n += 1
        else:
            n0 = nxtnum[newnum[n0] + 1]
        if n >= nn:
            break
    newnum_a = np.array(newnum, dtype=np.int64)
    # remap air-gap quadNodes (cuthill.cpp:321-330) and pbcs
    for a in mesh.ages:
        a["qn"] = newnum_a[a["qn"]].astype(np.int32)
    if len(mesh.pbc):
        mesh.pbc[:, 0] = newnum_a[mesh.pbc[:, 0]]
        mesh.pbc[:, 1] = newnum_a[mesh.pbc[:, 1]]
    # new bandwidth
    newwide = 0
    for a in range(nn):
        for b in ocon[a]:
            d = abs(newnum[a] - newnum[b])
            if d > newwide:
                newwide = d
    mesh.bandwidth = newwide + 1
    mesh.p = newnum_a[mesh.p].astype(np.int32)
    # SortNodes: node i moves to position newnum[i]
    inv = np.empty(nn, dtype=np.int64)
    inv[newnum_a] = np.arange(nn)
    mesh.x = mesh.x[inv]
    mesh.y = mesh.y[inv]
    mesh.marker = mesh.marker[inv]
    _sort_elements(mesh)
    return newnum_a


def _sort_elements(mesh: Mesh) -> None:
    """FEASolver::SortElements: comb sort on p0+p1+p2 (cuthill.cpp:39-86).
    The comb sort is not stable, so it is restated exactly."""
    ne = len(mesh.lbl)
    score = (mesh.p[:, 0].astype(np.int64) + mesh.p[:, 1] + mesh.p[:, 2]).tolist()
    order = list(range(ne))
    gap = ne
    while True:
        if gap > 1:
            gap = (gap * 10) // 13
            if gap == 10 or gap == 9:
                gap = 11
        swapped = 0
        j = 0
        while j + gap < ne:
            if score[j] > score[j + gap]:
                k = j + gap
                score[j], score[k] = score[k], score[j]
                order[j], order[k] = order[k], order[j]
                swapped = 1
            j += 1
        if not (gap > 1 and swapped > 0):
            break
    o = np.array(order, dtype=np.int64)
    mesh.p = mesh.p[o]
    mesh.e = mesh.e[o]
    mesh.lbl = mesh.lbl[o]
    mesh.blk = mesh.blk[o]


# --------------------------------------------------------------------------
# .ans reader (WriteStatic2D layout, static2d.cpp:1038-1195; old FEMM 4.0 too)
# --------------------------------------------------------------------------

@dataclass
class AnsSolution:
    x: np.ndarray     # in problem length units
    y: np.ndarray
    A: np.ndarray
    marker: Optional[np.ndarray]
    p: np.ndarray
    lbl: np.ndarray
    circ: List[tuple]
    pbc: Optional[np.ndarray] = None
    ages: list = dataclasses.field(default_factory=list)   # as Mesh.ages, renumbered node ids


def _parse_age_blocks(lines, i, nage):
    """AGE blocks as FSolver::LoadMesh reads them from the .pbc and
    WriteStatic2D writes them to the .ans (fsolver.cpp:425-515,
    static2d.cpp:1161-1190): name, parameter line, n_arc + 1 quadNodes."""
    ages = []
    for _ in range(nage):
        name = lines[i].strip().strip('"')
        f = lines[i + 1].split()
        n = int(f[8])
        q = [lines[i + 2 + k].split() for k in range(n + 1)]
        ages.append(dict(name=name, format=int(f[0]), inner_angle=float(f[1]), outer_angle=float(f[2]),
                         ri=float(f[3]), ro=float(f[4]), total_arc_length=float(f[5]),
                         inner_shift=float(f[9]), outer_shift=float(f[10]),
                         qn=np.array([[int(r[0]), int(r[2]), int(r[4]), int(r[6])] for r in q], np.int32),
                         qw=np.array([[float(r[1]), float(r[3]), float(r[5]), float(r[7])] for r in q])))
        i += n + 3
    return ages, i


def read_ans(path: str) -> AnsSolution:
    with open(path, "r") as fh:
        lines = fh.read().splitlines()
    k = next(i for i, ln in enumerate(lines) if ln.strip().lower().startswith("[solution]"))
    i = k + 1
    nn = int(lines[i]); i += 1
    node = [lines[i + j].split() for j in range(nn)]
    i += nn
    x = np.array([float(f[0]) for f in node])
    y = np.array([float(f[1]) for f in node])
    A = np.array([float(f[2]) for f in node])
    marker = np.array([int(f[3]) for f in node]) if len(node[0]) > 3 else None
    ne = int(lines[i]); i += 1
    ele = np.array([[int(v) for v in lines[i + j].split()[:4]] for j in range(ne)], dtype=np.int64)
    i += ne
    nl = int(lines[i]); i += 1
    circ = []
    for j in range(nl):
        f = lines[i + j].split()
        circ.append((int(f[0]), float(f[1])))
    i += nl
    pbc, ages = None, []
    if i < len(lines) and lines[i].strip():       # periodic pairs + air-gap elements (static2d.cpp:1152-1190)
        npbc = int(lines[i]); i += 1
        pbc = np.array([[int(v) for v in lines[i + j].split()[:3]] for j in range(npbc)], dtype=np.int32)
        i += npbc
        if i < len(lines) and lines[i].strip():
            nage = int(lines[i]); i += 1
            ages, i = _parse_age_blocks(lines, i, nage)
    return AnsSolution(x=x, y=y, A=A, marker=marker, p=ele[:, :3].astype(np.int32),
                       lbl=ele[:, 3].astype(np.int32), circ=circ, pbc=pbc, ages=ages)


@dataclass
class PrevSolution:
    """What FSolver::loadPreviousSolution keeps: the mesh and, for PrevType != 0,
    A of the previous (DC) solution per node; Jprev per element."""
    mesh: Mesh
    Aprev: Optional[np.ndarray]
    Jprev: np.ndarray


def _scan(fields, conv):
    """sscanf over whitespace fields with the given converters: the values up
    to the first field that is missing or does not convert."""
    out = []
    for f, c in zip(fields, conv):
        try:
            out.append(c(f))
        except ValueError:
            break
    return out


def _c_int(tok: str) -> int:
    """%i of sscanf: the leading integer of the token ("-10.5" -> -10)."""
    import re
    m = re.match(r"[+-]?(0[xX][0-9a-fA-F]+|0[0-7]*|[1-9][0-9]*)", tok)
    if not m:
        raise ValueError(tok)
    return int(m.group(0), 0)


def load_previous_solution(pr: FemProblem, path: str, load_aprev: bool) -> PrevSolution:
    """FSolver::loadPreviousSolution (fsolver.cpp:990-1081) with
    LoadMeshNodesFromSolution (:801-840), LoadMeshElementsFromSolution
    (:842-880), LoadPBCFromSolution (:882-909), LoadAGEsFromSolution (:911-988).

    Reproduced as the reference reads a WriteStatic2D .ans: element lines
    carry p0 p1 p2 lbl only, so the sscanf of 8 fields leaves e[] and Jprev at
    the CMElement defaults -- e = {0, 0, 0} (CElement.cpp:30-39): EVERY edge of
    every element carries boundary property 0 -- and Jprev = 0.  Node
    coordinates come back through x / unitconv * 100 LengthConvMeters."""
    if not os.path.exists(path):
        raise PrevSolnError("Failed to open the specified previous solution file, file path was:\n%s\n" % path)
    with open(path, "r") as fh:
        lines = fh.read().split("\n")
    i, has = 0, False
    while i < len(lines):
        toks = lines[i].split()
        q = toks[0].lower() if toks else ""
        if q.startswith("[frequency]"):
            v = lines[i].split("=", 1)[1] if "=" in lines[i] else ""
            f = _scan(v.split(), [float])
            if f and f[0] != 0:
                raise PrevSolnError("Previous solution file (%s) appears to be an AC problem, only DC previous "
                                    "solutions are presently supported\n" % path)
        i += 1
        if q.startswith("[solution]"):
            has = True
            break
    if not has:
        raise PrevSolnError("No solution was found in previous solution file, file path was:\n%s\n" % path)
    conv = 100.0 * LENGTH_CONV_METERS[pr.LengthUnits]
    nn = _c_int(lines[i].split()[0]); i += 1
    x, y, A, mk = np.zeros(nn), np.zeros(nn), np.zeros(nn), np.zeros(nn, np.int32)
    for j in range(nn):
        v = _scan(lines[i + j].split(), [float, float, float, _c_int])
        x[j], y[j], A[j], mk[j] = v[0] * conv, v[1] * conv, v[2], v[3]
    i += nn
    ne = _c_int(lines[i].split()[0]); i += 1
    p = np.zeros((ne, 3), np.int32)
    lbl = np.zeros(ne, np.int32)
    e = np.zeros((ne, 3), np.int32)      # CElement() default, not -1
    Jprev = np.zeros(ne)
    for j in range(ne):
        v = _scan(lines[i + j].split(), [_c_int] * 7 + [float])
        p[j], lbl[j] = v[0:3], v[3]
        for q in range(3):
            if len(v) > 4 + q:
                e[j, q] = v[4 + q]
        if len(v) > 7:
            Jprev[j] = v[7]
    i += ne
    blk = np.array([pr.labels[l].BlockType for l in lbl], np.int32)
    nlab = _c_int(lines[i].split()[0]); i += 1 + nlab      # block-label circuit lines: skipped
    npbc = _c_int(lines[i].split()[0]) if i < len(lines) and lines[i].split() else 0
    i += 1
    pbc = np.zeros((npbc, 3), np.int32)
    for j in range(npbc):
        pbc[j] = _scan(lines[i + j].split(), [_c_int] * 3)
    i += npbc
    nage = _c_int(lines[i].split()[0]) if i < len(lines) and lines[i].split() else 0
    ages, _ = _parse_age_blocks(lines, i + 1, nage)
    mesh = Mesh(x=x, y=y, marker=mk, p=p, e=e, lbl=lbl, blk=blk, pbc=pbc, bandwidth=0, ages=ages)
    return PrevSolution(mesh=mesh, Aprev=A if load_aprev else None, Jprev=Jprev)


def load_problem(base: str, renumber: bool = True, with_prev: bool = False):
    """Convenience: parse + prepare + mesh (+ Cuthill) like FSolver::runSolver.
    With [PrevSoln] the mesh is the previous solution's (no Cuthill,
    fsolver.cpp:1224); ``with_prev`` also returns the PrevSolution."""
    pr = prepare_problem(parse_fem(base + ".fem"))
    prev = None
    if pr.PrevSoln:
        # FSolver::runSolver (fsolver.cpp:1245-1320)
        if pr.Frequency == 0 and pr.PrevType != 0:
            raise PrevSolnError("Cannot handle incremental permeability problems with frequency 0.\n")
        if pr.Frequency != 0 and pr.ProblemType == 1:
            raise PrevSolnError("Cannot handle harmonic axisymmetric incremental problems.\n")
        prev = load_previous_solution(pr, pr.PrevSoln, pr.PrevType != 0)
        mesh = prev.mesh
    else:
        mesh = load_mesh(base, pr)
        if renumber:
            cuthill(mesh)
    get_fill_factor(pr, mesh)
    return (pr, mesh, prev) if with_prev else (pr, mesh)
