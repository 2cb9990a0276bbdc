"""Synthetic magnetostatic problems on refined square-domain meshes.

The bench workloads of BASELINE.json ("Synthetic 2M-tri square-domain
magnetostatic", linear mu and M-19 nonlinear B-H) need meshes far larger than
the reference's test problems; fmesher (Triangle) is outside this project's
scope, so this module generates structured triangulations directly in the
in-memory form FSolver::LoadMesh produces (cfemm/fsolver/fsolver.cpp:350-718):
node coordinates in cm, 0-based element nodes, block-label index per element,
boundary-property index per element edge, plus the .fem-level property tables.

Geometry (unit square of side L cm, n x n cells, each split into 2 triangles
with alternating diagonals):
  * air everywhere, Dirichlet A = 0 ("A=0" boundary, BdryFormat 0) on the outer edge
  * a steel C-core (linear mu_r or the M-19 B-H curve, LamFill 0.98, LamType 0)
  * two coil sides with +J / -J (MA/m^2)
  * a NdFeB magnet block (H_c = 979 kA/m, magnetised along +y)
"""
from __future__ import annotations

import os
from typing import Optional

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))


def m19_curve():
    """M-19 steel B-H points (FEMM material library, mfemm/matlib.dat:1168-1221)."""
    path = os.path.join(_HERE, "data", "M19_Steel.bh")
    data = np.loadtxt(path)
    return data[:, 0].copy(), data[:, 1].copy()


def square_mesh(n: int, L: float = 10.0, order: str = "rows"):
    """Nodes (n+1)^2 on [0,L]^2 (cm), 2 n^2 triangles (counter-clockwise)."""
    m = n + 1
    xs = np.linspace(0.0, L, m)
    X, Y = np.meshgrid(xs, xs, indexing="xy")     # row j = y index
    x = X.reshape(-1).copy()
    y = Y.reshape(-1).copy()
    j, i = np.meshgrid(np.arange(n), np.arange(n), indexing="ij")
    i = i.reshape(-1)
    j = j.reshape(-1)
    n00 = j * m + i
    n10 = n00 + 1
    n01 = n00 + m
    n11 = n01 + 1
    alt = ((i + j) & 1) == 0
    # two triangles per cell, both counter-clockwise
    t1 = np.where(alt[:, None], np.stack([n00, n10, n11], 1), np.stack([n00, n10, n01], 1))
    t2 = np.where(alt[:, None], np.stack([n00, n11, n01], 1), np.stack([n10, n11, n01], 1))
    p = np.empty((2 * n * n, 3), dtype=np.int32)
    p[0::2] = t1
    p[1::2] = t2
    return x, y, p


def _boundary_edges(p, x, y, L, tol):
    """e[el, j] = 0 for edges (p[j], p[j+1]) on the outer boundary, else -1."""
    on = (np.abs(x) < tol) | (np.abs(x - L) < tol) | (np.abs(y) < tol) | (np.abs(y - L) < tol)
    e = -np.ones(p.shape, dtype=np.int32)
    for j in range(3):
        a, b = p[:, j], p[:, (j + 1) % 3]
        same_x = (np.abs(x[a] - x[b]) < tol) & ((np.abs(x[a]) < tol) | (np.abs(x[a] - L) < tol))
        same_y = (np.abs(y[a] - y[b]) < tol) & ((np.abs(y[a]) < tol) | (np.abs(y[a] - L) < tol))
        e[(on[a] & on[b]) & (same_x | same_y), j] = 0
    return e


def magnetostatic(n: int, nonlinear: bool = False, L: float = 10.0, J: float = 2.0,
                  mu_steel: float = 1000.0, precision: float = 1e-8, with_magnet: bool = True):
    """Keyword arguments for kernels.Static2DProblem (and the oracle) of an
    n x n-cell square problem: 2 n^2 triangles, (n+1)^2 nodes."""
    x, y, p = square_mesh(n, L)
    cx = (x[p[:, 0]] + x[p[:, 1]] + x[p[:, 2]]) / 3.0
    cy = (y[p[:, 0]] + y[p[:, 1]] + y[p[:, 2]]) / 3.0
    u, v = cx / L, cy / L
    lbl = np.zeros(len(p), dtype=np.int32)                       # 0: air
    core = (u > 0.25) & (u < 0.75) & (v > 0.25) & (v < 0.75)
    window = (u > 0.35) & (u < 0.65) & (v > 0.35) & (v < 0.65)
    gap = (u > 0.70) & (v > 0.45) & (v < 0.55)
    steel = core & ~window & ~gap
    lbl[steel] = 1                                               # 1: steel
    coil_a = (u > 0.37) & (u < 0.45) & (v > 0.38) & (v < 0.62)
    coil_b = (u > 0.55) & (u < 0.63) & (v > 0.38) & (v < 0.62)
    lbl[coil_a] = 2                                              # 2: coil +J
    lbl[coil_b] = 3                                              # 3: coil -J
    if with_magnet:
        mag = (u > 0.08) & (u < 0.16) & (v > 0.40) & (v < 0.60)
        lbl[mag] = 4                                             # 4: magnet
    blocks = [
        dict(mu_x=1.0, mu_y=1.0),                                # air
        dict(mu_x=mu_steel, mu_y=mu_steel, LamFill=1.0),         # steel (linear)
        dict(mu_x=1.0, mu_y=1.0, J_re=J),                        # coil +
        dict(mu_x=1.0, mu_y=1.0, J_re=-J),                       # coil -
        dict(mu_x=1.049, mu_y=1.049, H_c=979000.0, Cduct=0.667), # NdFeB 40 MGOe
    ]
    if nonlinear:
        blocks[1] = dict(mu_x=1.0, mu_y=1.0, LamFill=0.98, LamType=0, bh="M19")
    labels = [dict(block=0), dict(block=1), dict(block=2), dict(block=3), dict(block=4, mag_dir=90.0)]
    for b in blocks:
        if b.get("bh") == "M19":
            from .fsolver import bh_get_slopes
            Bc, Hc, Sc, mu = bh_get_slopes(*m19_curve(), lam_type=b.get("LamType", 0),
                                           lam_fill=b.get("LamFill", 1.0))
            b.update(B=Bc, H=Hc, slope=Sc, mu_x=mu, mu_y=mu)
    tol = 1e-9 * L
    e = _boundary_edges(p, x, y, L, tol)
    lines = [dict(format=0)]
    return dict(x=x, y=y, p=p, lbl=lbl, e=e, marker=None, pbc=None, blocks=blocks, labels=labels,
                lines=lines, points=[], circuits=[], precision=precision, length_units=2, coords=0, relax=1.0)


def fem_text(blocks, lines, precision=1e-8, units="centimeters", frequency=0.0, problem_type=0,
             ext=(0.0, 0.0, 0.0), ac_solver=0) -> str:
    """A .fem header carrying the property tables (no geometry: meshes are given)."""
    out = ["[Format]      =  4.0", "[Frequency]   =  %.17g" % frequency, "[Precision]   =  %.17g" % precision,
           "[MinAngle]    =  30", "[Depth]       =  1", "[LengthUnits] =  %s" % units,
           "[ProblemType] =  %s" % ("axisymmetric" if problem_type == 1 else "planar"),
           "[Coordinates] =  cartesian", "[ACSolver]    =  %d" % ac_solver,
           "[extZo] = %.17g" % ext[0], "[extRo] = %.17g" % ext[1], "[extRi] = %.17g" % ext[2],
           '[PrevSoln]    = ""', "[PrevType]    =  0", '[Comment]     =  "synthetic"',
           "[PointProps]   = 0", "[BdryProps]   = %d" % len(lines)]
    for k, ln in enumerate(lines):
        out += ["  <BeginBdry>", '    <BdryName> = "b%d"' % k, "    <BdryType> = %d" % ln.get("format", 0),
                "    <A_0> = %.17g" % ln.get("A0", 0.0), "    <A_1> = %.17g" % ln.get("A1", 0.0),
                "    <A_2> = %.17g" % ln.get("A2", 0.0), "    <Phi> = %.17g" % ln.get("phi", 0.0),
                "    <c0> = %.17g" % ln.get("c0", 0.0), "    <c0i> = %.17g" % ln.get("c0_im", 0.0),
                "    <c1> = %.17g" % ln.get("c1", 0.0), "    <c1i> = %.17g" % ln.get("c1_im", 0.0),
                "    <Mu_ssd> = %.17g" % ln.get("Mu", 0.0), "    <Sigma_ssd> = %.17g" % ln.get("Sig", 0.0),
                "  <EndBdry>"]
    out.append("[BlockProps]  = %d" % len(blocks))
    for k, b in enumerate(blocks):
        out += ["  <BeginBlock>", '    <BlockName> = "m%d"' % k, "    <Mu_x> = %.17g" % b.get("mu_x", 1.0),
                "    <Mu_y> = %.17g" % b.get("mu_y", 1.0), "    <H_c> = %.17g" % b.get("H_c", 0.0),
                "    <H_cAngle> = 0", "    <J_re> = %.17g" % b.get("J_re", 0.0),
                "    <J_im> = %.17g" % b.get("J_im", 0.0), "    <Sigma> = %.17g" % b.get("Cduct", 0.0),
                "    <d_lam> = %.17g" % b.get("Lam_d", 0.0), "    <Phi_h> = %.17g" % b.get("Theta_hn", 0.0),
                "    <Phi_hx> = %.17g" % b.get("Theta_hx", 0.0), "    <Phi_hy> = %.17g" % b.get("Theta_hy", 0.0),
                "    <LamType> = %d" % b.get("LamType", 0),
                "    <LamFill> = %.17g" % b.get("LamFill", 1.0), "    <NStrands> = %d" % b.get("NStrands", 0),
                "    <WireD> = %.17g" % b.get("WireD", 0.0)]
        if b.get("bh") == "M19":
            B, H = m19_curve()
            out.append("    <BHPoints> = %d" % len(B))
            out += ["      %.17g\t%.17g" % (bb, hh) for bb, hh in zip(B, H)]
        else:
            out.append("    <BHPoints> = 0")
        out.append("  <EndBlock>")
    out.append("[CircuitProps]  = 0")
    return "\n".join(out) + "\n"


def write_problem(base: str, kw: dict, label_xy: Optional[np.ndarray] = None) -> None:
    """Write <base>.fem/.node/.ele/.edge/.pbc in the fmesher layout so the same
    synthetic problem runs through the file-based FSolver path."""
    x, y, p, lbl, e = kw["x"], kw["y"], kw["p"], kw["lbl"], kw["e"]
    conv = 1.0   # centimeters
    text = fem_text(kw["blocks"], kw["lines"], kw["precision"], frequency=kw.get("frequency", 0.0),
                    problem_type=kw.get("problem_type", 0),
                    ext=(kw.get("ext_zo", 0.0), kw.get("ext_ro", 0.0), kw.get("ext_ri", 0.0)),
                    ac_solver=kw.get("ac_solver", 0))
    labels = kw["labels"]
    text += "[NumPoints] = 0\n[NumSegments] = 0\n[NumArcSegments] = 0\n[NumHoles] = 0\n"
    text += "[NumBlockLabels] = %d\n" % len(labels)
    for k, lb in enumerate(labels):
        text += "0\t0\t%d\t-1\t%d\t%.17g\t0\t%d\t%d\n" % (lb["block"] + 1, lb.get("in_circuit", -1) + 1,
                                                        lb.get("mag_dir", 0.0), int(lb.get("turns", 1)),
                                                        int(lb.get("is_external", 0)))
    with open(base + ".fem", "w") as fh:
        fh.write(text)
    x = np.asarray(x, dtype=np.float64)
    y = np.asarray(y, dtype=np.float64)
    p = np.asarray(p).reshape(-1, 3)
    lbl = np.asarray(lbl)
    e = np.asarray(e).reshape(-1, 3)
    with open(base + ".node", "w") as fh:
        fh.write("%d\t2\t0\t1\n" % len(x))
        fh.write("".join("%d\t%.17g\t%.17g\t0\n" % t for t in zip(range(len(x)), (x / conv).tolist(),
                                                                      (y / conv).tolist())))
    with open(base + ".ele", "w") as fh:
        fh.write("%d\t3\t1\n" % len(p))
        fh.write("".join("%d\t%d\t%d\t%d\t%d\n" % t for t in zip(range(len(p)), p[:, 0].tolist(), p[:, 1].tolist(),
                                                                    p[:, 2].tolist(), (lbl + 1).tolist())))
    # every element edge once, sorted by (min, max) node; an edge carrying a
    # boundary property keeps the marker -(prop + 2) (the last one in element
    # order when several elements give one), else 0
    a = p.reshape(-1)
    b = p[:, [1, 2, 0]].reshape(-1)
    lo, hi = np.minimum(a, b).astype(np.int64), np.maximum(a, b).astype(np.int64)
    mk = np.where(e.reshape(-1) >= 0, -(e.reshape(-1).astype(np.int64) + 2), 0)
    key = lo * (int(hi.max()) + 1 if len(hi) else 1) + hi
    order = np.lexsort((np.arange(len(key)), mk != 0, key))   # per key: unmarked first, then marked in element order
    ks = key[order]
    last = np.r_[ks[1:] != ks[:-1], True]                      # the last entry of each key wins
    sel = order[last]
    with open(base + ".edge", "w") as fh:
        fh.write("%d\t1\n" % len(sel))
        fh.write("".join("%d\t%d\t%d\t%d\n" % t for t in zip(range(len(sel)), lo[sel].tolist(), hi[sel].tolist(),
                                                               mk[sel].tolist())))
    # .pbc: periodic pairs, then the air-gap elements (writepoly.cpp:1836-1966)
    pbc = kw.get("pbc")
    pbc = np.zeros((0, 3), np.int32) if pbc is None else np.asarray(pbc).reshape(-1, 3)
    with open(base + ".pbc", "w") as fh:
        fh.write("%d\n" % len(pbc))
        for k, (a, b, t) in enumerate(pbc):
            fh.write("%d\t%d\t%d\t%d\n" % (k, a, b, t))
        ages = kw.get("ages", [])
        fh.write("%d\n" % len(ages))
        for k, a in enumerate(ages):
            qn, qw = np.asarray(a["qn"]), np.asarray(a["qw"])
            c = a.get("center", (0.0, 0.0))
            fh.write('"age%d"\n' % k)
            fh.write("%d %.17g %.17g %.17g %.17g %.17g %.17g %.17g %d %.17g %.17g\n" % (
                a.get("format", 0), a.get("inner_angle", 0.0), a.get("outer_angle", 0.0), a["ri"], a["ro"],
                a["total_arc_length"], c[0], c[1], len(qn) - 1, a["inner_shift"], a["outer_shift"]))
            for i in range(len(qn)):
                fh.write("%d %g %d %g %d %g %d %g\n" % (qn[i, 0], qw[i, 0], qn[i, 1], qw[i, 1], qn[i, 2], qw[i, 2],
                                                        qn[i, 3], qw[i, 3]))


def axisymmetric(n: int, nonlinear: bool = False, L: float = 10.0, J: float = 2.0, mu_steel: float = 1000.0,
                 precision: float = 1e-8, mixed: bool = True, circuit: bool = False, external: bool = False):
    """Keyword arguments of an axisymmetric (StaticAxisymmetric) problem on the
    n x n-cell square r in [0, L], z in [0, L] (cm): a steel pot core around a
    coil ring, a radially thin NdFeB ring magnetised along +z, A = 0 on the
    outer radius and the bottom, a mixed (c0, c1) condition on the top unless
    `mixed` is off; the axis r = 0 takes A = 0 by the solver's own rule.
    `circuit`: the coil carries a series circuit current instead of J;
    `external`: the outer band r > 0.8 L is a conformally mapped exterior
    region (IsExternal, extRo = 0.8 L, extRi = 0.7 L, extZo = L / 2)."""
    x, y, p = square_mesh(n, L)
    cx = (x[p[:, 0]] + x[p[:, 1]] + x[p[:, 2]]) / 3.0
    cy = (y[p[:, 0]] + y[p[:, 1]] + y[p[:, 2]]) / 3.0
    u, v = cx / L, cy / L
    lbl = np.zeros(len(p), dtype=np.int32)                                      # 0: air
    pot = (u < 0.45) & (v > 0.25) & (v < 0.75)
    cavity = (u > 0.12) & (u < 0.38) & (v > 0.32) & (v < 0.68)
    lbl[pot & ~cavity] = 1                                                      # 1: steel
    lbl[(u > 0.16) & (u < 0.32) & (v > 0.36) & (v < 0.64)] = 2                  # 2: coil
    lbl[(u > 0.55) & (u < 0.6) & (v > 0.42) & (v < 0.58)] = 3                   # 3: magnet ring
    if external:
        lbl[(u > 0.8) & (lbl == 0)] = 4                                         # 4: exterior air
    blocks = [dict(mu_x=1.0, mu_y=1.0),
              dict(mu_x=mu_steel, mu_y=mu_steel, LamFill=1.0),
              dict(mu_x=1.0, mu_y=1.0, J_re=0.0 if circuit else J, Cduct=58.0 if circuit else 0.0),
              dict(mu_x=1.049, mu_y=1.049, H_c=979000.0, Cduct=0.667)]
    if nonlinear:
        blocks[1] = dict(mu_x=1.0, mu_y=1.0, LamFill=0.98, LamType=0, bh="M19")
    labels = [dict(block=0), dict(block=1), dict(block=2, in_circuit=0 if circuit else -1, is_wound=1),
              dict(block=3, mag_dir=90.0)]
    if external:
        labels.append(dict(block=0, is_external=1))
    for b in blocks:
        if b.get("bh") == "M19":
            from .fsolver import bh_get_slopes
            Bc, Hc, Sc, mu = bh_get_slopes(*m19_curve(), lam_type=b.get("LamType", 0),
                                           lam_fill=b.get("LamFill", 1.0))
            b.update(B=Bc, H=Hc, slope=Sc, mu_x=mu, mu_y=mu)
    tol = 1e-9 * L
    e = _boundary_edges(p, x, y, L, tol)
    lines = [dict(format=0)]
    if mixed:   # top edge: c0 A + dA/dn = c1
        lines.append(dict(format=2, c0=2.0e5, c1=0.5))
        for j in range(3):
            a, b2 = p[:, j], p[:, (j + 1) % 3]
            top = (np.abs(y[a] - L) < tol) & (np.abs(y[b2] - L) < tol)
            e[top & (e[:, j] >= 0), j] = 1
    circuits = [dict(type=0, amps_re=4000.0)] if circuit else []
    kw = dict(x=x, y=y, p=p, lbl=lbl, e=e, marker=None, pbc=None, blocks=blocks, labels=labels, lines=lines,
              points=[], circuits=circuits, precision=precision, length_units=2, coords=0, relax=1.0,
              problem_type=1)
    if external:
        kw.update(ext_zo=L / 2, ext_ro=0.8 * L, ext_ri=0.7 * L)
    return kw


def axisymmetric_uniform(n: int, B0: float = 1.0, L: float = 10.0, precision: float = 1e-12):
    """Air-filled axisymmetric box with A = B0 r / 2 imposed on the outer
    boundary (A1 = B0 / 2 per metre of r, the mesh in cm): the solution is the
    uniform axial field, flux 2 pi r A = pi B0 r^2 (Wb, r in m) -- inside the
    formulation's c0 + c1 r^2 + c2 z flux space, so reproduced to roundoff."""
    x, y, p = square_mesh(n, L)
    e = _boundary_edges(p, x, y, L, 1e-9 * L)
    lines = [dict(format=0, A1=0.5 * B0 * 0.01)]
    return dict(x=x, y=y, p=p, lbl=np.zeros(len(p), dtype=np.int32), e=e, marker=None, pbc=None,
                blocks=[dict(mu_x=1.0, mu_y=1.0)], labels=[dict(block=0)], lines=lines, points=[], circuits=[],
                precision=precision, length_units=2, coords=0, relax=1.0, problem_type=1)


def harmonic_axisymmetric(n: int, L: float = 10.0, frequency: float = 60.0, precision: float = 1e-8,
                          circuits: bool = True, nonlinear: bool = False, external: bool = False,
                          prox: Optional[int] = None):
    """Keyword arguments of a time-harmonic axisymmetric problem
    (FSolver::HarmonicAxisymmetric, cfemm/fsolver/harmonicaxi.cpp) on the
    n x n-cell square r in [0, L], z in [0, L] (cm): a laminated lossy steel
    pot core (hysteresis lag) around a coil with a complex current density, an
    aluminium ring below it (eddy currents), A with a phase on the outer
    radius, a complex mixed condition on the top, a small-skin-depth bottom, a
    complex point current; the axis takes A = 0 by the solver's rule.
    `circuits`: the coil is a wound specified-current circuit (Case 1) and the
    ring is driven by a voltage gradient (Case 0); `nonlinear`: the steel
    follows the M-19 curve processed for the frequency; `external`: the outer
    band r > 0.8 L is a mapped exterior region; `prox` (wiretype 0-3): the coil
    is a copper winding of LamType 3 + prox with AC proximity effects."""
    x, y, p = square_mesh(n, L)
    cxm = (x[p[:, 0]] + x[p[:, 1]] + x[p[:, 2]]) / (3.0 * L)
    cym = (y[p[:, 0]] + y[p[:, 1]] + y[p[:, 2]]) / (3.0 * L)
    lbl = np.zeros(len(p), dtype=np.int32)                                          # 0: air
    pot = (cxm < 0.45) & (cym > 0.25) & (cym < 0.75)
    cavity = (cxm > 0.12) & (cxm < 0.38) & (cym > 0.32) & (cym < 0.68)
    lbl[pot & ~cavity] = 1                                                          # 1: steel
    lbl[(cxm > 0.16) & (cxm < 0.32) & (cym > 0.36) & (cym < 0.64)] = 2              # 2: coil
    lbl[(cxm > 0.1) & (cxm < 0.5) & (cym > 0.08) & (cym < 0.16)] = 3                # 3: aluminium ring
    if external:
        lbl[(cxm > 0.8) & (lbl == 0)] = 4                                           # 4: exterior air
    blocks = [dict(mu_x=1.0, mu_y=1.0),
              dict(mu_x=900.0, mu_y=900.0, Lam_d=0.35, LamFill=0.96, Cduct=2.0, Theta_hx=10.0, Theta_hy=10.0),
              dict(mu_x=1.0, mu_y=1.0, J_re=0.0 if circuits else 2.0, J_im=0.0 if circuits else 0.7),
              dict(mu_x=1.0, mu_y=1.0, Cduct=35.0)]
    if nonlinear:
        from .fsolver import bh_get_slopes_ac
        b1 = blocks[1]
        Bc, Hc, Sc, mu, _ = bh_get_slopes_ac(*m19_curve(), 2 * np.pi * frequency, lam_type=0,
                                             lam_fill=b1["LamFill"], theta_hn=b1["Theta_hx"], lam_d=b1["Lam_d"],
                                             cduct=b1["Cduct"])
        b1.update(B=Bc, H=Hc, slope=Sc, mu_x=mu, mu_y=mu, bh="M19", Theta_hn=b1["Theta_hx"])
    labels = [dict(block=0), dict(block=1), dict(block=2), dict(block=3)]
    circs = []
    if circuits:
        labels[2] = dict(block=2, in_circuit=0, is_wound=1)
        labels[3] = dict(block=3, in_circuit=1)
        circs = [dict(type=0, amps_re=3000.0, amps_im=800.0), dict(type=1, dvolts_re=0.02, dvolts_im=-0.01)]
    if prox is not None:
        blocks[2].update(LamType=3 + prox, Cduct=58.0, WireD=1.0, NStrands=7 if prox in (1, 2) else 1)
        labels[2] = dict(labels[2], is_wound=1, turns=30)
    if external:
        labels.append(dict(block=0, is_external=1))
    tol = 1e-9 * L
    e = -np.ones(p.shape, dtype=np.int32)
    for j in range(3):
        a, b2 = p[:, j], p[:, (j + 1) % 3]
        right = (np.abs(x[a] - L) < tol) & (np.abs(x[b2] - L) < tol)
        bot = (np.abs(y[a]) < tol) & (np.abs(y[b2]) < tol)
        top = (np.abs(y[a] - L) < tol) & (np.abs(y[b2] - L) < tol)
        e[right, j] = 0
        e[top, j] = 1
        e[bot, j] = 2
    lines = [dict(format=0, A0=2e-4, A1=1e-5, phi=20.0),
             dict(format=2, c0=2.0e5, c0_im=3.0e4, c1=0.5, c1_im=-0.2),
             dict(format=1, Mu=1.0, Sig=5.8)]
    m = n + 1
    marker = -np.ones(len(x), dtype=np.int32)
    marker[(m // 2) * m + (2 * m) // 3] = 0
    kw = dict(x=x, y=y, p=p, lbl=lbl, e=e, marker=marker, pbc=None, blocks=blocks, labels=labels, lines=lines,
              points=[dict(J_re=4.0, J_im=1.5)], circuits=circs, precision=precision, length_units=2, coords=0,
              relax=1.0, problem_type=1, frequency=frequency)
    if external:
        kw.update(ext_zo=L / 2, ext_ro=0.8 * L, ext_ri=0.7 * L)
    return kw


def bc_showcase(n: int, anti: bool = False, nonlinear: bool = False, L: float = 10.0):
    """Every static boundary-condition path of Static2D on one square mesh:
    left side prescribed A = (A0 + A1*y)*cos(phi) (BdryFormat 0, static2d.cpp:840-926),
    right side mixed c0/c1 (BdryFormat 2, static2d.cpp:459-480), bottom/top
    periodic or antiperiodic node pairs including the corner nodes
    (static2d.cpp:929-940), a point current and a prescribed point value
    (static2d.cpp:818-838)."""
    kw = magnetostatic(n, nonlinear=nonlinear, L=L)
    x, y, p = kw["x"], kw["y"], kw["p"]
    tol = 1e-9 * L
    m = n + 1
    e = -np.ones(p.shape, dtype=np.int32)
    for j in range(3):
        a, b = p[:, j], p[:, (j + 1) % 3]
        left = (np.abs(x[a]) < tol) & (np.abs(x[b]) < tol)
        right = (np.abs(x[a] - L) < tol) & (np.abs(x[b] - L) < tol)
        bot = (np.abs(y[a]) < tol) & (np.abs(y[b]) < tol)
        top = (np.abs(y[a] - L) < tol) & (np.abs(y[b] - L) < tol)
        e[left, j] = 0
        e[right, j] = 1
        e[bot | top, j] = 2
    kw["e"] = e
    kw["lines"] = [dict(format=0, A0=1e-3, A1=2e-4, A2=0.0, phi=30.0),
                   dict(format=2, c0=3.0, c1=0.5),
                   dict(format=5 if anti else 4)]
    bottom = np.arange(m)                 # row 0
    top = (m - 1) * m + np.arange(m)      # row n
    kw["pbc"] = np.stack([bottom, top, np.full(m, 1 if anti else 0)], 1).astype(np.int32)
    marker = -np.ones(len(x), dtype=np.int32)
    marker[(m // 2) * m + m // 3] = 0     # point current
    marker[(m // 3) * m + (2 * m) // 3] = 1   # fixed A
    kw["marker"] = marker
    kw["points"] = [dict(J_re=5.0), dict(A_re=2e-3)]
    return kw


def bc_chain(n: int, L: float = 10.0):
    """Doubly periodic square: left/right and bottom/top node pairs, so the
    four corner nodes each sit in two pairs and the reference's sequential
    CBigLinProb::Periodicity calls (spars.cpp:421-474) chain.  A prescribed
    point value pins the otherwise floating potential."""
    kw = magnetostatic(n, L=L)
    x, y, p = kw["x"], kw["y"], kw["p"]
    m = n + 1
    kw["e"] = -np.ones(p.shape, dtype=np.int32)
    kw["lines"] = [dict(format=4)]
    rows = np.arange(m)
    lr = np.stack([rows * m, rows * m + (m - 1), np.zeros(m, int)], 1)
    bt = np.stack([np.arange(m), (m - 1) * m + np.arange(m), np.zeros(m, int)], 1)
    kw["pbc"] = np.concatenate([lr, bt]).astype(np.int32)
    marker = -np.ones(len(x), dtype=np.int32)
    marker[(m // 2) * m + m // 2] = 0
    kw["marker"] = marker
    kw["points"] = [dict(A_re=0.0)]
    return kw


def harmonic(n: int, L: float = 10.0, frequency: float = 60.0, precision: float = 1e-8, periodic: bool = False,
             circuits: bool = True, nonlinear: bool = False, prox: Optional[int] = None, anti: bool = False):
    """Keyword arguments of a linear time-harmonic planar problem
    (FSolver::Harmonic2D, cfemm/fsolver/harmonic2d.cpp) on the magnetostatic
    square: laminated lossy steel (lamination thickness with conductivity,
    hysteresis lag), an anisotropic block, a conducting aluminium plate
    (eddy currents), coils with complex current densities, a prescribed-A
    side with phase, a mixed side with complex c0/c1, a small-skin-depth side,
    a complex point current and point value; optionally bottom/top periodic
    pairs and circuits (a wound coil with specified current -> Case 1, the
    plate driven by a specified voltage gradient -> Case 0).  `nonlinear`:
    the steel follows the M-19 curve processed for the frequency
    (GetSlopes(omega): hysteresis lag, lamination eddy currents, fill), which
    starts the reference's successive approximation.  `prox` (wiretype 0-3:
    magnet, stranded, litz, rectangular wire): the coil- region becomes a
    wound copper winding of LamType 3 + prox with AC proximity effects
    (FSolver::GetFillFactor's ProximityMu, harmonic2d.cpp:664-668).  `anti`:
    the bottom/top pairs are antiperiodic (BdryFormat 5) instead."""
    kw = magnetostatic(n, L=L, precision=precision)
    x, y, p = kw["x"], kw["y"], kw["p"]
    tol = 1e-9 * L
    m = n + 1
    e = -np.ones(p.shape, dtype=np.int32)
    for j in range(3):
        a, b = p[:, j], p[:, (j + 1) % 3]
        left = (np.abs(x[a]) < tol) & (np.abs(x[b]) < tol)
        right = (np.abs(x[a] - L) < tol) & (np.abs(x[b] - L) < tol)
        bot = (np.abs(y[a]) < tol) & (np.abs(y[b]) < tol)
        top = (np.abs(y[a] - L) < tol) & (np.abs(y[b] - L) < tol)
        e[left, j] = 0
        e[right, j] = 1
        e[bot, j] = 3 if periodic else 0
        e[top, j] = 3 if periodic else 2
    kw["e"] = e
    kw["frequency"] = frequency
    kw["lines"] = [dict(format=0, A0=1e-3, A1=2e-4, A2=0.0, phi=30.0),
                   dict(format=2, c0=3.0, c0_im=1.0, c1=0.5, c1_im=-0.2),
                   dict(format=1, Mu=1.0, Sig=5.8),
                   dict(format=5 if anti else 4)]
    kw["blocks"] = [
        dict(mu_x=1.0, mu_y=1.0),                                                    # air
        dict(mu_x=800.0, mu_y=800.0, Lam_d=0.35, LamFill=0.96, Cduct=2.0,             # laminated lossy steel
             Theta_hx=12.0, Theta_hy=12.0),
        dict(mu_x=1.0, mu_y=1.0, J_re=2.0, J_im=0.5),                                # coil +
        dict(mu_x=1.0, mu_y=1.0, J_re=-2.0, J_im=-0.5),                              # coil -
        dict(mu_x=1.0, mu_y=1.0, Cduct=35.0),                                        # aluminium plate
        dict(mu_x=50.0, mu_y=5.0, Lam_d=0.5, LamFill=0.9),                           # anisotropic, no conduction
    ]
    if nonlinear:
        from .fsolver import bh_get_slopes_ac
        b1 = kw["blocks"][1]
        Bc, Hc, Sc, mu, _ = bh_get_slopes_ac(*m19_curve(), 2 * np.pi * frequency, lam_type=0,
                                             lam_fill=b1["LamFill"], theta_hn=b1["Theta_hx"], lam_d=b1["Lam_d"],
                                             cduct=b1["Cduct"])
        # (bh / Theta_hn: what a .fem of this problem carries -- the raw curve)
        b1.update(B=Bc, H=Hc, slope=Sc, mu_x=mu, mu_y=mu, bh="M19", Theta_hn=b1["Theta_hx"])
    lbl = kw["lbl"]
    cx = (x[p[:, 0]] + x[p[:, 1]] + x[p[:, 2]]) / (3.0 * L)
    cy = (y[p[:, 0]] + y[p[:, 1]] + y[p[:, 2]]) / (3.0 * L)
    lbl = lbl.copy()
    lbl[(lbl == 0) & (cx > 0.8) & (cx < 0.95) & (cy > 0.1) & (cy < 0.3)] = 5
    kw["lbl"] = lbl
    labels = [dict(block=0), dict(block=1), dict(block=2), dict(block=3), dict(block=4), dict(block=5)]
    if prox is not None:
        kw["blocks"][3].update(LamType=3 + prox, Cduct=58.0, WireD=1.0, NStrands=7 if prox in (1, 2) else 1)
        labels[3] = dict(block=3, is_wound=1, turns=30)
    if circuits:
        labels[2] = dict(block=2, in_circuit=0, is_wound=1)
        labels[4] = dict(block=4, in_circuit=1)
        kw["circuits"] = [dict(type=0, amps_re=3.0, amps_im=1.0), dict(type=1, dvolts_re=0.02, dvolts_im=-0.01)]
    kw["labels"] = labels
    marker = -np.ones(len(x), dtype=np.int32)
    marker[(m // 2) * m + m // 3] = 0
    marker[(m // 3) * m + (2 * m) // 3] = 1
    kw["marker"] = marker
    kw["points"] = [dict(J_re=5.0, J_im=2.0), dict(A_re=2e-3, A_im=1e-3)]
    if periodic:
        bottom = np.arange(m)
        top = (m - 1) * m + np.arange(m)
        kw["pbc"] = np.stack([bottom, top, np.full(m, 1 if anti else 0)], 1).astype(np.int32)
    return kw


def age_rings(inner_nodes, outer_nodes, x, y, total_arc_length: float, fmt: int = 0, inner_angle: float = 0.0,
              outer_angle: float = 0.0, ri: float = 1.0, ro: float = 1.0, center=(0.0, 0.0)) -> dict:
    """One air-gap element as fmesher writes it into the .pbc file
    (cfemm/fmesher/writepoly.cpp:1852-1966): the slice's ring nodes are copied
    round the full circle (antiperiodic copies signed -1 when fmt == 1), placed
    by angle in arc-element units, sorted, and each quadNode k lists the ring
    nodes either side of arc position k with their signs."""
    n = len(inner_nodes)
    dtta = total_arc_length / n
    n0 = int(round(360.0 / dtta))
    n1 = int(round(360.0 / total_arc_length))
    agc = complex(*center)

    def ring(nodes, angle):
        out = []
        for j in range(n1):
            dL = -1.0 if (fmt == 1 and j % 2 != 0) else 1.0
            a = np.exp(1j * (j * total_arc_length + angle) * np.pi / 180.0)
            for nd in nodes:
                z = a * (complex(x[nd], y[nd]) - agc)
                deg = np.angle(z) if z.imag >= 0 else np.angle(z) + 2.0 * np.pi
                out.append((int(nd), deg * 180.0 / np.pi / dtta, dL))
        return sorted(out, key=lambda t: t[1])   # the reference's bubble sort is stable too

    IR, OR = ring(inner_nodes, inner_angle), ring(outer_nodes, outer_angle)
    qn = np.zeros((n + 1, 4), np.int32)
    qw = np.zeros((n + 1, 4))
    for i in range(n + 1):
        p1 = 0 if i == n0 else i
        p0 = p1 - 1 if p1 > 0 else n0 - 1
        qn[i] = (IR[p0][0], IR[p1][0], OR[p0][0], OR[p1][0])
        qw[i] = (IR[p0][2], IR[p1][2], OR[p0][2], OR[p1][2])
    return dict(format=fmt, inner_angle=inner_angle, outer_angle=outer_angle, ri=ri, ro=ro,
                total_arc_length=total_arc_length, inner_shift=IR[0][1], outer_shift=OR[0][1], qn=qn, qw=qw,
                center=center)


def age_motor(n_theta: int = 48, n_r: int = 4, half: bool = False, rotor_angle: float = 0.0,
              nonlinear: bool = False, precision: float = 1e-8, J: float = 3.0, gap: float = 0.1):
    """Two-pole permanent-magnet machine with an air-gap element between rotor
    and stator: a rotor annulus (shaft hole, steel core, x-magnetised ring) and
    a stator annulus (steel with a +-J winding sector), each a structured polar
    mesh with n_theta nodes per full ring; the unmeshed gap between radii
    ri = 2 and ro = 2 + gap is bridged by one AGE.  half: the 0..180 degree
    slice with antiperiodic sides (AGE BdryFormat 1).  rotor_angle rotates the
    rotor through the AGE's InnerAngle (degrees, no remeshing)."""
    r_shaft, ri, ro, r_out = 0.5, 2.0, 2.0 + gap, 4.0
    nt = n_theta // 2 if half else n_theta
    na = nt + 1 if half else nt                 # nodes per ring
    radii_rotor = np.linspace(r_shaft, ri, n_r + 1)
    radii_stator = np.linspace(ro, r_out, n_r + 1)
    dth = 2.0 * np.pi / n_theta
    xs, ys, rings = [], [], []
    for r in list(radii_rotor) + list(radii_stator):
        idx = []
        for m in range(na):
            idx.append(len(xs))
            xs.append(r * np.cos(m * dth))
            ys.append(r * np.sin(m * dth))
        rings.append(idx)
    x, y = np.array(xs), np.array(ys)
    p, lbl, e = [], [], []
    nseg = nt                                  # angular cells per ring pair
    for part, off in ((0, 0), (1, n_r + 1)):
        for j in range(n_r):
            a_r, b_r = rings[off + j], rings[off + j + 1]
            for m in range(nseg):
                m1 = (m + 1) % na
                th = (m + 0.5) * dth * 180.0 / np.pi
                if part == 0:
                    lab = 2 if j == n_r - 1 else 1          # magnet ring outside a steel core
                else:
                    lab = 1
                    if j == 1 and (30.0 < th < 60.0):
                        lab = 3
                    elif j == 1 and (210.0 < th < 240.0):
                        lab = 4
                # counter-clockwise, as Triangle writes them
                for k, tri in enumerate(((a_r[m], b_r[m1], a_r[m1]), (a_r[m], b_r[m], b_r[m1]))):
                    p.append(tri)
                    lbl.append(lab)
                    ee = [-1, -1, -1]
                    # Dirichlet A = 0 on the shaft and the stator's outer rim
                    if part == 0 and j == 0 and k == 0:
                        ee[2] = 0        # edge a_r[m1] -> a_r[m]
                    if part == 1 and j == n_r - 1 and k == 1:
                        ee[1] = 0        # edge b_r[m] -> b_r[m1]
                    e.append(ee)
    p = np.array(p, np.int32)
    blocks = [
        dict(mu_x=1.0, mu_y=1.0),
        dict(mu_x=800.0, mu_y=800.0, LamFill=1.0),
        dict(mu_x=1.049, mu_y=1.049, H_c=979000.0),
        dict(mu_x=1.0, mu_y=1.0, J_re=J),
        dict(mu_x=1.0, mu_y=1.0, J_re=-J),
    ]
    if nonlinear:
        from .fsolver import bh_get_slopes
        Bc, Hc, Sc, mu = bh_get_slopes(*m19_curve(), lam_type=0, lam_fill=0.98)
        blocks[1] = dict(mu_x=mu, mu_y=mu, LamFill=0.98, LamType=0, bh="M19", B=Bc, H=Hc, slope=Sc)
    labels = [dict(block=0), dict(block=1), dict(block=2, mag_dir=0.0), dict(block=3), dict(block=4)]
    inner, outer = rings[n_r], rings[n_r + 1]
    if half:
        inner, outer = inner[:nt], outer[:nt]
    age = age_rings(inner, outer, x, y, 180.0 if half else 360.0, fmt=1 if half else 0,
                    inner_angle=rotor_angle, ri=ri, ro=ro)
    pbc = None
    if half:   # antiperiodic sides: the 0 and 180 degree nodes of every ring
        pbc = np.array([(rg[0], rg[-1], 1) for k, rg in enumerate(rings)], np.int32)
    return dict(x=x, y=y, p=p, lbl=np.array(lbl, np.int32), e=np.array(e, np.int32), marker=None, pbc=pbc,
                blocks=blocks, labels=labels, lines=[dict(format=0)], points=[], circuits=[], precision=precision,
                length_units=2, coords=0, relax=1.0, ages=[age])
