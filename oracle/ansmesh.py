"""Rebuild a solvable mesh from a reference .ans golden file -- TEST INFRASTRUCTURE.

The reference's golden solutions (cfemm/fsolver/test/Temp.ans.check and
Temp1.ans.check) were written by the reference fsolver in the FEMM 4.0 layout
(static2d.cpp:1079-1148 minus the marker / PBC columns): they carry the solved
mesh (node x, y, A; element nodes and block label) but not the boundary data
fmesher derived from the .fem geometry.  This module re-derives that boundary
data geometrically from the .fem [NumPoints]/[NumSegments] tables exactly as
fmesher's output would carry it:
  * element edge markers e[j] for every mesh edge lying on a .fem segment with
    a boundary property (what FSolver::LoadMesh reads from .edge, fsolver.cpp:659-697)
  * (anti)periodic node pairs for segments sharing a periodic boundary
    property (what LoadMesh reads from .pbc, fsolver.cpp:394-415)
  * node point-property markers for .fem points carrying a point property.
"""
from __future__ import annotations

import numpy as np

from . import femfile


def _fem_geometry(path):
    with open(path) as fh:
        lines = fh.read().splitlines()
    pts, segs = [], []
    i = 0
    while i < len(lines):
        s = lines[i].strip().lower()
        if s.startswith("[numpoints]"):
            n = int(s.split("=")[1])
            for j in range(n):
                f = lines[i + 1 + j].split()
                pts.append((float(f[0]), float(f[1]), int(f[2])))
            i += n
        elif s.startswith("[numsegments]"):
            n = int(s.split("=")[1])
            for j in range(n):
                f = lines[i + 1 + j].split()
                segs.append((int(f[0]), int(f[1]), int(f[3])))
            i += n
        elif s.startswith("[numarcsegments]"):
            if int(s.split("=")[1]) != 0:
                raise NotImplementedError("arc segments")
        i += 1
    return pts, segs


def _on_segment(x, y, x0, y0, x1, y1, tol):
    dx, dy = x1 - x0, y1 - y0
    L2 = dx * dx + dy * dy
    t = ((x - x0) * dx + (y - y0) * dy) / L2
    px, py = x0 + t * dx, y0 + t * dy
    d = np.hypot(x - px, y - py)
    ok = (d < tol) & (t > -1e-9) & (t < 1 + 1e-9)
    return ok, t


def mesh_from_ans(fem_path: str, ans_path: str, pr: femfile.FemProblem):
    sol = femfile.read_ans(ans_path)
    pts, segs = _fem_geometry(fem_path)
    conv = 100.0 * femfile.LENGTH_CONV_METERS[pr.LengthUnits]
    xs, ys = sol.x, sol.y
    scale = max(np.ptp(xs), np.ptp(ys))
    tol = 1e-9 * scale
    nn = len(xs)
    marker = -np.ones(nn, dtype=np.int32)
    for (px, py, pm) in pts:
        if pm > 0:
            k = np.nonzero(np.hypot(xs - px, ys - py) < tol)[0]
            marker[k] = pm - 1
    ne = len(sol.lbl)
    e = -np.ones((ne, 3), dtype=np.int32)
    pbc_pairs = []
    by_prop = {}
    for (a, b, m) in segs:
        if m <= 0:
            continue
        x0, y0, _ = pts[a]
        x1, y1, _ = pts[b]
        on, t = _on_segment(xs, ys, x0, y0, x1, y1, tol)
        p = sol.p
        for j in range(3):
            k = (j + 1) % 3
            hit = on[p[:, j]] & on[p[:, k]]
            e[hit, j] = m - 1
        by_prop.setdefault(m - 1, []).append((np.nonzero(on)[0], t[on]))
    for prop, lst in by_prop.items():
        fmt = pr.bdrys[prop].BdryFormat
        if fmt not in (4, 5):
            continue
        if len(lst) != 2:
            raise ValueError("periodic property %d on %d segments" % (prop, len(lst)))
        (n1, t1), (n2, t2) = lst
        o1, o2 = np.argsort(t1), np.argsort(t2)
        n1, t1, n2, t2 = n1[o1], t1[o1], n2[o2], t2[o2]
        if len(n1) != len(n2):
            raise ValueError("non-conforming periodic boundary")
        if not np.allclose(t1, t2, atol=1e-7):
            n2, t2 = n2[::-1], 1 - t2[::-1]
            if not np.allclose(t1, t2, atol=1e-7):
                raise ValueError("cannot pair periodic nodes")
        for i1, i2 in zip(n1, n2):
            pbc_pairs.append((int(i1), int(i2), 0 if fmt == 4 else 1))
    pbc = np.array(sorted(set(pbc_pairs)), dtype=np.int32).reshape(-1, 3)
    lbl = sol.lbl.astype(np.int32)
    blk = np.array([pr.labels[l].BlockType for l in lbl], dtype=np.int32)
    mesh = femfile.Mesh(x=xs * conv, y=ys * conv, marker=marker, p=sol.p.astype(np.int32), e=e,
                        lbl=lbl, blk=blk, pbc=pbc, bandwidth=0, edges=None)
    return mesh, sol
