"""Flux density at a point, as the reference post-processor gives it -- TEST
INFRASTRUCTURE ONLY (used by tests/test_gpu_antiperiodic_flux.py).

A restatement of what femmcli's mo_getpointvalues(x, y) returns for Bx, By on
a planar magnetostatic .ans (cfemm/fpproc/fpproc.cpp, temudschin/xfemm
@ 2025-02-04), real parts only (Frequency 0):

  * the containing element: FPProc::InTriangle (fpproc.cpp:2180-2235), which
    starts at the element found by the previous call and walks outwards
    (hi = k+1, lo = k-1, ...), with the circumradius pre-test and
    FPProc::InTriangleTest (:3387-3424);
  * element flux density: FPProc::GetElementB, planar (:2970-3003),
    B1 = sum A c / (da L), B2 = -sum A b / (da L);
  * Smooth = true (:100): FPProc::GetPointB (:2669-2702) interpolates nodal
    values b1, b2 that FPProc::GetNodalB (:2704-2967) builds by the patch
    method -- centroid-distance-weighted element values around a node away
    from material interfaces, the interface rule (tangential B from the
    element, normal B from the A difference along the interface side) next to
    one, and the "too sharp a corner" punt.
"""
from __future__ import annotations

import math

import numpy as np

LENGTH_CONV = [0.0254, 0.001, 0.01, 1.0, 2.54e-5, 1.0e-6]   # fpproc.cpp:106-112 (meters per unit)


def _cabs(re: float, im: float) -> float:   # femmcomplex.cpp:749-757
    if re == 0 and im == 0:
        return 0.0
    if abs(re) > abs(im):
        return abs(re) * math.sqrt(1. + (im / re) * (im / re))
    return abs(im) * math.sqrt(1. + (re / im) * (re / im))


class FluxPost:
    """Post-processor state of one solved planar static problem: nodes x, y
    (drawing units), A (Wb/m), elements p (0-based), label index per
    element, per-label block index and MagDir, per-block (mu_x, mu_y, H_c)."""

    def __init__(self, x, y, A, p, lbl, label_block, label_magdir, block_props, length_units: int):
        self.x = np.asarray(x, float)
        self.y = np.asarray(y, float)
        self.A = np.asarray(A, float)
        self.p = np.asarray(p, np.int64).reshape(-1, 3)
        self.lbl = np.asarray(lbl, np.int64)
        self.blk = np.asarray(label_block, np.int64)[self.lbl]
        self.magdir = np.asarray(label_magdir, float)[self.lbl]
        self.bprops = [tuple(b) for b in block_props]
        self.L = LENGTH_CONV[length_units]
        X, Y, p = self.x, self.y, self.p
        # FPProc::Ctr (:3426-3438) and rsqr (:1622-1630)
        cx = X[p[:, 0]] / 3. + X[p[:, 1]] / 3. + X[p[:, 2]] / 3.
        cy = Y[p[:, 0]] / 3. + Y[p[:, 1]] / 3. + Y[p[:, 2]] / 3.
        self.cx, self.cy = cx, cy
        self.rsqr = np.max(np.stack([(X[p[:, j]] - cx) ** 2 + (Y[p[:, j]] - cy) ** 2 for j in range(3)]), axis=0)
        # GetElementB, planar (:2976-2995)
        b = np.stack([Y[p[:, 1]] - Y[p[:, 2]], Y[p[:, 2]] - Y[p[:, 0]], Y[p[:, 0]] - Y[p[:, 1]]], 1)
        c = np.stack([X[p[:, 2]] - X[p[:, 1]], X[p[:, 0]] - X[p[:, 2]], X[p[:, 1]] - X[p[:, 0]]], 1)
        da = b[:, 0] * c[:, 1] - b[:, 1] * c[:, 0]
        Ae = self.A[p]
        B1 = np.zeros(len(p))
        B2 = np.zeros(len(p))
        for i in range(3):
            B1 = B1 + Ae[:, i] * c[:, i] / (da * self.L)
            B2 = B2 - Ae[:, i] * b[:, i] / (da * self.L)
        self.B1, self.B2 = B1, B2
        # ConList: the elements around each node, ascending (:1766-1786)
        order = np.argsort(p.reshape(-1), kind="stable")
        self.con_elem = order // 3
        self.con_ptr = np.concatenate([[0], np.cumsum(np.bincount(p.reshape(-1), minlength=len(X)))])
        self.k = 0   # InTriangle's static start element

    def conlist(self, node: int):
        return self.con_elem[self.con_ptr[node]:self.con_ptr[node + 1]]

    def in_triangle_test(self, x: float, y: float, i: int) -> bool:   # :3387-3424
        X, Y, p = self.x, self.y, self.p[i]
        for j in range(3):
            k = (j + 1) % 3
            if p[k] > p[j]:
                z = (X[p[k]] - X[p[j]]) * (y - Y[p[j]]) - (Y[p[k]] - Y[p[j]]) * (x - X[p[j]])
                if z < 0:
                    return False
            else:
                z = (X[p[j]] - X[p[k]]) * (y - Y[p[k]]) - (Y[p[j]] - Y[p[k]]) * (x - X[p[k]])
                if z > 0:
                    return False
        return True

    def in_triangle(self, x: float, y: float) -> int:   # :2180-2235
        sz = len(self.p)
        if self.k < 0 or self.k >= sz:
            self.k = 0
        if self.in_triangle_test(x, y, self.k):
            return self.k
        # candidates by the circumradius pre-test, then the reference's visiting order
        z = (self.cx - x) ** 2 + (self.cy - y) ** 2
        cand = np.where(z <= self.rsqr)[0]
        k = self.k
        best, best_rank = -1, None
        for c in cand:
            c = int(c)
            if c == k:
                continue
            # iteration t of the loop visits hi = k + 1 + t, then lo = k - 1 - t
            niter = (sz + 1) // 2
            ranks = [2 * t for t in [(c - k) % sz - 1] if t < niter] + \
                    [2 * t + 1 for t in [(k - c) % sz - 1] if t < niter]
            if not ranks:
                continue
            rank = min(ranks)
            if (best_rank is None or rank < best_rank) and self.in_triangle_test(x, y, c):
                best, best_rank = c, rank
        if best >= 0:
            self.k = best
        return best

    def _same_material(self, e: int, m: int) -> bool:   # the m++ test of :2723-2737 (Frequency 0)
        if self.lbl[e] == self.lbl[m]:
            return True
        be, bm = self.bprops[self.blk[e]], self.bprops[self.blk[m]]
        if be == bm and self.magdir[e] == self.magdir[m]:
            return True
        return self.blk[e] == self.blk[m] and self.magdir[e] == self.magdir[m]

    def _interface(self, e: int, k: int, pt: int):
        """Contribution of the interface side k-pt seen from element e (:2800-2826)."""
        X, Y = self.x, self.y
        tnx, tny = X[pt] - X[k], Y[pt] - Y[k]
        atn = _cabs(tnx, tny)
        bn = (self.A[pt] - self.A[k]) / (atn * self.L)
        z = 0.5 / atn
        tnx, tny = tnx / atn, tny / atn
        bt = self.B1[e] * tnx + self.B2[e] * tny
        return z, z * tnx * bt + z * tny * bn, z * tny * bt - z * tnx * bn, (tnx, tny)

    def _next(self, e: int, k: int, ccw: bool):
        """The side of e at node k (ccw or cw) and the element across it (-1: none)."""
        pe = [int(v) for v in self.p[e]]
        pt = pe[(pe.index(k) + (-1 if ccw else 1)) % 3]
        nxt = -1
        for m in self.conlist(k):
            if m != e and pt in self.p[m]:
                nxt = int(m)
        return pt, nxt

    def nodal_b(self, elm: int):
        """GetNodalB (:2704-2967) for the three nodes of element elm."""
        X, Y = self.x, self.y
        out = []
        for i in range(3):
            k = int(self.p[elm][i])
            con = self.conlist(k)
            m = sum(1 for e in con if self._same_material(elm, int(e)))
            if m == len(con):   # normal smoothing away from interfaces (:2740-2753)
                R = b1 = b2 = 0.0
                for e in con:
                    z = 1. / _cabs(X[k] - self.cx[e], Y[k] - self.cy[e])
                    R += z
                    b1 += z * self.B1[e]
                    b2 += z * self.B2[e]
                out.append((b1 / R, b2 / R))
                continue
            R = b1 = b2 = 0.0
            v1 = v2 = (0.0, 0.0)
            e = elm
            for _ in range(len(con)):   # scan ccw for an interface (:2762-2830)
                pt, nxt = self._next(e, k, True)
                if nxt == -1:           # the special-case punt
                    b1, b2 = self.B1[e], self.B2[e]
                    v1 = v2 = (1.0, 0.0)
                    break
                if self.lbl[elm] != self.lbl[nxt]:
                    z, d1, d2, v1 = self._interface(e, k, pt)
                    R += z
                    b1 += d1
                    b2 += d2
                    break
                e = nxt
            if v2 == (0.0, 0.0):        # scan cw (:2833-2891), skipped after a punt
                e = elm
                for _ in range(len(con)):
                    pt, nxt = self._next(e, k, False)
                    if nxt == -1:
                        b1, b2 = self.B1[e], self.B2[e]
                        v1 = v2 = (1.0, 0.0)
                        break
                    if self.lbl[elm] != self.lbl[nxt]:
                        z, d1, d2, v2 = self._interface(e, k, pt)
                        R += z
                        b1 += d1
                        b2 += d2
                        break
                    e = nxt
                b1, b2 = b1 / R, b2 / R
            flag = (_cabs(*v1) < 0.9 or _cabs(*v2) < 0.9) or (-v1[0] * v2[0] - v1[1] * v2[1]) > 0.985
            if not flag:   # too sharp a corner: punt (:2893-2932), real parts
                bn = 0.0
                for e in con:
                    if self.lbl[elm] == self.lbl[e]:
                        bn = max(bn, math.sqrt(self.B1[e] ** 2 + self.B2[e] ** 2))
                R = math.sqrt(self.B1[elm] ** 2 + self.B2[elm] ** 2)
                if R != 0:
                    b1, b2 = bn / R * self.B1[elm], bn / R * self.B2[elm]
                else:
                    b1 = b2 = 0.0
            out.append((b1, b2))
        return out

    def point_b(self, x: float, y: float):
        """(Bx, By) in T as mo_getpointvalues returns them, or None outside the mesh."""
        e = self.in_triangle(x, y)
        if e < 0:
            return None
        X, Y = self.x, self.y
        n = self.p[e]
        a = [X[n[1]] * Y[n[2]] - X[n[2]] * Y[n[1]], X[n[2]] * Y[n[0]] - X[n[0]] * Y[n[2]],
             X[n[0]] * Y[n[1]] - X[n[1]] * Y[n[0]]]
        b = [Y[n[1]] - Y[n[2]], Y[n[2]] - Y[n[0]], Y[n[0]] - Y[n[1]]]
        c = [X[n[2]] - X[n[1]], X[n[0]] - X[n[2]], X[n[1]] - X[n[0]]]
        da = b[0] * c[1] - b[1] * c[0]
        nb = self.nodal_b(e)
        B1 = B2 = 0.0
        for i in range(3):
            w = (a[i] + b[i] * x + c[i] * y) / da
            B1 += nb[i][0] * w
            B2 += nb[i][1] * w
        return B1, B2
