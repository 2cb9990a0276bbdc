"""Independent numpy restatement of the planar Static2D system for full-size checks.

TEST INFRASTRUCTURE.  The C oracle (oracle/static2d_oracle.c) runs the
reference's linked-list matrix and SSOR-PCG, far too slow at the bench sizes
(2M triangles: 86 s just to export its system).  This module restates the same
element loop vectorised over all elements, for the problems xfemm_amd.synth
makes (planar, no circuits, no periodic pairs, isotropic LamType 0):

  * element matrices Mx / My and the area a        static2d.cpp:394-450
  * source J_re a / 3, magnetisation H_c terms      static2d.cpp:470-520
  * linear mu (LamFill) or, given V, the secant permeability of the B-H curve
    1 / (mu0 v(B)), v = H / B by CMMaterialProp::GetBHProps' Hermite
    interpolation (CMaterialProp.cpp:997-1057)      static2d.cpp:560-600
  * Dirichlet A = 0 (BdryFormat 0 edges): rows / columns cleared, diagonal
    kept (CBigLinProb::SetValue, spars.cpp:388-420)

so the device's full-size configs[2] system is compared entry by entry and
solved directly (scipy SuperLU), and the configs[3] Newton answer is checked
as a fixed point of the secant system it converged to.
"""
from __future__ import annotations

import numpy as np
import scipy.sparse as sp

PI = 3.141592653589793238462643383
MUO = 1.2566370614359173e-6
C_ANS = PI * 4.0e-5


def bh_v(block, B):
    """v = H / B of the B-H curve at |B| (vectorised GetBHProps)."""
    Bd, Hd, S = (np.asarray(block.Bdata), np.asarray(block.Hdata), np.asarray(block.slope))
    b = np.abs(B)
    v = np.empty_like(b)
    zero = b == 0
    v[zero] = S[0]
    hi = b > Bd[-1]
    v[hi] = (Hd[-1] + S[-1] * (b[hi] - Bd[-1])) / b[hi]
    mid = ~zero & ~hi
    i = np.clip(np.searchsorted(Bd, b[mid], side="left") - 1, 0, len(Bd) - 2)
    l = Bd[i + 1] - Bd[i]
    z = (b[mid] - Bd[i]) / l
    z2 = z * z
    h = ((1. - 3. * z2 + 2. * z2 * z) * Hd[i] + z * (1. - 2. * z + z2) * l * S[i]
         + z2 * (3. - 2. * z) * Hd[i + 1] + z2 * (z - 1.) * l * S[i + 1])
    v[mid] = h / b[mid]
    return v


def assemble(pr, mesh, V=None):
    """(K csr, b, fixed-node mask) of the planar Static2D system; with V (the
    potential A / c) the nonlinear blocks use the secant permeability at V."""
    x, y, p = mesh.x, mesh.y, mesh.p
    assert not len(mesh.pbc) and not mesh.ages and not pr.circuits
    X, Y = x[p], y[p]
    P = np.stack([Y[:, 1] - Y[:, 2], Y[:, 2] - Y[:, 0], Y[:, 0] - Y[:, 1]], 1)
    Q = np.stack([X[:, 2] - X[:, 1], X[:, 0] - X[:, 2], X[:, 1] - X[:, 0]], 1)
    a = (P[:, 0] * Q[:, 1] - P[:, 1] * Q[:, 0]) / 2.
    Kf = -1. / (4. * a)
    blk = mesh.blk
    mu_x = np.array([b.mu_x for b in pr.blocks])[blk]
    mu_y = np.array([b.mu_y for b in pr.blocks])[blk]
    fill = np.array([b.LamFill for b in pr.blocks])[blk]
    assert all(b.LamType == 0 for b in pr.blocks)
    mu1 = mu_x * fill + (1. - fill)
    mu2 = mu_y * fill + (1. - fill)
    if V is not None:
        for k, bp in enumerate(pr.blocks):
            if not bp.BHpoints:
                continue
            sel = np.where(blk == k)[0]
            Vn = V[p[sel]]
            B1 = (Vn * Q[sel]).sum(1)
            B2 = (Vn * P[sel]).sum(1)
            B = C_ANS * np.sqrt(B1 * B1 + B2 * B2) / (0.02 * a[sel])
            mu = 1. / (MUO * bh_v(bp, B))
            mu1[sel] = mu
            mu2[sel] = mu
    # Me = Mx / mu2 + My / mu1, added as -Me (the reference's sign)
    Me = Kf[:, None, None] * (P[:, :, None] * P[:, None, :] / mu2[:, None, None]
                              + Q[:, :, None] * Q[:, None, :] / mu1[:, None, None])
    J = np.array([b.J_re for b in pr.blocks])[blk]
    Hc = np.array([b.H_c for b in pr.blocks])[blk]
    t = np.array([lb.MagDir for lb in pr.labels])[mesh.lbl] * PI / 180.
    be = np.repeat((-J * a / 3.)[:, None], 3, 1)
    for j in range(3):
        k = (j + 1) % 3
        Km = 0.0001 * Hc * (np.cos(t) * (X[:, k] - X[:, j]) + np.sin(t) * (Y[:, k] - Y[:, j])) / 2.
        be[:, j] += Km
        be[:, k] += Km
    n = len(x)
    rows = np.repeat(p, 3, axis=1).reshape(-1)
    cols = np.tile(p, (1, 3)).reshape(-1)
    K = sp.coo_matrix((-Me.reshape(-1), (rows, cols)), shape=(n, n)).tocsr()
    b = -np.bincount(p.reshape(-1), weights=be.reshape(-1), minlength=n)
    fixed = np.zeros(n, bool)
    fmt = np.array([ln.BdryFormat for ln in pr.bdrys] + [-1])
    for j in range(3):
        e = mesh.e[:, j]
        on = (e >= 0) & (fmt[np.where(e >= 0, e, -1)] == 0)
        fixed[p[on, j]] = True
        fixed[p[on, (j + 1) % 3]] = True
    assert all(ln.A0 == 0 and ln.A1 == 0 and ln.A2 == 0 for ln in pr.bdrys if ln.BdryFormat == 0)
    if fixed.any():
        D = sp.diags((~fixed).astype(float))
        diag = K.diagonal()
        K = (D @ K @ D + sp.diags(np.where(fixed, diag, 0.))).tocsr()
        b = np.where(fixed, 0., b)
    K.eliminate_zeros()
    return K, b, fixed
