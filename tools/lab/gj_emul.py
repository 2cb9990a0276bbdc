"""numpy emulation of the device dense-coarsest inverse (unit-diagonal scaling,
64-wide blocked Gauss-Jordan, 4-pivot diagonal steps with the scalar null
fallback) on a pure-Neumann operator: is the null direction caught?"""
import sys

import numpy as np
import scipy.sparse as sp


def laplace_random(n, seed):
    rng = np.random.default_rng(seed)
    N = n * n
    idx = np.arange(N).reshape(n, n)
    rows, cols, vals = [], [], []
    diag = np.zeros(N)
    for a, b in [(idx[:, :-1], idx[:, 1:]), (idx[:-1, :], idx[1:, :])]:
        a = a.ravel()
        b = b.ravel()
        c = np.exp(rng.uniform(-3, 3, len(a)))
        rows += [a, b]
        cols += [b, a]
        vals += [-c, -c]
        np.add.at(diag, a, c)
        np.add.at(diag, b, c)
    rows.append(np.arange(N))
    cols.append(np.arange(N))
    vals.append(diag)
    return sp.csr_matrix((np.concatenate(vals), (np.concatenate(rows), np.concatenate(cols))), shape=(N, N))


def emulate(A, thr):
    n = A.shape[0]
    s = 1 / np.sqrt(np.diag(A))
    S = A * s[:, None] * s[None, :]

    def scalar_gj(a, p):
        piv = a[p, p]
        if not abs(piv) > thr:
            a[p, :] = 0
            a[:, p] = 0
            return
        ip = 1 / piv
        r = a[p, :] * ip
        r[p] = 1 + ip
        c = a[:, p].copy()
        c[p] -= 1
        a -= np.outer(c, r)

    def diag_inv(Bk):
        a = Bk.copy()
        for p0 in range(0, 64, 4):
            P = slice(p0, p0 + 4)
            Dv = a[P, P].copy()
            ok = True
            for q in range(4):
                piv = Dv[q, q]
                ok = ok and abs(piv) > thr
                ip = 1 / piv
                Dv[q, q] = 1
                Dv[q, :] *= ip
                for s2 in range(4):
                    if s2 != q:
                        f = Dv[s2, q]
                        Dv[s2, q] = 0
                        Dv[s2, :] -= f * Dv[q, :]
            if not ok:
                for p in range(p0, p0 + 4):
                    scalar_gj(a, p)
                continue
            R = Dv @ a[P, :]
            for t in range(4):
                R[:, p0 + t] = np.eye(4)[:, t] + Dv[:, t]
            C = a[:, P].copy()
            a -= C @ R
            a[P, :] += R
        return a

    ld = (n + 63) // 64 * 64
    Mp = np.eye(ld)
    Mp[:n, :n] = S
    nbk = ld // 64
    for k in range(nbk):
        K = slice(64 * k, 64 * k + 64)
        D = diag_inv(Mp[K, K])
        C = Mp[:, K].copy()
        T = D @ Mp[K, :]
        Mp[K, :] = T
        for i in range(nbk):
            if i != k:
                I = slice(64 * i, 64 * i + 64)
                Mp[I, :] -= C[I, :] @ T
                Mp[I, K] = -C[I, :] @ D
        Mp[K, K] = D
    return Mp[:n, :n] * s[:, None] * s[None, :]


A = laplace_random(30, 11).toarray()
b = np.random.default_rng(5).standard_normal(A.shape[0])
b -= b.mean()
for thr in [float(a) for a in sys.argv[1:]] or [1e-13, 1e-10]:
    Mi = emulate(A, thr)
    x = Mi @ b
    print("thr %g: resid %.3e max|Minv| %.3e" % (thr, np.linalg.norm(A @ x - b) / np.linalg.norm(b), np.abs(Mi).max()))
