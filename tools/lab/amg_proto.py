"""CPU prototype (scipy) of the smoothed-aggregation AMG planned for the GPU
PCG: parallel MIS-2 aggregation, Jacobi-smoothed prolongator, Galerkin
coarse operators, V-cycle with damped Jacobi / Chebyshev smoothing.  Used to
pick parameters (strength threshold, smoother, cycle) by PCG iteration count
on the synthetic magnetostatic matrices.  Lab tool, not product code."""
import sys, os, time
import numpy as np
import scipy.sparse as sp
import scipy.sparse.linalg as spla
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT); sys.path.insert(0, os.path.join(ROOT, "tests"))


def hash32(x):
    x = x.astype(np.uint32)
    x = ((x >> 16) ^ x) * np.uint32(0x45d9f3b)
    x = ((x >> 16) ^ x) * np.uint32(0x45d9f3b)
    return (x >> 16) ^ x


def strength(A, theta):
    A = A.tocoo()
    d = np.abs(A.diagonal())
    off = A.row != A.col
    keep = off & (np.abs(A.data) > theta * np.sqrt(d[A.row] * d[A.col])) & (A.data != 0)
    n = A.shape[0]
    return sp.csr_matrix((np.ones(keep.sum()), (A.row[keep], A.col[keep])), shape=(n, n))


def mis2_aggregate(S):
    n = S.shape[0]
    deg = np.diff(S.indptr)
    iso = deg == 0
    state = np.where(iso, 0, 1).astype(np.int64)        # 2 in, 1 undecided, 0 out
    r = hash32(np.arange(n)).astype(np.int64)
    idx = np.arange(n, dtype=np.int64)
    rounds = 0
    G = (S + sp.identity(n, format="csr")).tocsr()
    while (state == 1).any():
        rounds += 1
        key = (state << 52) | (r << 20) | idx                # n < 2^20 in the proto
        assert n < (1 << 20)
        T = key.copy()
        for _ in range(2):
            # T_i = max over neighbourhood
            rows = np.repeat(np.arange(n), np.diff(G.indptr))
            m = T.copy()
            np.maximum.at(m, rows, T[G.indices])
            T = m
        und = state == 1
        win = und & ((T & ((1 << 20) - 1)) == idx)
        lose = und & ((T >> 52) == 2)
        state[win] = 2
        state[lose & ~win] = 0
    roots = np.flatnonzero(state == 2)
    agg = -np.ones(n, np.int64)
    agg[roots] = np.arange(len(roots))
    # distance 1: join the max-key root neighbour
    rows = np.repeat(np.arange(n), np.diff(S.indptr))
    for _ in range(2):
        cand = np.where(agg[S.indices] >= 0, (r[S.indices] << 20) | S.indices, -1)
        best = -np.ones(n, np.int64)
        np.maximum.at(best, rows, cand)
        sel = (agg < 0) & (best >= 0) & ~iso
        src = best[sel] & ((1 << 20) - 1)
        agg_new = agg.copy()
        agg_new[sel] = agg[src]
        agg = agg_new
    assert ((agg >= 0) | iso).all(), "unaggregated non-isolated nodes"
    return agg, len(roots), rounds


def build_level(A, theta, smooth_p=True):
    n = A.shape[0]
    S = strength(A, theta)
    agg, nc, rounds = mis2_aggregate(S)
    rows = np.flatnonzero(agg >= 0)
    T = sp.csr_matrix((np.ones(len(rows)), (rows, agg[rows])), shape=(n, nc))
    if smooth_p:
        # filtered A: weak off-diagonals lumped onto the diagonal
        Ac = A.tocoo()
        off = Ac.row != Ac.col
        strong = S.tocoo()
        sk = set()
        Sm = (S != 0).astype(np.int8)
        keepmask = np.asarray(Sm[Ac.row, Ac.col]).ravel().astype(bool) | ~off
        AF = sp.csr_matrix((Ac.data * keepmask, (Ac.row, Ac.col)), shape=(n, n))
        lump = np.asarray(A.sum(axis=1)).ravel() - np.asarray(AF.sum(axis=1)).ravel()
        AF = AF + sp.diags(lump)
        D = AF.diagonal()
        Dinv = 1.0 / D
        DA = sp.diags(Dinv) @ AF
        rho = gershgorin(DA)
        w = 4.0 / 3.0 / rho
        P = (T - w * (DA @ T)).tocsr()
    else:
        P = T
    Ac = (P.T @ A @ P).tocsr()
    return P, Ac, rounds


def gershgorin(DA):
    return np.abs(DA).sum(axis=1).max()


def power_rho(A, Dinv, its=15):
    x = hash32(np.arange(A.shape[0])).astype(float) / 2**32 + 0.1
    for _ in range(its):
        y = Dinv * (A @ x)
        lam = np.linalg.norm(y) / np.linalg.norm(x)
        x = y / np.linalg.norm(y)
    return lam


class AMG:
    def __init__(self, A, theta=0.08, coarse=400, smoother="jacobi", deg=2, smooth_p=True):
        self.levels = []
        t0 = time.time()
        while A.shape[0] > coarse:
            Dinv = 1.0 / A.diagonal()
            rho = power_rho(A, Dinv)
            P, Ac, rounds = build_level(A, theta, smooth_p)
            self.levels.append(dict(A=A, P=P, Dinv=Dinv, rho=rho, rounds=rounds))
            A = Ac
            if len(self.levels) > 25:
                break
        self.Ac = A.toarray()
        self.setup_s = time.time() - t0
        self.smoother, self.deg = smoother, deg

    def info(self):
        s = []
        for L in self.levels:
            A = L["A"]
            s.append("n=%d nnz/row=%.1f rho=%.2f rounds=%d" % (A.shape[0], A.nnz / A.shape[0], L["rho"], L["rounds"]))
        s.append("coarse n=%d" % self.Ac.shape[0])
        return "\n".join(s)

    def smooth(self, L, x, b):
        A, Dinv, rho = L["A"], L["Dinv"], L["rho"]
        if self.smoother == "jacobi":
            w = 1.0 / rho  # damped (4/3 too aggressive for symmetric V)
            for _ in range(self.deg):
                x = x + w * Dinv * (b - A @ x)
            return x
        # Chebyshev on D^-1 A over [rho/ratio, 1.1 rho]
        lmax = 1.1 * rho
        lmin = lmax / 30.0
        theta = 0.5 * (lmax + lmin)
        delta = 0.5 * (lmax - lmin)
        sigma = theta / delta
        rho_k = 1.0 / sigma
        r = Dinv * (b - A @ x)
        d = r / theta
        for k in range(self.deg):
            x = x + d
            if k == self.deg - 1:
                break
            r = r - Dinv * (A @ d)
            rho_n = 1.0 / (2 * sigma - rho_k)
            d = rho_n * rho_k * d + 2 * rho_n / delta * r
            rho_k = rho_n
        return x

    def vcycle(self, b, l=0):
        if l == len(self.levels):
            return np.linalg.lstsq(self.Ac, b, rcond=None)[0] if False else np.linalg.solve(self.Ac, b)
        L = self.levels[l]
        x = self.smooth(L, np.zeros_like(b), b)
        r = b - L["A"] @ x
        x = x + L["P"] @ self.vcycle(L["P"].T @ r, l + 1)
        x = self.smooth(L, x, b)
        return x


def pcg(A, b, M, tol=1e-8, maxit=5000):
    x = np.zeros_like(b)
    r = b.copy()
    z = M(r)
    res_o = z @ b
    p = z.copy()
    g = z @ r
    for it in range(maxit):
        Ap = A @ p
        a = g / (p @ Ap)
        x += a * p
        r -= a * Ap
        z = M(r)
        gn = z @ r
        if np.sqrt(gn / res_o) <= tol:
            return x, it + 1
        p = z + gn / g * p
        g = gn
    return x, maxit


if __name__ == "__main__":
    from oracle import oracle
    from util import synth_to_oracle
    from xfemm_amd import synth
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 300
    kw = synth.magnetostatic(n, nonlinear=False)
    pr, mesh, _ = synth_to_oracle(kw)
    A, b = oracle.system(pr, mesh)
    print("N", A.shape[0], "nnz", A.nnz)
    xd = spla.spsolve(A.tocsc(), b)
    D = A.diagonal()
    x, it = pcg(A, b, lambda r: r / D)
    print("jacobi iters", it, "err", np.abs(x - xd).max() / np.abs(xd).max())
    for theta in [0.02, 0.08, 0.25]:
        for sm, deg in [("jacobi", 1), ("jacobi", 2), ("cheb", 2), ("cheb", 3)]:
            M = AMG(A, theta=theta, smoother=sm, deg=deg)
            x, it = pcg(A, b, M.vcycle)
            print("theta %.2f %s(%d): levels %d iters %d err %.2e  setup %.1fs" % (
                theta, sm, deg, len(M.levels), it, np.abs(x - xd).max() / np.abs(xd).max(), M.setup_s))
    print(M.info())
