"""MIS-2 round tail on the configs[2] hierarchy (numpy prototype): undecided
rows after every round, per level, and the PCG iteration count when the MIS
stops after K rounds and the rows still undecided become roots of their own.
usage: python tools/lab/mis_tail.py [N=1000] [K...]   (lab tool)"""
import sys, os
import numpy as np
import scipy.sparse as sp
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import amg_proto as ap

CUT = [None]
LOG = []


def mis2_cut(S):
    n = S.shape[0]
    deg = np.diff(S.indptr)
    iso = deg == 0
    state = np.where(iso, 0, 1).astype(np.int64)
    r = ap.hash32(np.arange(n)).astype(np.int64)
    idx = np.arange(n, dtype=np.int64)
    G = (S + sp.identity(n, format="csr")).tocsr()
    rows = np.repeat(np.arange(n), np.diff(G.indptr))
    hist = []
    rounds = 0
    while (state == 1).any():
        if CUT[0] is not None and rounds >= CUT[0]:
            state[state == 1] = 2      # leftovers: roots of their own
            break
        rounds += 1
        key = (state << 52) | (r << 20) | idx
        T = key.copy()
        for _ in range(2):
            m = T.copy()
            np.maximum.at(m, rows, T[G.indices])
            T = m
        und = state == 1
        win = und & ((T & ((1 << 20) - 1)) == idx)
        lose = und & ((T >> 52) == 2)
        state[win] = 2
        state[lose & ~win] = 0
        hist.append(int((state == 1).sum()))
    LOG.append((n, hist))
    roots = np.flatnonzero(state == 2)
    agg = -np.ones(n, np.int64)
    agg[roots] = np.arange(len(roots))
    srows = np.repeat(np.arange(n), np.diff(S.indptr))
    for _ in range(2):
        cand = np.where(agg[S.indices] >= 0, (r[S.indices] << 20) | S.indices, -1)
        best = -np.ones(n, np.int64)
        np.maximum.at(best, srows, cand)
        sel = (agg < 0) & (best >= 0) & ~iso
        src = best[sel] & ((1 << 20) - 1)
        agg_new = agg.copy()
        agg_new[sel] = agg[src]
        agg = agg_new
    return agg, len(roots), rounds


ap.mis2_aggregate = mis2_cut

if __name__ == "__main__":
    from oracle import oracle
    from util import synth_to_oracle
    from xfemm_amd import synth
    N = int(sys.argv[1]) if len(sys.argv) > 1 else 1000
    kw = synth.magnetostatic(N, nonlinear=False)
    pr, mesh, _ = synth_to_oracle(kw)
    A, b = oracle.system(pr, mesh)
    print("N", A.shape[0], "nnz", A.nnz, flush=True)
    for K in [None] + [int(k) for k in sys.argv[2:]]:
        CUT[0] = K
        LOG.clear()
        M = ap.AMG(A, theta=0.08, coarse=2048)
        x, it = ap.pcg(A, b, M.vcycle)
        print("cut", K, "iters", it, "levels", [L["A"].shape[0] for L in M.levels], M.Ac.shape[0], flush=True)
        for n, h in LOG:
            print("   n %d undecided per round %s" % (n, h), flush=True)
