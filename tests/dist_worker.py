"""Worker of tests/test_sharded_cpu.py: one rank of the sharded PCG, restated
on the CPU over torch.distributed (gloo).

It runs the algorithm of the GPU path (xfemm_amd/csrc/xfk_pcg.hip with the
sharded driver in xfk_api.hip) on the oracle's assembled system: the rank
owns the rows of its xfk_partition_plan block, receives each halo range as one
contiguous slice of a peer's vector, and all-reduces the inner-product partials
once per iteration (Chronopoulos-Gear PCG, Jacobi preconditioner, stopping test
sqrt(z.r / z0.b) <= Precision as in CBigLinProb::PCGSolve, spars.cpp:238-316).
"""
import os

import numpy as np
import scipy.sparse as sp
import torch
import torch.distributed as dist


def _exchange(u, plan):
    """Fill the halo slices of u from the peers' owned slices (gloo p2p)."""
    reqs = []
    bufs = []
    for peer, off, ln, _g0 in plan["recv"]:
        b = torch.empty(int(ln), dtype=torch.float64)
        bufs.append((off, ln, b))
        reqs.append(dist.irecv(b, src=int(peer)))
    for peer, off, ln, _g0 in plan["send"]:
        reqs.append(dist.isend(torch.from_numpy(np.ascontiguousarray(u[off:off + ln])), dst=int(peer)))
    for r in reqs:
        r.wait()
    for off, ln, b in bufs:
        u[off:off + ln] = b.numpy()


def _allreduce(v):
    t = torch.tensor(v, dtype=torch.float64)
    dist.all_reduce(t)
    return t.numpy()


def run(rank, world, port, n, out_dir):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from oracle import oracle
    from util import synth_to_oracle
    from xfemm_amd import kernels, synth

    pr, mesh, kw = synth_to_oracle(synth.magnetostatic(n))
    O, bo = oracle.system(pr, mesh)
    O = sp.csr_matrix(O)
    N = O.shape[0]
    plan = kernels.partition_plan(N, mesh.p, rank, world)
    row0, n_own, l2g = plan["row0"], plan["n_own"], plan["l2g"]
    g2l = {int(g): l for l, g in enumerate(l2g)}
    # local rows, local column ids; every column of an owned row must be local
    A = O[row0:row0 + n_own].tocoo()
    cols = np.array([g2l.get(int(c), -1) for c in A.col])
    assert (cols >= 0).all(), "halo misses a column of an owned row"
    Al = sp.csr_matrix((A.data, (A.row, cols)), shape=(n_own, len(l2g)))
    b = bo[row0:row0 + n_own]
    dinv = 1.0 / Al[:, :n_own].diagonal()

    # Chronopoulos-Gear PCG (x0 = 0)
    x = np.zeros(n_own)
    r = b.copy()
    u = np.zeros(len(l2g))
    u[:n_own] = dinv * r
    _exchange(u, plan)
    w = Al @ u
    g = _allreduce([float((dinv * b) @ b), float(r @ u[:n_own]), float(w @ u[:n_own])])
    res_o, gam, dlt = g
    z = np.zeros(n_own)
    p = np.zeros(n_own)
    gp = ap = None
    tol = pr.Precision
    it = 0
    while True:
        if it == 0:
            beta, alpha = 0.0, gam / dlt
        else:
            beta = gam / gp
            alpha = gam / (dlt - beta * gam / ap)
        er = np.sqrt(gam / res_o) if res_o else 0.0
        if res_o == 0.0 or (it >= 1 and er <= tol):
            break
        z = w + beta * z
        p = u[:n_own] + beta * p
        x = x + alpha * p
        r = r - alpha * z
        u[:n_own] = dinv * r
        gp, ap = gam, alpha
        _exchange(u, plan)
        w = Al @ u
        gam, dlt = _allreduce([float(r @ u[:n_own]), float(w @ u[:n_own])])
        it += 1
        assert it < 20 * N

    # gather and compare with a direct solve of the global system
    parts = [None] * world
    dist.all_gather_object(parts, (row0, x))
    if rank == 0:
        X = np.zeros(N)
        for r0, xs in parts:
            X[r0:r0 + len(xs)] = xs
        ref = sp.linalg.spsolve(O.tocsc(), bo)
        err = float(np.abs(X - ref).max() / np.abs(ref).max())
        with open(os.path.join(out_dir, "result.txt"), "w") as f:
            f.write("%d %.6e %d\n" % (it, err, sum(1 for _ in plan["recv"])))
    dist.barrier()
    dist.destroy_process_group()
