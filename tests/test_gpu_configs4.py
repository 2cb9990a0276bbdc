"""BASELINE configs[4] at full size: the synthetic 20M-triangle mesh
(3162 x 3162 cells, 10,004,569 DoF) solved on one device and sharded in row
blocks over 2 and 8 ranks.

The ranks run through the in-process communicator (one host thread per rank,
all on cuda:0: RCCL refuses two ranks on one device), so the whole sharded
path -- partition plan, ghost-element assembly, halo exchanges, the sharded
AMG hierarchy with its replicated coarse tail, the all-reduced PCG partials --
runs at the size the 8-GPU bench line uses.  The oracle's linked-list solver
cannot run at 20M triangles, so parity is carried by size-independent
properties (as in test_gpu_fullsize.py for configs[2]):

  * the device system after boundary conditions equals the independent
    vectorised restatement (tests/fullsize.py) to 1e-12 of max |K|, |b|;
  * every answer solves that system: |b - K A/c| / |b| <= 1e-6;
  * sharded vs single device: max |A_s - A_1| <= 1e-6 max |A_1| (the
    linear parity tolerance), every rank returns the same gathered A, and the
    PCG needs at most 1.25 x the single-device iterations + 2.

Each test stays well under gpurun's 3-minute silence limit; the mesh and the
single-device solve are module fixtures shared by all of them.
"""
import threading

import numpy as np
import pytest
import scipy.sparse as sp

import fullsize
from util import C_ANS, rel_err
from xfemm_amd import kernels, synth

pytestmark = pytest.mark.gpu

CELLS = 3162          # 2 * 3162^2 = 19,996,488 triangles, 10,004,569 nodes (configs[4])
TOL_LINEAR = 1e-6
TOL_RESIDUAL = 1e-6


@pytest.fixture(scope="module")
def kw():
    return synth.magnetostatic(CELLS)


@pytest.fixture(scope="module")
def single(kw):
    P = kernels.Static2DProblem(**kw)
    r = P.solve()
    A = P.solution()
    rp, col, val, b = P.csr()
    P.close()
    n = len(rp) - 1
    K = sp.csr_matrix((val, col, rp), shape=(n, n))
    return r, A, K, b


def residual(K, b, A):
    V = A / C_ANS
    return float(np.linalg.norm(b - K @ V) / np.linalg.norm(b))


def run_sharded(kw, nranks):
    comms = kernels.Comm.local_group(nranks)
    probs = [kernels.Static2DProblem(**kw, comm=comms[q]) for q in range(nranks)]
    out = [None] * nranks
    err = [None] * nranks

    def work(q):
        try:
            out[q] = (probs[q].solve(), probs[q].solution(), probs[q].dist_info())
        except Exception as ex:   # surfaced below
            err[q] = ex

    th = [threading.Thread(target=work, args=(q,)) for q in range(nranks)]
    for t in th:
        t.start()
    for t in th:
        t.join()
    for p in probs:
        p.close()
    for c in comms:
        c.close()
    for e in err:
        if e is not None:
            raise e
    return out


def test_configs4_single_device_solves_its_system(kw, single):
    r, A, K, b = single
    assert len(kw["x"]) == 10_004_569 and len(kw["p"]) == 2 * CELLS * CELLS
    assert r["precond"] == kernels.XFK_PRECOND_AMG and r["newton_iters"] == 1
    res = residual(K, b, A)
    print("configs[4] single device: %d PCG iterations, %d AMG levels, |b - K V| / |b| = %.3e"
          % (r["cg_iters"], r["amg_levels"], res))
    assert np.isfinite(A).all()
    assert res <= TOL_RESIDUAL, res


def test_configs4_system_matches_restatement(kw, single):
    from util import synth_to_oracle
    _, _, G, bg = single
    pr, mesh, _ = synth_to_oracle(kw)
    K, b, _ = fullsize.assemble(pr, mesh)
    dK = abs(G - K).max()
    assert dK <= 1e-12 * abs(K).max(), dK
    assert np.abs(bg - b).max() <= 1e-12 * np.abs(b).max()


@pytest.mark.parametrize("nranks", [2, 8])
def test_configs4_sharded_matches_single_device(kw, single, nranks):
    r1, A1, K, b = single
    outs = run_sharded(kw, nranks)
    res0, A0, _ = outs[0]
    rows = sum(o[2]["n_own"] for o in outs)
    assert rows == len(A1)
    for res, A, info in outs:
        assert info["nranks"] == nranks and info["n_halo"] > 0
        assert res["cg_iters"] == res0["cg_iters"]          # every rank stops together
        assert np.array_equal(A, A0)                        # same gathered solution everywhere
    err = rel_err(A0, A1)
    rr = residual(K, b, A0)
    print("configs[4] %d ranks: %d PCG iterations (single %d), max|dA|/max|A| vs single %.3e, residual %.3e"
          % (nranks, res0["cg_iters"], r1["cg_iters"], err, rr))
    assert res0["precond"] == kernels.XFK_PRECOND_AMG
    assert res0["cg_iters"] <= 1.25 * r1["cg_iters"] + 2, (res0["cg_iters"], r1["cg_iters"])
    assert err <= TOL_LINEAR, err
    assert rr <= TOL_RESIDUAL, rr
