"""Sharded solve (configs[4] path) on the GPU: the mesh split in row blocks over
several ranks, each assembling its rows, exchanging PCG halos and
all-reducing the inner-product partials.

These tests drive the real sharded HIP path through the in-process local
communicator (one host thread per rank, all ranks on cuda:0): RCCL refuses two
ranks on one device, and the GPU test box has one.  The RCCL transport itself
runs in bench.py at N > 1 (one process per GPU).

Tolerances as in test_gpu_static2d.py: linear 1e-6, nonlinear 1e-5 of max|A|
against the oracle; against the single-device solve the same bounds (the
partial sums are grouped per rank, so iterates differ in the last bits and
both stop at the same PCG criterion).  One rank must reproduce the
single-device solve bit for bit.
"""
import threading

import numpy as np
import pytest

from oracle import oracle
from util import assert_parity, converged, rel_err, synth_to_oracle
from xfemm_amd import kernels, synth

pytestmark = pytest.mark.gpu

TOL_LINEAR = 1e-6
TOL_NONLINEAR = 1e-5


def run_sharded(kw, nranks, **opt):
    comms = kernels.Comm.local_group(nranks)
    probs = [kernels.Static2DProblem(**kw, comm=comms[r], **opt) for r in range(nranks)]
    out = [None] * nranks
    err = [None] * nranks

    def work(r):
        try:
            res = probs[r].solve()
            out[r] = (res, probs[r].solution(), probs[r].circuits(), probs[r].dist_info())
        except Exception as ex:   # surfaced below
            err[r] = ex

    th = [threading.Thread(target=work, args=(r,)) for r in range(nranks)]
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


def single(kw):
    P = kernels.Static2DProblem(**kw)
    r = P.solve()
    return r, P.solution(), P.circuits()


def test_one_rank_is_bit_identical_to_single_device():
    kw = synth.magnetostatic(40)
    r1, A1, _ = single(kw)
    (rs, As, _, info), = run_sharded(kw, 1)
    assert info["n_halo"] == 0 and info["n_own"] == len(kw["x"])
    assert rs["cg_iters"] == r1["cg_iters"]
    assert np.array_equal(As, A1)


@pytest.mark.parametrize("nranks", [2, 3, 4])
def test_sharded_linear_matches_oracle(nranks):
    pr, mesh, kw = synth_to_oracle(synth.magnetostatic(48))
    Ao, _, _ = oracle.solve(pr, mesh)
    outs = run_sharded(kw, nranks)
    r1, A1, _ = single(kw)
    for res, A, _, info in outs:
        assert info["nranks"] == nranks and info["n_halo"] > 0
        assert rel_err(A, Ao) <= TOL_LINEAR
        assert rel_err(A, A1) <= TOL_LINEAR
        assert res["cg_iters"] == outs[0][0]["cg_iters"]     # every rank stops together
    assert np.array_equal(outs[0][1], outs[-1][1])             # same gathered solution everywhere


@pytest.mark.parametrize("nranks", [2, 4, 8])
def test_sharded_amg_iterations_match_single_device(nranks):
    """The sharded hierarchy (rank-local aggregation, Galerkin product over the
    full rows with the peers' P rows, global replicated coarse levels) keeps
    every inter-rank coupling: the PCG needs about as many iterations as on
    one device, not the growth of a block preconditioner."""
    kw = synth.magnetostatic(120)
    r1, A1, _ = single(kw)
    outs = run_sharded(kw, nranks)
    res, A, _, _ = outs[0]
    assert res["precond"] == kernels.XFK_PRECOND_AMG
    assert res["cg_iters"] <= 1.25 * r1["cg_iters"] + 2, (res["cg_iters"], r1["cg_iters"])
    assert rel_err(A, A1) <= TOL_LINEAR


@pytest.mark.parametrize("nranks", [2, 3, 4])
def test_sharded_coarse_levels(nranks):
    """A low replication threshold keeps several coarse levels sharded (each
    with its own halo plan over the peers' aggregate ids) before the global
    replicated tail: same answer, iterations as on one device."""
    pr, mesh, kw = synth_to_oracle(synth.magnetostatic(48))
    Ao, _, _ = oracle.solve(pr, mesh)
    r1, A1, _ = single(kw)
    outs = run_sharded(kw, nranks, amg_replicate=40)
    for res, A, _, _ in outs:
        assert res["precond"] == kernels.XFK_PRECOND_AMG
        assert rel_err(A, Ao) <= TOL_LINEAR
        assert rel_err(A, A1) <= TOL_LINEAR
        assert res["cg_iters"] <= 1.25 * r1["cg_iters"] + 2, (res["cg_iters"], r1["cg_iters"])
    assert np.array_equal(outs[0][1], outs[-1][1])


@pytest.mark.parametrize("nranks,cells,rep", [(3, 200, 250000), (2, 480, 1000)])
def test_exchange_overlap_is_bit_identical(monkeypatch, nranks, cells, rep):
    """With XFK_OVERLAP=1 the sharded halo exchanges (PCG SpMV, V-cycle
    sweeps on tile levels) run on a side stream while the tiles without halo
    columns compute; by default each exchange precedes one launch over every
    tile.  Same tiles, same partial-sum slots: the same bits and iterations.
    The second case keeps a level-1 of > 16k rows per rank sharded (tile
    kernels there too)."""
    kw = synth.magnetostatic(cells)
    off = run_sharded(kw, nranks, amg_replicate=rep)
    monkeypatch.setenv("XFK_OVERLAP", "1")
    on = run_sharded(kw, nranks, amg_replicate=rep)
    for (r_on, A_on, _, _), (r_off, A_off, _, _) in zip(on, off):
        assert r_on["precond"] == kernels.XFK_PRECOND_AMG
        assert r_on["cg_iters"] == r_off["cg_iters"]
        assert np.array_equal(A_on, A_off)


def test_sharded_nonlinear_matches_oracle():
    pr, mesh, kw = synth_to_oracle(synth.magnetostatic(32, nonlinear=True))
    Ao, st, _ = oracle.solve(pr, mesh)
    P = kernels.Static2DProblem(**kw)
    P.solve()
    A1 = P.solution()
    P.close()
    Ac = converged(pr, mesh)
    assert_parity(A1, Ao, Ac, TOL_NONLINEAR)
    outs = run_sharded(kw, 3)
    for res, A, _, _ in outs:
        assert res["newton_iters"] >= 3
        assert_parity(A, Ao, Ac, TOL_NONLINEAR)
        assert rel_err(A, A1) <= TOL_NONLINEAR
    assert len({o[0]["newton_iters"] for o in outs}) == 1


def test_sharded_scrambled_numbering():
    """A random node numbering: every rank needs halo ranges from every peer."""
    kw = synth.magnetostatic(36)
    N = len(kw["x"])
    perm = np.random.default_rng(3).permutation(N)
    inv = np.argsort(perm)
    kw2 = dict(kw)
    kw2["x"] = np.asarray(kw["x"])[inv]
    kw2["y"] = np.asarray(kw["y"])[inv]
    kw2["p"] = perm[np.asarray(kw["p"])]
    r1, A1, _ = single(kw2)
    outs = run_sharded(kw2, 3)
    for res, A, _, info in outs:
        assert info["n_recv"] == 2
        assert rel_err(A, A1) <= TOL_LINEAR


def test_sharded_circuit_and_point_current():
    """Circuit currents and point currents are evaluated on the global mesh."""
    kw = synth.magnetostatic(40)
    kw = dict(kw)
    kw["labels"] = [dict(l) for l in kw["labels"]]
    coil = next(k for k, l in enumerate(kw["labels"]) if kw["blocks"][l["block"]].get("J_re", 0) > 0)
    kw["labels"][coil]["in_circuit"] = 0
    kw["circuits"] = [dict(type=0, amps_re=3.0)]
    N = len(kw["x"])
    marker = -np.ones(N, np.int32)
    marker[N // 2 + 7] = 0
    kw["marker"] = marker
    kw["points"] = [dict(J_re=0.5)]
    r1, A1, c1 = single(kw)
    outs = run_sharded(kw, 2)
    for res, A, c, _ in outs:
        assert rel_err(A, A1) <= TOL_LINEAR
        assert np.array_equal(c[1], c1[1])


@pytest.mark.parametrize("anti,nranks", [(False, 2), (True, 3), (False, 4)])
def test_sharded_periodic_matches_oracle(anti, nranks):
    """Periodic / antiperiodic pairs across rank blocks: the coupled nodes'
    rows are assembled on every rank (extra rows), so each rank's periodic
    averaging map (the reference's sequential Periodicity / AntiPeriodicity)
    reads every pre-map entry locally."""
    pr, mesh, kw = synth_to_oracle(synth.bc_showcase(24, anti=anti))
    Ao, _, _ = oracle.solve(pr, mesh)
    Ac = converged(pr, mesh)
    r1, A1, _ = single(kw)
    outs = run_sharded(kw, nranks)
    assert any(o[3]["n_extra"] > 0 for o in outs)
    for res, A, _, info in outs:
        assert_parity(A, Ao, Ac, TOL_LINEAR)
        assert rel_err(A, A1) <= TOL_LINEAR
    assert np.array_equal(outs[0][1], outs[-1][1])


def test_sharded_periodic_nonlinear():
    pr, mesh, kw = synth_to_oracle(synth.bc_showcase(20, nonlinear=True))
    Ao, _, _ = oracle.solve(pr, mesh)
    Ac = converged(pr, mesh)
    for res, A, _, _ in run_sharded(kw, 3):
        assert_parity(A, Ao, Ac, TOL_NONLINEAR)


@pytest.mark.parametrize("nranks", [2, 4])
def test_sharded_torque_benchmark(tmp_path, nranks):
    """configs[0] (TorqueBenchmark: periodic pbc1/pbc2 + air gap + magnets)
    sharded: A vs the converged oracle and the reference's torque check."""
    from oracle import femfile, gaptorque
    from torque import torque_ok, write_case
    from util import kernel_kwargs
    deg = 30
    pr, mesh = femfile.load_problem(write_case(tmp_path, deg))
    kw = kernel_kwargs(pr, mesh)
    Ao, _, _ = oracle.solve(pr, mesh)
    Ac = converged(pr, mesh)
    outs = run_sharded(kw, nranks)
    assert any(o[3]["n_extra"] > 0 for o in outs)
    for res, A, _, info in outs:
        assert_parity(A, Ao, Ac, TOL_LINEAR)
        tq = gaptorque.gap_dc_torque(mesh.ages[0], A, pr.Depth, pr.LengthUnits)
        assert torque_ok(tq, deg)[0], tq


def test_rccl_single_rank_is_bit_identical():
    """The production transport (RCCL) with one rank: init, all-reduce, all-gather."""
    kw = synth.magnetostatic(40)
    r1, A1, _ = single(kw)
    comm = kernels.Comm.rccl(kernels.Comm.unique_id(), 0, 1, 0)
    P = kernels.Static2DProblem(**kw, comm=comm)
    r = P.solve()
    A = P.solution()
    P.close()
    comm.close()
    assert r["cg_iters"] == r1["cg_iters"]
    assert np.array_equal(A, A1)
