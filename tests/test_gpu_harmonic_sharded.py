"""Sharded time-harmonic solve (xfk_problem_create_harmonic_dist): the
Harmonic2D COCG with the AMG surrogate preconditioner over row blocks, as the
static sharded path -- each rank assembles its rows, exchanges the halo of
x / u before each SpMV, all-reduces the COCG partials after it, runs the
sharded AMG setup / V-cycle, and sums the successive-approximation change
over the ranks.

Driven through the in-process transport (one host thread per rank, all ranks
on cuda:0), every communicator recording its calls so that
kernels.check_comm_logs proves the issue order (same sequence on every rank,
matched sends / receives, the wait on every stream switch).

Tolerances: against the single-device solve 1e-6 of max|A| (linear) and 1e-5
(nonlinear successive approximation) -- the partial sums are grouped per rank,
so iterates differ in the last bits and both stop at the same COCG
criterion; one rank reproduces the single-device solve bit for bit.
"""
import threading

import numpy as np
import pytest

from util import rel_err
from xfemm_amd import kernels, synth

pytestmark = pytest.mark.gpu

TOL_LINEAR = 1e-6
TOL_NONLINEAR = 1e-5


def run_sharded(kw, nranks, solves=1, **opt):
    comms = kernels.Comm.local_group(nranks)
    for c in comms:
        c.record(1)
    probs = [kernels.Harmonic2DProblem(**kw, comm=comms[q], **opt) for q in range(nranks)]
    out = [None] * nranks
    err = [None] * nranks

    def work(q):
        try:
            for _ in range(solves):
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
    logs = [c.log() for c in comms]
    for c in comms:
        c.close()
    for e in err:
        if e is not None:
            raise e
    return out, logs


def single(kw, **opt):
    P = kernels.Harmonic2DProblem(**kw, **opt)
    r = P.solve()
    A = P.solution()
    P.close()
    return r, A


def test_one_rank_is_bit_identical_to_single_device():
    kw = synth.harmonic(30)
    r1, A1 = single(kw)
    ((rs, As, info),), _ = run_sharded(kw, 1)
    assert info["n_halo"] == 0 and info["n_own"] == len(kw["x"])
    assert rs["cg_iters"] == r1["cg_iters"]
    assert np.array_equal(As, A1)


@pytest.mark.parametrize("nranks", [2, 4])
@pytest.mark.parametrize("periodic", [None, "per", "anti"])
def test_sharded_linear_matches_single_device(nranks, periodic):
    kw = synth.harmonic(48, periodic=periodic is not None, anti=periodic == "anti")
    r1, A1 = single(kw)
    out, logs = run_sharded(kw, nranks)
    for rs, As, info in out:
        assert rs["precond"] == r1["precond"] == kernels.XFK_PRECOND_AMG
        assert rel_err(As, A1) <= TOL_LINEAR, (nranks, periodic, rel_err(As, A1))
        # the sharded V-cycle is the single-device one up to rounding
        assert abs(rs["cg_iters"] - r1["cg_iters"]) <= max(2, r1["cg_iters"] // 10)
    assert sum(o[2]["n_own"] for o in out) == len(kw["x"])
    kernels.check_comm_logs(logs)


@pytest.mark.parametrize("nranks", [2, 4])
def test_sharded_jacobi_matches_single_device(nranks):
    kw = synth.harmonic(32, circuits=False)
    r1, A1 = single(kw, precond="jacobi")
    out, logs = run_sharded(kw, nranks, precond="jacobi")
    for rs, As, _ in out:
        assert rs["precond"] == kernels.XFK_PRECOND_JACOBI
        assert rel_err(As, A1) <= TOL_LINEAR
    kernels.check_comm_logs(logs)


@pytest.mark.parametrize("nranks", [2, 4])
def test_sharded_nonlinear_matches_single_device(nranks):
    """Successive approximation: the elements read V at their halo nodes (one
    exchange per pass), the change |dV| / |V| is summed over the ranks, so
    every rank takes the same number of passes."""
    kw = synth.harmonic(36, nonlinear=True)
    r1, A1 = single(kw)
    out, logs = run_sharded(kw, nranks, solves=2)
    assert r1["newton_iters"] > 1
    for rs, As, _ in out:
        assert rel_err(As, A1) <= TOL_NONLINEAR
        assert abs(rs["newton_iters"] - r1["newton_iters"]) <= 2
        assert rs["newton_iters"] == out[0][0]["newton_iters"]
    kernels.check_comm_logs(logs)


def test_sharded_unsupported_cases_are_reported():
    """Case-2 circuits (bordered system) and the Newton AC solver stay on one
    device: refused at creation with the reason."""
    kw = synth.harmonic(12, nonlinear=True)
    comms = kernels.Comm.local_group(2)
    try:
        with pytest.raises(kernels.XfkError, match="ACSolver"):
            kernels.Harmonic2DProblem(**kw, ac_solver=1, comm=comms[0])
    finally:
        for c in comms:
            c.close()
