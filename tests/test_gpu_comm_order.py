"""Issue order of the sharded path's collectives, proved on recordings.

RCCL matches collectives by their order on a communicator and blocks each
kernel until the peers' matching kernels run, so every rank must issue the same
sequence of collectives, and two collectives of one communicator must never run
out of issue order on the device.  The sharded path issues halo exchanges on a
side stream (overlapped with the interior tiles of the PCG SpMV and the
V-cycle sweeps) and all-reduces / all-gathers on the main stream.

Every communicator (xfemm_amd/csrc/xfk_comm.hip) orders its collectives by
construction -- a collective on another stream than the previous one first
waits for the event recorded after it -- and records (op, stream, bytes,
peers, ranges) per call (xfk_comm_record).  These tests run the sharded HIP
path through the in-process transport at 2, 4 and 8 ranks and check with
kernels.check_comm_logs that

  * every rank made the same sequence of calls (op, stream index, payload);
  * in every exchange, each send of rank a to rank b has the matching receive
    of b from a (length, first global row) and the reverse;
  * every change of stream between two collectives carries the ordering wait;

over the overlapped SpMV and sweeps, the sharded AMG setup (aggregate counts,
P-row exchanges, the replicated-level all-gathers), the Newton loop (halo of
V, all-reduced residual sums), periodic / antiperiodic coupled rows, and the
all-ranks Jacobi fallback (one rank reports an aggregation failure through the
XFK_TEST_AMG_FAIL_RANK hook).  The replay transport then runs rank 0 alone from
its recording and must reproduce the recorded run bit for bit.
"""
import threading

import numpy as np
import pytest

from util import rel_err
from xfemm_amd import kernels, synth

pytestmark = pytest.mark.gpu

TOL_LINEAR = 1e-6
TOL_NONLINEAR = 1e-5


def run_recorded(kw, nranks, modes=None, solves=1, **opt):
    """`solves` x (solve + gathered solution) on nranks in-process ranks, every
    communicator recording; returns the last (results, solutions), the logs
    and the communicators."""
    comms = kernels.Comm.local_group(nranks)
    for q, c in enumerate(comms):
        c.record((modes or {}).get(q, 1))
    probs = [kernels.Static2DProblem(**kw, comm=comms[q], **opt) for q in range(nranks)]
    out = [None] * nranks
    err = [None] * nranks

    def work(q):
        try:
            for _ in range(solves):
                out[q] = (probs[q].solve(), probs[q].solution())
        except Exception as ex:   # surfaced below
            err[q] = ex

    th = [threading.Thread(target=work, args=(q,)) for q in range(nranks)]
    for t in th:
        t.start()
    for t in th:
        t.join()
    for p in probs:
        p.close()
    for e in err:
        if e is not None:
            raise e
    logs = [c.log() for c in comms]
    return [o[0] for o in out], [o[1] for o in out], logs, comms


def close_all(comms):
    for c in comms:
        c.close()


def single(kw, **opt):
    P = kernels.Static2DProblem(**kw, **opt)
    r = P.solve()
    A = P.solution()
    P.close()
    return r, A


@pytest.mark.parametrize("nranks", [2, 4, 8])
def test_linear_sharded_issue_order(monkeypatch, nranks):
    """Overlapped SpMV / level-0 sweeps (XFK_OVERLAP=1: exchanges on side
    streams), sharded AMG setup with a sharded coarse level (low replication
    threshold) and the replicated tail."""
    monkeypatch.setenv("XFK_OVERLAP", "1")
    kw = synth.magnetostatic(240)
    res, sols, logs, comms = run_recorded(kw, nranks, amg_replicate=2000)
    close_all(comms)
    summ = kernels.check_comm_logs(logs)
    print("%d ranks: %s" % (nranks, summ))
    assert res[0]["precond"] == kernels.XFK_PRECOND_AMG
    assert {"allreduce", "exchange", "allgather"} <= set(summ["ops"])
    # main stream + the SpMV's and the V-cycle's exchange side streams, every switch ordered
    assert len(summ["streams"]) == 3 and summ["stream_switches"] > 0
    r1, A1 = single(kw)
    for A in sols:
        assert rel_err(A, A1) <= TOL_LINEAR


@pytest.mark.parametrize("nranks", [2, 8])
def test_default_sharded_issue_order_one_stream(nranks):
    """The default (no overlap): every collective on the solve stream."""
    kw = synth.magnetostatic(240)
    res, sols, logs, comms = run_recorded(kw, nranks, amg_replicate=2000)
    close_all(comms)
    summ = kernels.check_comm_logs(logs)
    assert len(summ["streams"]) == 1 and summ["stream_switches"] == 0


@pytest.mark.parametrize("nranks", [2, 4])
def test_newton_sharded_issue_order(nranks):
    kw = synth.magnetostatic(64, nonlinear=True)
    res, sols, logs, comms = run_recorded(kw, nranks)
    close_all(comms)
    summ = kernels.check_comm_logs(logs)
    print("%d ranks, Newton %d: %s" % (nranks, res[0]["newton_iters"], summ))
    assert res[0]["newton_iters"] >= 3
    r1, A1 = single(kw)
    for A in sols:
        assert rel_err(A, A1) <= TOL_NONLINEAR


@pytest.mark.parametrize("anti,nranks", [(False, 2), (True, 4)])
def test_periodic_sharded_issue_order(anti, nranks):
    """Coupled rows of periodic / antiperiodic pairs: several ranges per peer."""
    kw = synth.bc_showcase(24, anti=anti)
    res, sols, logs, comms = run_recorded(kw, nranks)
    close_all(comms)
    kernels.check_comm_logs(logs)
    r1, A1 = single(kw)
    for A in sols:
        assert rel_err(A, A1) <= TOL_LINEAR


@pytest.mark.parametrize("nranks,fail_rank", [(2, 1), (4, 2)])
def test_jacobi_fallback_issue_order(monkeypatch, nranks, fail_rank):
    """One rank cannot aggregate: every rank still makes the same collective
    calls, agrees on the failure and falls back to Jacobi together."""
    monkeypatch.setenv("XFK_TEST_AMG_FAIL_RANK", str(fail_rank))
    kw = synth.magnetostatic(48)
    res, sols, logs, comms = run_recorded(kw, nranks)
    close_all(comms)
    summ = kernels.check_comm_logs(logs)
    print("%d ranks, fallback: %s" % (nranks, summ))
    assert all(r["precond"] == kernels.XFK_PRECOND_JACOBI for r in res)
    monkeypatch.delenv("XFK_TEST_AMG_FAIL_RANK")
    r1, A1 = single(kw, precond="jacobi")
    for A in sols:
        assert rel_err(A, A1) <= TOL_LINEAR


@pytest.mark.parametrize("nranks", [4])
def test_replay_reproduces_rank0_bit_for_bit(nranks):
    """Rank 0 recorded with its received bytes (mode 2) over a first and a
    repeated solve, then run alone on the replay transport: the same PCG
    iterations and the same bits of A in three solves (the repeated solve's
    segment is served again), and a solve that issues other collectives than
    its recorded segment is refused."""
    kw = synth.magnetostatic(160)
    res, sols, logs, comms = run_recorded(kw, nranks, modes={0: 2}, solves=2)
    kernels.check_comm_logs(logs)
    rep = comms[0].replay()
    close_all(comms)            # the replay owns the recording
    P = kernels.Static2DProblem(**kw, comm=rep)
    for _ in range(3):
        r = P.solve()
        A = P.solution()
        assert r["cg_iters"] == res[0]["cg_iters"]
        assert np.array_equal(A, sols[0])
    r = P.solve()
    with pytest.raises(kernels.XfkError, match="replay"):
        P.solve()               # the solution's all-gather of the segment was never issued
    P.close()
    rep.close()
