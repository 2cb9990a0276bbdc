"""Device memory of a problem solved again and again (a rotor-angle loop, a
session's repeated analyses) stays at the footprint of its largest solve.

Every solve carves its scratch (the AMG setup's temporaries, KludgeSolve's
update vector, the sharded setup's gathered rows, the old block of a buffer
that grows) out of the problem's arena; freed blocks become reusable at the
end of the solve (xfemm_amd/csrc/xfk_api.hip: DevArena::recycle), so after the
first few solves the arena's chunk bytes must not grow.  Answers stay
bit-identical across the repeats (a reused block holds stale bytes: every
kernel must overwrite what it reads).  The process-wide caches of destroyed
problems can be given back (xfk_release_cache).
"""
import threading

import numpy as np
import pytest

from xfemm_amd import kernels, synth

pytestmark = pytest.mark.gpu


def _flat(mems):
    """chunk bytes after the warm-up solves equal those after the last one"""
    return mems[-1]["chunk_bytes"] == mems[2]["chunk_bytes"], [m["chunk_bytes"] for m in mems]


@pytest.mark.parametrize("nonlinear", [False, True])
def test_static_arena_stays_flat_over_50_solves(nonlinear):
    P = kernels.Static2DProblem(**synth.magnetostatic(60, nonlinear=nonlinear))
    mems, A0 = [], None
    for k in range(50):
        P.solve(rebuild_symbolic=(k % 2 == 0))
        A = P.solution()
        if A0 is None:
            A0 = A
        assert np.array_equal(A, A0), "solve %d differs from the first" % k
        mems.append(P.memory())
    P.close()
    ok, trace = _flat(mems)
    assert ok, trace
    assert mems[-1]["live_bytes"] <= mems[-1]["chunk_bytes"]


def test_harmonic_newton_ac_arena_stays_flat():
    kw = synth.harmonic(14, nonlinear=True)
    kw["ac_solver"] = 1
    P = kernels.Harmonic2DProblem(**kw)
    mems, A0 = [], None
    for k in range(20):
        P.solve(rebuild_symbolic=(k % 2 == 0))
        A = P.solution()
        if A0 is None:
            A0 = A
        assert np.array_equal(A, A0), "solve %d differs from the first" % k
        mems.append(P.memory())
    P.close()
    ok, trace = _flat(mems)
    assert ok, trace


def test_sharded_arena_stays_flat():
    R = 2
    kw = synth.magnetostatic(80, nonlinear=True)
    comms = kernels.Comm.local_group(R)
    probs = [kernels.Static2DProblem(**kw, comm=comms[q], amg_replicate=1000) for q in range(R)]
    mems = [[] for _ in range(R)]
    sols = [[] for _ in range(R)]
    err = [None] * R

    def work(q):
        try:
            for k in range(20):
                probs[q].solve(rebuild_symbolic=(k % 2 == 0))
                sols[q].append(probs[q].solution())
                mems[q].append(probs[q].memory())
        except Exception as ex:   # surfaced below
            err[q] = ex

    th = [threading.Thread(target=work, args=(q,)) for q in range(R)]
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
    for q in range(R):
        ok, trace = _flat(mems[q])
        assert ok, (q, trace)
        for k, A in enumerate(sols[q]):
            assert np.array_equal(A, sols[q][0]), (q, k)


def test_release_cache_returns_destroyed_problems_blocks():
    kw = synth.magnetostatic(50)
    P = kernels.Static2DProblem(**kw)
    P.solve()
    A = P.solution()
    P.close()
    assert kernels.cache_stats()["device_bytes"] > 0
    kernels.release_cache()
    st = kernels.cache_stats()
    assert st["device_bytes"] == 0 and st["pinned_bytes"] == 0 and st["idle_streams"] == 0
    Q = kernels.Static2DProblem(**kw)     # a fresh problem after the release allocates anew
    Q.solve()
    assert np.array_equal(Q.solution(), A)
    Q.close()
