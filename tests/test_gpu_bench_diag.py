"""The N > 1 bench line's diagnosis (bench.py sharded_diagnosis /
local_ranks_run): time inside each kind of collective per rank
(xfk_comm_time / xfk_comm_timing), the per-rank phases and their maxima.
Driven through the in-process transport (2 ranks on this GPU), the same
code path the RCCL run reports."""
import json
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
pytestmark = pytest.mark.gpu


def test_local_ranks_line_carries_the_collective_diagnosis():
    """bench.py --force-sharded --local-ranks 2, called in this process (no
    child process: this one has the GPU up already)."""
    import argparse
    sys.path.insert(0, ROOT)
    import bench
    args = argparse.Namespace(local_ranks=2, shard_cells=300, nonlinear=False, precond="amg", amg_sweeps=1,
                              amg_omega=1.75, amg_dense=None, amg_theta=None, amg_replicate=None, steps=2, warmup=1)
    line = json.loads(json.dumps(bench.local_ranks_run(args)))
    d = line["sharded_diagnosis"]
    assert len(d["ranks"]) == 2
    ops = d["comm"]["ops"]
    assert ops["allreduce"]["calls_per_solve"] >= d["ranks"][0]["pcg_iters"]
    assert ops["exchange"]["calls_per_solve"] >= d["ranks"][0]["pcg_iters"]
    assert d["comm"]["calls_per_solve"] == sum(v["calls_per_solve"] for v in ops.values())
    assert 0 < d["comm"]["ms_in_collectives_rank0"] <= d["comm"]["ms_in_collectives_max_over_ranks"]
    for k in ("ms_amg_setup", "ms_pcg", "us_per_pcg_iteration"):
        assert d["max_over_ranks"][k] == max(q[k] for q in d["ranks"])
    assert all(q["rows"] > 0 and q["halo"] > 0 for q in d["ranks"])


def test_comm_timing_counts_every_collective():
    from xfemm_amd import kernels, synth
    kw = synth.magnetostatic(120)
    comms = kernels.Comm.local_group(2)
    import threading
    probs = [kernels.Static2DProblem(comm=comms[q], **kw) for q in range(2)]
    for c in comms:
        c.record(1)
        c.time(True)
    res, err = [None, None], [None, None]

    def work(q):
        try:
            res[q] = probs[q].solve(rebuild_symbolic=True)
        except Exception as ex:
            err[q] = ex

    th = [threading.Thread(target=work, args=(q,)) for q in range(2)]
    for t in th:
        t.start()
    for t in th:
        t.join()
    assert err == [None, None]
    for c in comms:
        tm = c.timing()
        log = c.log()
        n = {k: sum(1 for o in log if o["op"] == k) for k in ("allreduce", "exchange", "allgather")}
        assert {k: v["calls"] for k, v in tm.items()} == n
        assert all(v["us"] >= 0 and v["us_max_call"] <= v["us"] + 1e-9 for v in tm.values())
        again = c.timing()   # read and cleared
        assert all(v["calls"] == 0 for v in again.values())
    for p in probs:
        p.close()
    for c in comms:
        c.close()
