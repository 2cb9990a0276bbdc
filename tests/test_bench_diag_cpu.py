"""bench.py's N > 1 diagnosis over real ranks (2 gloo processes, CPU): every
rank's row reaches rank 0 through all_gather_object, and the summary carries
per-op calls, rank-0 and maximum-over-ranks times (tests/diag_worker.py stands
in for the GPU measurement of each rank)."""
import json
import os
import socket
import tempfile

import torch.multiprocessing as mp

import diag_worker


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def test_sharded_diagnosis_gathers_every_rank():
    with tempfile.TemporaryDirectory() as d:
        mp.spawn(diag_worker.run, args=(2, _free_port(), d), nprocs=2, join=True)
        out = json.load(open(os.path.join(d, "diag.json")))
    assert out["transport"] == "rccl"
    assert [r["rank"] for r in out["ranks"]] == [0, 1]
    ops = out["comm"]["ops"]
    assert ops["allreduce"]["calls_per_solve"] == 10 and ops["allgather"]["calls_per_solve"] == 12
    assert ops["exchange"]["us_rank0"] == 101.0 and ops["exchange"]["us_max_over_ranks"] == 201.0
    assert out["comm"]["calls_per_solve"] == 33
    assert out["max_over_ranks"]["ms_amg_setup"] == 2.0 and out["max_over_ranks"]["ms_solve"] == 4.5
    assert out["comm"]["ms_in_collectives_max_over_ranks"] >= out["comm"]["ms_in_collectives_rank0"]
