"""Worker of tests/test_bench_diag_cpu.py: one gloo rank calling bench.py's
sharded_diagnosis with a stand-in for the per-rank GPU measurement
(bench.diagnosis_row), so the gather over ranks and the summary of the N > 1
line run as they do on the GPU ranks."""
import json
import os
import sys

import torch.distributed as dist


def run(rank, world, port, out_dir):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path.insert(0, root)
    import bench

    def fake_row(P, comm, r):
        ops = {nm: {"calls": 10 + k, "us": 100.0 * (r + 1) + k, "us_max_call": 5.0 + r}
               for k, nm in enumerate(("allreduce", "exchange", "allgather"))}
        return {"rank": r, "rows": 1000 + r, "halo": 10, "pcg_iters": 20, "ms_symbolic": 0.1, "ms_assemble": 0.2,
                "ms_amg_setup": 1.0 + r, "ms_pcg": 2.0 + 0.5 * r, "ms_solve": 3.0 + 1.5 * r,
                "us_per_pcg_iteration": 100.0 + r, "ms_in_collectives": 1e-3 * sum(v["us"] for v in ops.values()),
                "collectives": ops, "replicated_tail": {"ms_setup": 0.5, "us_per_vcycle": 70.0, "vcycles": 21}}

    bench.diagnosis_row = fake_row
    d = bench.sharded_diagnosis(None, None, dist, rank, world)
    if rank == 0:
        with open(os.path.join(out_dir, "diag.json"), "w") as fh:
            json.dump(d, fh)
    else:
        assert d is None
    dist.barrier()
    dist.destroy_process_group()
