"""Probe: can two RCCL ranks share one GPU (for 2-rank tests on a 1-GPU box)?"""
import os, sys
import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def worker(rank, world):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = "29533"
    torch.cuda.set_device(0)
    dist.init_process_group("nccl", rank=rank, world_size=world, device_id=torch.device("cuda", 0))
    t = torch.full((4,), float(rank + 1), device="cuda")
    dist.all_reduce(t)
    x = torch.full((3,), float(rank), device="cuda")
    y = torch.empty(3, device="cuda")
    if rank == 0:
        dist.send(x, 1)
        dist.recv(y, 1)
    else:
        dist.recv(y, 0)
        dist.send(x, 0)
    torch.cuda.synchronize()
    print("rank", rank, "allreduce", t.tolist(), "recv", y.tolist(), flush=True)
    dist.destroy_process_group()


if __name__ == "__main__":
    mp.spawn(worker, args=(2,), nprocs=2)
