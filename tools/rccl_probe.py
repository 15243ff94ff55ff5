"""Probe: can two processes on ONE GPU form an RCCL (backend "nccl") group? (profiling aid)
Each rank does an all_reduce and an isend/irecv exchange of a device tensor, then prints the result."""
import os
import socket
import sys

import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def worker(rank, world, port):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dev = torch.device("cuda:0")
    torch.cuda.set_device(dev)
    dist.init_process_group("nccl", rank=rank, world_size=world, device_id=dev)
    t = torch.full((1 << 20,), float(rank + 1), device=dev)
    dist.all_reduce(t)
    torch.cuda.synchronize()
    r = torch.empty(1 << 20, device=dev)
    peer = 1 - rank
    if rank == 0:
        w = [dist.isend(t * 2, peer), dist.irecv(r, peer)]
    else:
        w = [dist.irecv(r, peer), dist.isend(t * 3, peer)]
    for x in w:
        x.wait()
    torch.cuda.synchronize()
    print(f"rank {rank}: all_reduce {t[0].item()} recv {r[0].item()}", flush=True)
    dist.destroy_process_group()


if __name__ == "__main__":
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    mp.spawn(worker, args=(2, port), nprocs=2, join=True)
    print("RCCL two ranks on one GPU: ok", flush=True)
