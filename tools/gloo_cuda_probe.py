import os, torch, torch.distributed as dist
dist.init_process_group("gloo")
r = dist.get_rank()
t = torch.full((4,), float(r), device="cuda:0")
try:
    if r == 0:
        dist.send(t, 1)
    else:
        dist.recv(t, 0)
    print("rank", r, "send/recv ok", t.tolist(), flush=True)
except Exception as e:
    print("rank", r, "send/recv FAIL", repr(e)[:200], flush=True)
try:
    w = dist.isend(t, 1) if r == 0 else dist.irecv(t, 0)
    w.wait()
    print("rank", r, "isend ok", flush=True)
except Exception as e:
    print("rank", r, "isend FAIL", repr(e)[:200], flush=True)
u = torch.ones(3, device="cuda:0") * (r + 1)
dist.all_reduce(u)
print("rank", r, "allreduce", u.tolist(), flush=True)
dist.barrier()
dist.destroy_process_group()
