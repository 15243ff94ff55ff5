"""Profiling-only: the data-parallel Replicated step (bench.py's N > 1 headline path, eager + RCCL
all-reduce) at world size 1 on one GPU, against the single-GPU HIP-graph SplitTrainer step, so the
per-GPU cost of the N > 1 path is known before a multi-GPU run. usage: python tools/rep_probe.py"""
import json
import os
import sys
import time

import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "split-learning-k8s_amd"), ROOT]
from bench import make_pool  # noqa: E402
from splitcnn import dist as sd  # noqa: E402
from splitcnn.data import init_models  # noqa: E402
from splitcnn.engine import ClientStage, ServerStage, SplitTrainer  # noqa: E402

os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
os.environ.setdefault("MASTER_PORT", "29533")
dist.init_process_group("nccl", rank=0, world_size=1)
dev = torch.device("cuda:0")
torch.cuda.set_device(dev)
B, K = 4096, 30
X, Y = make_pool(B, 4, dev)
a, b = init_models(seed=0)
rep = sd.Replicated(ClientStage(a, device=dev), ServerStage(b, device=dev))
a2, b2 = init_models(seed=0)
tr = SplitTrainer(a2, b2, device=dev, graph=True)
res = {}
for name, fn in (("replicated_graph", lambda i: rep.step(X[i % 4], Y[i % 4])),
                 ("trainer_graph", lambda i: tr.step(X[i % 4], Y[i % 4]))) * 2:
    for i in range(5):
        fn(i)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(K):
        fn(i)
    torch.cuda.synchronize()
    res.setdefault(name, []).append((time.perf_counter() - t0) / K * 1e3)
print(json.dumps({k: [round(v, 4) for v in vs] for k, vs in res.items()}))
dist.destroy_process_group()
