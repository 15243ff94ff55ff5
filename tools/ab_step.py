"""Profiling-only: A/B the whole fused split step (HIP graph) between trainer variants in ONE process,
interleaved rounds, so box-to-box clock differences cancel. usage: python tools/ab_step.py"""
import json
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "split-learning-k8s_amd"), ROOT]
from bench import make_pool  # noqa: E402
from splitcnn.data import init_models  # noqa: E402
from splitcnn.engine import SplitTrainer  # noqa: E402

B, K, R = 4096, 20, 6
dev = torch.device("cuda:0")
X, Y = make_pool(B, 4, dev)
variants = {}
for name, fuse in (("fused_server_optim", True), ("separate_optim", False)):
    tr = SplitTrainer(*init_models(seed=0), device=dev, graph=True)
    tr.server.fuse_optim = fuse
    variants[name] = tr
res = {k: [] for k in variants}
for r in range(R):
    for name, tr in variants.items():
        for i in range(3):
            tr.step(X[i % 4], Y[i % 4])
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for i in range(K):
            tr.step(X[i % 4], Y[i % 4])
        torch.cuda.synchronize()
        res[name].append((time.perf_counter() - t0) / K * 1e3)
print(json.dumps({k: {"min_ms": round(min(v), 4), "median_ms": round(sorted(v)[len(v) // 2], 4)} for k, v in res.items()}))
