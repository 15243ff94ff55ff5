"""Minimal driver for profiling: N eager split steps at batch B (default 4096) on cuda:0."""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "split-learning-k8s_amd"), ROOT]

import torch  # noqa: E402

from splitcnn.data import SyntheticMNIST, init_models  # noqa: E402
from splitcnn.engine import SplitTrainer  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--batch", type=int, default=4096)
ap.add_argument("--steps", type=int, default=3)
args = ap.parse_args()
x, y = SyntheticMNIST(42).batch(args.batch)
x, y = x.cuda(), y.cuda()
tr = SplitTrainer(*init_models(seed=0), device="cuda:0", graph=False)
for _ in range(args.steps):
    tr.step(x, y)
torch.cuda.synchronize()
print("done", tr.loss_log.flush()[-1])
