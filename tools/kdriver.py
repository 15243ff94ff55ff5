"""Minimal driver for profiling: N eager split steps (k2: reference CNN fp32; k5: widened bf16) at batch B
(default 4096) on cuda:0."""
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
ap.add_argument("--config", default="k2", choices=["k2", "k5"])
ap.add_argument("--conv", default=None, help="K2 conv preset (splitcnn.engine.CONV_PRESETS; default CONV_DEFAULT)")
args = ap.parse_args()
if args.config == "k5":
    from splitcnn.wide import SyntheticCIFAR, WideTrainer, init_wide_models
    x, y = SyntheticCIFAR(42).batch(args.batch)
    tr = WideTrainer(*init_wide_models(seed=0), device="cuda:0", graph=False)
else:
    x, y = SyntheticMNIST(42).batch(args.batch)
    from splitcnn.engine import CONV_DEFAULT
    tr = SplitTrainer(*init_models(seed=0), device="cuda:0", graph=False, conv=args.conv or CONV_DEFAULT)
x, y = x.cuda(), y.cuda()
for _ in range(args.steps):
    tr.step(x, y)
torch.cuda.synchronize()
print("done", tr.loss_log.flush()[-1])
