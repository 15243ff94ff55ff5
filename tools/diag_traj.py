"""Diagnostic: the trajectory test's setting (B = 4096, a fresh noisy batch per step) for the default x3
trainer (graph and eager) and the f32 preset, printing the loss every 10 steps.
usage: python tools/diag_traj.py [B] [steps]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "split-learning-k8s_amd"), ROOT]
import torch  # noqa: E402

from splitcnn.data import SyntheticMNIST, init_models  # noqa: E402
from splitcnn.engine import SplitTrainer  # noqa: E402

gpu = torch.device("cuda:0")
B = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
steps = int(sys.argv[2]) if len(sys.argv) > 2 else 100
data = SyntheticMNIST(71)
xs, ys = zip(*(data.batch(B) for _ in range(8)))
X, Y = torch.stack(xs).to(gpu), torch.stack(ys).to(gpu)
for conv, graph in (("x3", True), ("x3", False), ("f32", True)):
    tr = SplitTrainer(*init_models(seed=72), device=gpu, graph=graph, conv=conv)
    for i in range(steps):
        g = torch.Generator(device=gpu).manual_seed(1000 + i)
        x = X[i % 8] + 0.05 * torch.randn(X[i % 8].shape, generator=g, device=gpu)
        tr.step(x, Y[i % 8])
    torch.cuda.synchronize()
    ls = [round(v, 4) for _, v in tr.loss_log.flush()]
    print(conv, "graph" if graph else "eager", ls[::10], flush=True)
