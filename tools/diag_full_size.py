"""Diagnostics for the B=4096 parity checks (round 3): (1) the routing differences between the x3 and
the direct f32 forward that are not ties at rtol 1e-5 — which one matches float64; (2) db1 / dW1 error
of every client-gradient path against float64."""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "split-learning-k8s_amd"), ROOT, os.path.join(ROOT, "tests")]
from ref64 import conv_relu64, dgrad64, route64  # noqa: E402
from test_x3_gpu import _c1_ref64, _inputs, _relu_bits  # noqa: E402

from splitcnn import ops  # noqa: E402
from splitcnn.data import SyntheticMNIST, init_models  # noqa: E402

gpu = torch.device("cuda:0")
B = 4096
act, p, _ = _inputs(gpu, B, seed=21)
px, cx = ops.conv2_fwd_pool(act, p["W2"], p["b2"], impl="x3")
pd, cd = ops.conv2_fwd_pool(act, p["W2"], p["b2"], impl="direct")
pw, cw = ops.conv2_fwd_pool(act, p["W2"], p["b2"], impl="wino")
diff = cx != cd
bad = diff.flatten(1).any(1).nonzero().flatten()
print("mismatched windows x3 vs direct:", int(diff.sum()), "samples", bad.numel(), " wino vs direct:", int((cw != cd).sum()))
r = conv_relu64(act[bad], p["W2"], p["b2"])
win = r.reshape(-1, 64, 12, 2, 12, 2).permute(0, 1, 2, 4, 3, 5).reshape(-1, 64, 12, 12, 4)
scale = r.abs().max().item()
d = diff[bad]
w = win[d]
a, bb = cx[bad][d].long(), cd[bad][d].long()
mx = w.max(-1).values
va = torch.where(a < 4, w.gather(-1, a.clamp_max(3)[:, None])[:, 0], torch.zeros_like(mx))
vb = torch.where(bb < 4, w.gather(-1, bb.clamp_max(3)[:, None])[:, 0], torch.zeros_like(mx))
# fp64 routing
best, idx = w[:, 0].clone(), torch.zeros_like(a)
for q in range(1, 4):
    bt = w[:, q] > best
    best = torch.where(bt, w[:, q], best)
    idx = torch.where(bt, torch.full_like(idx, q), idx)
c64 = torch.where(best > 0, idx, torch.full_like(idx, 4))
# per-window the x3 and direct conv values
cvx = None
for i in range(w.shape[0]):
    gap = (va[i] - vb[i]).abs().item()
    tol = 1e-5 * max(abs(mx[i].item()), 1e-3 * scale)
    tag = "TIE" if gap <= tol else "NOT-TIE"
    if tag == "NOT-TIE" or i < 5:
        print(f"{tag} x3={a[i].item()} direct={bb[i].item()} fp64={c64[i].item()} window={w[i].tolist()} "
              f"gap/scale={gap / scale:.3e} mx/scale={mx[i].item() / scale:.3e}")
print("pooled err vs fp64 / scale: x3", (px.double()[bad] - win.max(-1).values).abs().max().item() / scale,
      "direct", (pd.double()[bad] - win.max(-1).values).abs().max().item() / scale)

# (2) client gradient paths vs fp64
a_, b_ = init_models(seed=61)
x, y = SyntheticMNIST(62).batch(B)
x, y = x.to(gpu), y.to(gpu)
W1, b1 = a_.conv1.weight.detach().to(gpu), a_.conv1.bias.detach().to(gpu)
W2, b2 = b_.conv2.weight.detach().to(gpu), b_.conv2.bias.detach().to(gpu)
W3, b3 = b_.fc1.weight.detach().to(gpu), b_.fc1.bias.detach().to(gpu)
am = torch.empty(B, device=gpu)
act = ops.conv1_fwd(x, W1, b1, act_amax=am)
px, cx = ops.conv2_fwd_pool(act, W2, b2, impl="x3", act_amax=am)
dpa = torch.empty(B, device=gpu)
_, _, _, dp = ops.fc_xent(px, W3, b3, y, 1.0 / B, dp_amax=dpa)
g64 = dgrad64(route64(dp, cx), W2)
ref = torch.from_numpy(_c1_ref64(x, W1, b1, g64))
paths = {
    "fused_x3": ops.reduce_slabs(ops.conv2_dgrad_client_slabs(dp, cx, W2, x, _relu_bits(x, W1, b1), dp_amax=dpa)),
    "x3_then_remask": ops.reduce_slabs(ops.conv1_wgrad_remask_slabs(x, W1, b1, ops.conv2_dgrad(dp, cx, W2, impl="x3", dp_amax=dpa))),
    "direct_then_remask": ops.reduce_slabs(ops.conv1_wgrad_remask_slabs(x, W1, b1, ops.conv2_dgrad(dp, cx, W2, impl="direct"))),
    "wino_then_remask": ops.reduce_slabs(ops.conv1_wgrad_remask_slabs(x, W1, b1, ops.conv2_dgrad(dp, cx, W2, impl="wino"))),
    "fp64g_f32_then_remask": ops.reduce_slabs(ops.conv1_wgrad_remask_slabs(x, W1, b1, g64.float().contiguous())),
}
for k, v in paths.items():
    v = v.double().cpu()
    e1 = (v[:288] - ref[:288]).abs().max().item() / ref[:288].abs().max().item()
    e2 = (v[288:] - ref[288:]).abs().max().item() / ref[288:].abs().max().item()
    print(f"{k:24s} dW1 {e1:.3e}  db1 {e2:.3e}")
gx = ops.conv2_dgrad(dp, cx, W2, impl="x3", dp_amax=dpa).double()
gd = ops.conv2_dgrad(dp, cx, W2, impl="direct").double()
print("cut grad: x3 err", ((gx - g64).abs().max() / g64.abs().max()).item(), "direct", ((gd - g64).abs().max() / g64.abs().max()).item())
print("cut grad signed mean err / mean|g|: x3", ((gx - g64).mean() / g64.abs().mean()).item(),
      "direct", ((gd - g64).mean() / g64.abs().mean()).item())
print("sum g vs sum|g|:", g64.sum().item(), g64.abs().sum().item())
