"""The north star's fp32 parity run at the K2 batch, pinned to an INDEPENDENT float64 restatement.

100 steps of the default SplitTrainer (BASELINE config 2: B = 4096, x3 conv2 kernels, the client's
split images, the client backward fused into the dgrad, one HIP graph per step) against a float64
torch restatement of the reference's split step on the same batches, built from tests/ref64.py's conv
pieces (unfold + float64 matmul: no MIOpen, no reduced precision) plus float64 conv1, fc1, softmax
cross-entropy and SGD — src/model_def.py:8-28 forward, src/server_part.py:47-52 (loss, backward,
SGD on the server), src/client_part.py:132-133 (the client's backward + SGD). Neither side shares
code with the other: the float64 side never calls libslk.

Bars: every step's loss within 1e-4 relative; after 100 steps each parameter
tensor's update (w_100 - w_0) within 1e-3 of its largest element; and at every step every window
whose routing code (the kernel's, from its own inputs) differs from float64's is a numerical tie
(ref64.assert_routing_ties on the step's pre-update weights).
"""
import numpy as np
import pytest
import torch
import torch.nn.functional as F

from ref64 import assert_routing_ties, conv_relu64, dgrad64, route64, routing64, wgrad64

pytestmark = pytest.mark.gpu

CH = 512  # float64 conv chunk (samples)


class Ref64:
    """The reference split step in float64 on the GPU (state: W1 b1 W2 b2 W3 b3, SGD lr 0.01)."""

    def __init__(self, client, server, dev):
        sd = {**client.state_dict(), **server.state_dict()}
        self.p = {k: sd[m].detach().to(dev, torch.float64).clone() for k, m in
                  (("W1", "conv1.weight"), ("b1", "conv1.bias"), ("W2", "conv2.weight"), ("b2", "conv2.bias"),
                   ("W3", "fc1.weight"), ("b3", "fc1.bias"))}

    def step(self, x, y, lr=0.01):
        p = self.p
        B = x.shape[0]
        # client forward: act = relu(conv1(x))   (model_def.py:11-12)
        xc = F.unfold(x.double(), 3)                                             # B, 9, 676
        act = (torch.matmul(p["W1"].reshape(32, 9), xc) + p["b1"][None, :, None]).clamp_min(0.0)
        act = act.reshape(B, 32, 26, 26)
        # server forward: conv2 + relu + pool (first max wins) + fc1   (model_def.py:25-28)
        pooled = torch.empty(B, 64, 12, 12, dtype=torch.float64, device=x.device)
        code = torch.empty(B, 64, 12, 12, dtype=torch.long, device=x.device)
        for s in range(0, B, CH):
            c, win = routing64(conv_relu64(act[s:s + CH], p["W2"], p["b2"]))
            code[s:s + CH] = c
            pooled[s:s + CH] = win.max(-1).values
        flat = pooled.reshape(B, 9216)
        z = flat @ p["W3"].t() + p["b3"]
        # mean cross-entropy and its gradient   (server_part.py:16,49-51)
        lse = torch.logsumexp(z, 1)
        loss = (lse - z.gather(1, y[:, None])[:, 0]).mean()
        dz = torch.softmax(z, 1)
        dz[torch.arange(B, device=x.device), y] -= 1.0
        dz /= B
        gW3, gb3 = dz.t() @ flat, dz.sum(0)
        dpooled = dz @ p["W3"]
        gW2 = torch.zeros_like(p["W2"])
        gb2 = torch.zeros_like(p["b2"])
        gW1 = torch.zeros(32, 9, dtype=torch.float64, device=x.device)
        gb1 = torch.zeros_like(p["b1"])
        for s in range(0, B, CH):
            dc = route64(dpooled[s:s + CH], code[s:s + CH])
            w, b = wgrad64(act[s:s + CH], dc)
            gW2 += w
            gb2 += b
            # the cut gradient and the client's backward: relu mask, conv1 weight gradient (client_part.py:132)
            g = dgrad64(dc, p["W2"]) * (act[s:s + CH] > 0)
            gr = g.reshape(-1, 32, 676)
            gW1 += torch.matmul(gr, xc[s:s + CH].transpose(1, 2)).sum(0)
            gb1 += gr.sum((0, 2))
        for k, gk in (("W1", gW1.reshape(32, 1, 3, 3)), ("b1", gb1), ("W2", gW2), ("b2", gb2), ("W3", gW3), ("b3", gb3)):
            p[k] -= lr * gk
        return float(loss)


def test_trajectory_100_steps_b4096_vs_float64(gpu):
    from splitcnn import ops
    from splitcnn.data import SyntheticMNIST, init_models
    from splitcnn.engine import SplitTrainer
    B, steps = 4096, 100
    data = SyntheticMNIST(71)
    xs, ys = zip(*(data.batch(B) for _ in range(8)))
    X, Y = torch.stack(xs).to(gpu), torch.stack(ys).to(gpu)
    a, b = init_models(seed=72)
    ref = Ref64(a, b, gpu)
    init64 = {k: v.clone() for k, v in ref.p.items()}
    tr = SplitTrainer(a, b, device=gpu, graph=True)
    assert tr.server.impl_fwd == tr.server.impl_dgrad == tr.server.impl_wgrad == "x3"
    assert tr.client.emit_act16 and tr.fuse_client_backward
    c0, s0 = tr.client.params.clone(), tr.server.params.clone()
    losses, want, ties = [], [], 0
    for i in range(steps):
        g = torch.Generator(device=gpu).manual_seed(1000 + i)
        x = X[i % 8] + 0.05 * torch.randn(X[i % 8].shape, generator=g, device=gpu)
        W1, b1 = tr.client.params[:288].view(32, 1, 3, 3).clone(), tr.client.params[288:].clone()
        W2, b2 = tr.server.params[:18432].view(64, 32, 3, 3).clone(), tr.server.params[18432:18496].clone()
        tr.step(x, Y[i % 8])
        want.append(ref.step(x, Y[i % 8]))
        # the step's routing (the kernel's code for its own inputs) vs float64 on the same inputs
        code = tr.server._buf.get("code", (B, 64, 12, 12), torch.uint8, gpu)
        act = ops.conv1_fwd(x, W1, b1)
        ties += assert_routing_ties(act, W2, b2, code)
        if (i + 1) % 25 == 0:
            losses += [l for _, l in tr.loss_log.flush()]
    torch.cuda.synchronize()
    lx, lw = np.array(losses), np.array(want)
    assert len(lx) == steps
    rel = np.abs(lx - lw) / np.abs(lw)
    assert rel.max() <= 1e-4, (rel.max(), int(rel.argmax()), lx[-1], lw[-1])
    assert lx[-1] < 0.5 * lx[0]  # it trains
    dc = (tr.client.params - c0).double()
    ds = (tr.server.params - s0).double()
    got = {"W1": dc[:288], "b1": dc[288:], "W2": ds[:18432], "b2": ds[18432:18496], "W3": ds[18496:110656],
           "b3": ds[110656:]}
    for k, d in got.items():
        r = (ref.p[k] - init64[k]).reshape(-1)
        err = float((d - r).abs().max() / r.abs().max())
        assert err <= 1e-3, (k, err)
    print(f"100 steps: max loss rel {rel.max():.2e}; routing differences (all ties) {ties}")
