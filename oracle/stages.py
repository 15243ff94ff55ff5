"""ORACLE — TEST INFRASTRUCTURE ONLY. CPU (numpy float64) stand-ins for engine.ClientStage /
engine.ServerStage with the interface the topologies in splitcnn/dist.py drive, so the multi-rank
protocols (gloo, world_size 2-3) can be checked on the CPU against the single-process oracle step.
The math is oracle/split_step.py (src/client_part.py:112-133, src/server_part.py:38-58)."""
from __future__ import annotations

import numpy as np
import torch

from . import split_step as O

KEYS_C = ["W1", "b1"]
KEYS_S = ["W2", "b2", "W3", "b3"]
SHAPES = {"W1": (32, 1, 3, 3), "b1": (32,), "W2": (64, 32, 3, 3), "b2": (64,), "W3": (10, 9216), "b3": (10,)}


def _flat(d, keys):
    return torch.from_numpy(np.concatenate([np.asarray(d[k], dtype=np.float64).reshape(-1) for k in keys]))


def _unflat(t, keys):
    out, off = {}, 0
    a = t.detach().cpu().numpy()
    for k in keys:
        n = int(np.prod(SHAPES[k]))
        out[k] = a[off:off + n].reshape(SHAPES[k])
        off += n
    return out


class OracleClient:
    def __init__(self, params, lr=O.LR):
        self.params = _flat(params, KEYS_C)
        self.grads = torch.zeros_like(self.params)
        self.lr = lr
        self._x = self._act = None

    def bind_grads(self, view):
        view.copy_(self.grads)
        self.grads = view

    def forward(self, x, out=None):
        p = _unflat(self.params, KEYS_C)
        act = O.client_forward(x.double().numpy(), p["W1"], p["b1"])
        t = torch.from_numpy(act)
        if out is not None:
            out.copy_(t)
            t = out
        self._x, self._act = x, t
        return t

    def forward_images(self, x, act16, act_amax):
        """dist.Hub(images=True)'s client call, emulated for the protocol tests: the f32 act's bytes fill
        act16 (an x3 image sample has the same 86,528 bytes as an f32 cut sample) and act_amax takes
        the per-sample max; OracleServer.compute reads them back as the f32 act."""
        t = self.forward(x)
        act16.copy_(t.to(torch.float32).contiguous().view(-1).view(torch.uint8))
        act_amax.copy_(t.reshape(t.shape[0], -1).amax(dim=1).to(act_amax.dtype))

    def backward(self, cut_grad, x=None, act=None, accumulate=False):
        if act is None and x is not None:   # as engine.ClientStage: the mask re-derived from x
            p = _unflat(self.params, KEYS_C)
            act = torch.from_numpy(O.client_forward(x.double().numpy(), p["W1"], p["b1"]))
        x = self._x if x is None else x
        act = self._act if act is None else act
        dW, db = O.client_backward(x.double().numpy(), act.double().numpy(), cut_grad.double().numpy())
        g = torch.from_numpy(np.concatenate([dW.reshape(-1), db]))
        if accumulate:
            self.grads += g.to(self.grads.dtype)
        else:
            self.grads.copy_(g)

    def step(self):
        self.params -= self.lr * self.grads.to(self.params.dtype)

    def named(self):
        return _unflat(self.params, KEYS_C)


class OracleServer:
    def __init__(self, params, lr=O.LR):
        self.params = _flat(params, KEYS_S)
        self.grads = torch.zeros_like(self.params)
        self.lr = lr
        self.losses = []

    def bind_grads(self, view):
        view.copy_(self.grads)
        self.grads = view

    def compute(self, act, labels, grad_scale, accumulate=False, cut_grad=None, act16=None):
        if act is None:   # the image exchange, emulated: act16 carries the f32 act's bytes
            act = act16.view(torch.float32).view(-1, 32, 26, 26)
        p = _unflat(self.params, KEYS_S)
        r = O.server_step(act.double().numpy(), labels.numpy(), p["W2"], p["b2"], p["W3"], p["b3"],
                          grad_scale_batch=1.0 / grad_scale)
        g = torch.from_numpy(np.concatenate([r["dW2"].reshape(-1), r["db2"], r["dW3"].reshape(-1), r["db3"]]))
        if accumulate:
            self.grads += g.to(self.grads.dtype)
        else:
            self.grads.copy_(g)
        cut = torch.from_numpy(r["cut_grad"])
        if cut_grad is not None:
            cut_grad.copy_(cut)
            cut = cut_grad
        return cut, torch.from_numpy(r["loss_i"])

    def step(self):
        self.params -= self.lr * self.grads.to(self.params.dtype)

    def log_loss(self, values, scale=None, step=None):
        scale = 1.0 / values.numel() if scale is None else scale
        self.losses.append((step, float(values.double().sum() * scale)))

    def named(self):
        return _unflat(self.params, KEYS_S)


class OracleUServer:
    """conv2 trunk of the U-shape (splitcnn/ushaped.py UServerStage) in float64."""

    def __init__(self, params, lr=O.LR):
        self.params = _flat(params, ["W2", "b2"])
        self.lr = lr
        self._act = self._code = self._relu = None

    def forward(self, act):
        p = _unflat(self.params, ["W2", "b2"])
        a = act.double().numpy()
        r = O.relu(O.conv3x3(a, p["W2"], p["b2"]))
        pooled, idx = O.maxpool2(r)
        self._act, self._relu, self._code = a, r, O.route_code(pooled, idx)
        return torch.from_numpy(pooled)

    def backward_step(self, dpooled):
        p = _unflat(self.params, ["W2", "b2"])
        code = self._code
        dpool = np.where(code < O.CODE_NONE, dpooled.double().numpy(), 0.0)
        dc = O.maxpool2_bwd(dpool, np.minimum(code, 3), self._relu.shape)
        dW2, db2 = O.conv3x3_wgrad(self._act, dc)
        cut = O.conv3x3_dgrad(dc, p["W2"])
        self.params -= self.lr * torch.from_numpy(np.concatenate([dW2.reshape(-1), db2]))
        return torch.from_numpy(cut)

    def named(self):
        return _unflat(self.params, ["W2", "b2"])


class OracleUClient:
    """conv1 + fc1 head + CE of the U-shape (splitcnn/ushaped.py UClientStage) in float64."""

    def __init__(self, params, lr=O.LR):
        self.conv = OracleClient(params, lr)
        self.params = _flat(params, ["W3", "b3"])
        self.lr = lr
        self.losses = []

    def forward(self, x):
        return self.conv.forward(x)

    def head_step(self, pooled, labels, step=None):
        p = _unflat(self.params, ["W3", "b3"])
        pl = pooled.double().numpy()
        B = pl.shape[0]
        flat = pl.reshape(B, -1)
        loss, _, dlogits = O.cross_entropy(flat @ p["W3"].T + p["b3"], labels.numpy())
        dflat = dlogits @ p["W3"]
        g = np.concatenate([(dlogits.T @ flat).reshape(-1), dlogits.sum(axis=0)])
        self.params -= self.lr * torch.from_numpy(g)
        self.losses.append((step, float(loss)))
        return torch.from_numpy(dflat.reshape(pl.shape))

    def backward_step(self, cut_grad):
        self.conv.backward(cut_grad)
        self.conv.step()

    def named(self):
        return {**self.conv.named(), **_unflat(self.params, ["W3", "b3"])}
