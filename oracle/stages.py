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

    def backward(self, cut_grad, x=None, act=None, accumulate=False):
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

    def compute(self, act, labels, grad_scale, accumulate=False, cut_grad=None):
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
