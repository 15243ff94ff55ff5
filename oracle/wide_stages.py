"""ORACLE — TEST INFRASTRUCTURE ONLY. CPU (numpy float64) stand-ins for splitcnn.wide's
WideClientStage / WideServerStage with the interface dist.WideHub drives, so the widened SplitFed
protocol (gloo, world_size 3) can be checked on the CPU against the single-process widened step of
oracle/wide_step.py (bf16 roundings off: the protocol, not the rounding, is under test)."""
from __future__ import annotations

import numpy as np
import torch

from . import wide_step as W


def _flat(d, keys):
    return torch.from_numpy(np.concatenate([np.asarray(d[k], dtype=np.float64).reshape(-1) for k in keys]))


def _unflat(t, keys):
    out, off = {}, 0
    a = t.detach().cpu().numpy()
    for k in keys:
        n = int(np.prod(W.PARAM_SHAPES[k]))
        out[k] = a[off:off + n].reshape(W.PARAM_SHAPES[k])
        off += n
    return out


class _Adam:
    def __init__(self, n):
        self.m = np.zeros(n)
        self.v = np.zeros(n)
        self.t = 0

    def step(self, p, g):
        self.t += 1
        p2, self.m, self.v = W.adam(p, g, self.m, self.v, self.t, f32=False)
        return p2


class OracleWideClient:
    cut_dtype = torch.float64

    def __init__(self, params):
        self.params = _flat(params, W.CLIENT_KEYS)
        self.grads = torch.zeros_like(self.params)
        self.opt = _Adam(self.params.numel())

    @staticmethod
    def cut_shape(B):
        return (B, 256, 8, 8)

    def forward(self, x):
        P = _unflat(self.params, W.CLIENT_KEYS)
        self._x = x.double().numpy()
        cut, self._rec = W.client_forward(P, self._x, bf=False)
        return torch.from_numpy(cut).contiguous()

    def backward_grads(self, dcut):
        P = _unflat(self.params, W.CLIENT_KEYS)
        g, _ = W.client_backward(P, self._x, self._rec, dcut.double().numpy(), bf=False)
        self.grads.copy_(torch.from_numpy(np.concatenate([np.asarray(g[k]).reshape(-1) for k in W.CLIENT_KEYS])))

    def step_from_grads(self):
        self.params = torch.from_numpy(self.opt.step(self.params.numpy(), self.grads.numpy()))

    def named(self):
        return _unflat(self.params, W.CLIENT_KEYS)


class OracleWideServer:
    def __init__(self, params, seed=0):
        self.params = _flat(params, W.SERVER_KEYS)
        self.opt = _Adam(self.params.numel())
        self.seed = seed
        self.losses = []

    def step_request(self, cuts, labels, step=None):
        P = _unflat(self.params, W.SERVER_KEYS)
        G = cuts.shape[0]
        keep = W.dropout_keep(self.seed, self.opt.t, G)
        s = W.server_step(P, cuts.double().numpy(), labels.numpy(), keep, bf=False)
        g = np.concatenate([s["grads"][k].reshape(-1) for k in W.SERVER_KEYS])
        self.params = torch.from_numpy(self.opt.step(self.params.numpy(), g))
        self.losses.append((step, s["loss"]))
        return torch.from_numpy(s["dcut"]).contiguous(), torch.from_numpy(s["loss_i"])

    def named(self):
        return _unflat(self.params, W.SERVER_KEYS)
