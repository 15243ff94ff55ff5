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

    def forward(self, x, tag=""):
        P = _unflat(self.params, W.CLIENT_KEYS)
        xs = x.double().numpy()
        cut, rec = W.client_forward(P, xs, bf=False)
        self._saved = getattr(self, "_saved", {})
        self._saved[tag] = (xs, rec)
        return torch.from_numpy(cut).contiguous()

    def backward_grads(self, dcut, tag="", accumulate=False):
        P = _unflat(self.params, W.CLIENT_KEYS)
        xs, rec = self._saved[tag]
        g, _ = W.client_backward(P, xs, rec, dcut.double().numpy(), bf=False)
        gt = torch.from_numpy(np.concatenate([np.asarray(g[k]).reshape(-1) for k in W.CLIENT_KEYS]))
        if accumulate:
            self.grads += gt
        else:
            self.grads.copy_(gt)

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

    def accumulate(self, cut, labels, grad_scale, b0, k, nparts, dcut=None):
        P = _unflat(self.params, W.SERVER_KEYS)
        n = cut.shape[0]
        keep = W.dropout_keep(self.seed, self.opt.t, n, b0=b0)
        s = W.server_step(P, cut.double().numpy(), labels.numpy(), keep, grad_scale_batch=1.0 / grad_scale, bf=False)
        g = np.concatenate([s["grads"][key].reshape(-1) for key in W.SERVER_KEYS])
        self._g = g if k == 0 else self._g + g
        self._parts = ([] if k == 0 else self._parts) + [s["loss_i"].sum() * grad_scale]
        out = torch.from_numpy(s["dcut"]).contiguous()
        if dcut is not None:
            dcut.copy_(out)
            return dcut
        return out

    def finish_step(self, nparts, step=None):
        self.params = torch.from_numpy(self.opt.step(self.params.numpy(), self._g))
        self.losses.append((step, float(np.sum(self._parts))))

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
