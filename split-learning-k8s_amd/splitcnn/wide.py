"""Widened split CNN — BASELINE.json config 5 ("K5"): 64-256 channels, synthetic 3x32x32 batches,
deeper cut, bf16 MFMA implicit-GEMM convolutions, with the north star's dropout and Adam.

The reference has no such model; this keeps its step contract
(src/client_part.py:110-138 <-> src/server_part.py:25-58: activations out, cut gradient back, loss
logged, one optimizer step per side per request) and its module style (src/model_def.py:5-71:
client/server halves + a full model + a role factory) for a network whose convolutions are real
contractions:

  WideModelPartA (client)  conv1 3->64 3x3 p1 + ReLU; conv2 64->128 + ReLU + maxpool2;
                           conv3 128->256 + ReLU + maxpool2  -> cut [B,256,8,8]
  WideModelPartB (server)  Dropout(0.25) -> flatten -> fc Linear(16384, 10); CrossEntropyLoss(mean)
  optimiser                torch.optim.Adam(lr=1e-3) on both sides

The cut is client-heavy by construction (99.9 % of the FLOPs are on the client side), so SplitFed
with N-1 client GPUs feeding one server GPU scales (SURVEY.md §7 "server-bound scaling").
Numerics (bf16 activations and conv operands, f32 accumulation, f32 masters/head/Adam) are stated in
oracle/wide_step.py, which the GPU parity tests hold this path to.

Every op runs on the gfx950 kernels of libslk.so (csrc/slk_wide.hip, csrc/slk_wide_head.hip);
there is no CPU path. Activations live in HBM in the C8 layout [B][C/8][H][W][8] (bf16);
`c8_to_nchw` gives the logical NCHW view.
"""
from __future__ import annotations

import ctypes
import os
from typing import Optional

import numpy as np
import torch
import torch.nn as nn

from . import _lib
from .engine import TIMER, LossLog, _Buffers
from .ops import _dev, _stream

P_DROP = 0.25
KEEP_THRESHOLD = int(round(P_DROP * 4294967296.0))          # keep iff hash >= p * 2^32
KEEP_SCALE = float(np.float32(1.0 / (1.0 - P_DROP)))        # f32(1/(1-p)), as torch's dropout
LR, BETA1, BETA2, EPS = 1e-3, 0.9, 0.999, 1e-8
CLIENT_NPARAM = 370816   # [W1 1728 | b1 64 | W2 73728 | b2 128 | W3 294912 | b3 256]
SERVER_NPARAM = 163850   # [Wf 163840 | bf 10]
CUT_SHAPE = (32, 8, 8, 8)  # C8 layout of [256, 8, 8]
_BF = torch.bfloat16
_U8 = torch.uint8
_F32 = torch.float32


# ------------------------------------------------------------------------------------ modules
class WideModelPartA(nn.Module):
    """Client bottom stack of the widened split CNN (parameter container; kernels in WideClientStage)."""

    def __init__(self):
        super().__init__()
        self.conv1 = nn.Conv2d(3, 64, 3, 1, padding=1)
        self.conv2 = nn.Conv2d(64, 128, 3, 1, padding=1)
        self.conv3 = nn.Conv2d(128, 256, 3, 1, padding=1)
        self.relu = nn.ReLU()
        self.pool = nn.MaxPool2d(2)

    def forward(self, x):
        raise RuntimeError("splitcnn.WideModelPartA runs through WideClientStage / WideTrainer on the "
                           "MI355X HIP kernels; there is no CPU or eager-torch path")


class WideModelPartB(nn.Module):
    """Server top stack: Dropout(0.25) -> flatten -> Linear(16384, 10)."""

    def __init__(self):
        super().__init__()
        self.dropout = nn.Dropout(P_DROP)
        self.flatten = nn.Flatten()
        self.fc = nn.Linear(256 * 8 * 8, 10)

    def forward(self, x):
        raise RuntimeError("splitcnn.WideModelPartB runs through WideServerStage / WideTrainer on the "
                           "MI355X HIP kernels; there is no CPU or eager-torch path")


class WideFullModel(nn.Module):
    """The unsplit widened network; parameter names = A ∪ B (like FullModel, src/model_def.py:31-46)."""

    def __init__(self):
        super().__init__()
        a, b = WideModelPartA(), WideModelPartB()
        self.conv1, self.conv2, self.conv3 = a.conv1, a.conv2, a.conv3
        self.dropout, self.fc = b.dropout, b.fc

    def forward(self, x):
        raise RuntimeError("splitcnn.WideFullModel runs through WideTrainer on the MI355X HIP kernels")


def get_wide_model(role="client"):
    """Role factory in the style of get_model (src/model_def.py:49-71)."""
    mode = os.getenv("LEARNING_MODE", "split").lower()
    if mode == "federated":
        return WideFullModel()
    if mode == "split":
        return WideModelPartA() if role == "client" else WideModelPartB()
    raise ValueError(f"Unknown LEARNING_MODE: {mode}. Use 'split' or 'federated'.")


def init_wide_models(seed: int = 0):
    """Seeded default init, client (conv1, conv2, conv3) then server (fc)."""
    torch.manual_seed(seed)
    return WideModelPartA(), WideModelPartB()


class SyntheticCIFAR:
    """CIFAR-shape synthetic batches: class prototypes + noise, normalised (mean 0.5, std 0.25);
    seeded CPU generator (bit-identical everywhere, like data.SyntheticMNIST)."""

    def __init__(self, seed: int = 42):
        self.gen = torch.Generator().manual_seed(seed)
        self.proto = torch.rand(10, 3, 32, 32, generator=self.gen)

    def batch(self, B: int):
        y = torch.randint(0, 10, (B,), generator=self.gen)
        x = (self.proto[y] + 0.3 * torch.randn(B, 3, 32, 32, generator=self.gen) - 0.5) / 0.25
        return x.contiguous(), y


def c8_to_nchw(t: torch.Tensor) -> torch.Tensor:
    """[B, C/8, H, W, 8] -> logical [B, C, H, W] (a permuted copy)."""
    B, C8, H, W, _ = t.shape
    return t.permute(0, 1, 4, 2, 3).reshape(B, C8 * 8, H, W)


def nchw_to_c8(t: torch.Tensor) -> torch.Tensor:
    B, C, H, W = t.shape
    return t.reshape(B, C // 8, 8, H, W).permute(0, 1, 3, 4, 2).contiguous()


def _flat(params, device):
    n = sum(p.numel() for p in params)
    flat = torch.empty(n, dtype=_F32, device=device)
    grad = torch.zeros(n, dtype=_F32, device=device)
    off = 0
    for p in params:
        k = p.numel()
        flat[off:off + k].copy_(p.detach().reshape(-1).to(device=device, dtype=_F32))
        p.data = flat[off:off + k].view(p.shape)
        p.grad = grad[off:off + k].view(p.shape)
        off += k
    return flat, grad


def _q(name, *args):
    return _lib.query(name, *args)


def _k(name, *args):
    """Launch slk_<name> under the (optional) HIP-event kernel timer."""
    with TIMER(name):
        _lib.call("slk_" + name, *args)


# ------------------------------------------------------------------------------------ stages
class WideClientStage:
    """Client half: forward(x) -> cut (bf16 C8); backward_step(dcut) = activations.backward(grads) +
    Adam (client_part.py:114,132-133 for the widened model)."""

    OFF = {"W1": 0, "b1": 1728, "W2": 1792, "b2": 75520, "W3": 75648, "b3": 370560}

    def __init__(self, model: Optional[WideModelPartA] = None, device="cuda", lr=LR, betas=(BETA1, BETA2),
                 eps=EPS):
        self.device = torch.device(device)
        self.model = (model if model is not None else WideModelPartA()).to(self.device)
        m = self.model
        self.params, self.grads = _flat([m.conv1.weight, m.conv1.bias, m.conv2.weight, m.conv2.bias,
                                         m.conv3.weight, m.conv3.bias], self.device)
        assert self.params.numel() == CLIENT_NPARAM
        self.m = torch.zeros_like(self.params)
        self.v = torch.zeros_like(self.params)
        self.step_ctr = torch.zeros(1, dtype=torch.int32, device=self.device)
        self.lr, self.betas, self.eps = lr, betas, eps
        self.fuse_adam = True  # step_from_slabs: the three Adam segments in one launch
        self.w1b = torch.empty(64 * 32, dtype=_BF, device=self.device)
        self.w2f = torch.empty(73728, dtype=_BF, device=self.device)
        self.w2d = torch.empty(73728, dtype=_BF, device=self.device)
        self.w3f = torch.empty(294912, dtype=_BF, device=self.device)
        self.w3d = torch.empty(294912, dtype=_BF, device=self.device)
        self._buf = _Buffers()
        self._saved = {}
        self.refresh_shadows()

    def _b(self, name, shape, dtype):
        return self._buf.get(name, shape, dtype, self.device)

    def _p(self, k, n):
        o = self.OFF[k]
        return self.params[o:o + n]

    def refresh_shadows(self):
        """Rebuild the bf16 conv weight shadows from the f32 masters (after load_state_dict or Adam)."""
        W2, W3 = self._p("W2", 73728), self._p("W3", 294912)
        _k("wide_shadows", self._p("W1", 1728).data_ptr(), W2.data_ptr(), W3.data_ptr(), self.w1b.data_ptr(),
           self.w2f.data_ptr(), self.w2d.data_ptr(),
                  self.w3f.data_ptr(), self.w3d.data_ptr(), _stream(self.params))

    def forward(self, x: torch.Tensor, out: Optional[torch.Tensor] = None, tag="") -> torch.Tensor:
        """cut = client forward of x; `tag` keeps separate saved tensors per micro-batch."""
        B = x.shape[0]
        _dev(x, "x", (B, 3, 32, 32))
        s = _stream(x)
        a1 = self._b(f"a1{tag}", (B, 8, 32, 32, 8), _BF)
        p2 = self._b(f"p2{tag}", (B, 16, 16, 16, 8), _BF)
        code2 = self._b(f"code2{tag}", (B, 16, 16, 16, 8), _U8)
        cut = out if out is not None else self._b(f"cut{tag}", (B,) + CUT_SHAPE, _BF)
        _dev(cut, "cut", (B,) + CUT_SHAPE, _BF)
        code3 = self._b(f"code3{tag}", (B,) + CUT_SHAPE, _U8)
        _k("wide_conv1_fwd", x.data_ptr(), self.w1b.data_ptr(), self._p("b1", 64).data_ptr(), a1.data_ptr(), B, s)
        _k("wide_conv2_fwd", a1.data_ptr(), self.w2f.data_ptr(), self._p("b2", 128).data_ptr(),
                  p2.data_ptr(), code2.data_ptr(), B, s)
        _k("wide_conv3_fwd", p2.data_ptr(), self.w3f.data_ptr(), self._p("b3", 256).data_ptr(),
                  cut.data_ptr(), code3.data_ptr(), B, s)
        self._x, self._a1, self._p2, self._code2, self._code3 = x, a1, p2, code2, code3
        self._saved[tag] = (x, a1, p2, code2, code3)
        return cut

    def backward_slabs(self, dcut: torch.Tensor, tag=""):
        """Client backward into three slab sets (conv3, conv2, conv1); returns them."""
        B = dcut.shape[0]
        _dev(dcut, "dcut", (B,) + CUT_SHAPE, _BF)
        self._x, self._a1, self._p2, self._code2, self._code3 = self._saved[tag]
        s = _stream(dcut)
        dc3 = self._b("dc3", (B, 32, 16, 16, 8), _BF)
        dc2 = self._b("dc2", (B, 16, 32, 32, 8), _BF)
        da1m = self._b("da1m", (B, 8, 32, 32, 8), _BF)
        s3 = self._b("s3", (_q("slk_wide_conv3_wgrad_nslab", B), 294912 + 256), _F32)
        s2 = self._b("s2", (_q("slk_wide_conv2_wgrad_nslab", B), 73728 + 128), _F32)
        s1 = self._b("s1", (_q("slk_wide_conv1_wgrad_nslab", B), 1728 + 64), _F32)
        _k("wide_unpool", dcut.data_ptr(), self._code3.data_ptr(), dc3.data_ptr(), B, s)
        _k("wide_conv3_wgrad", dc3.data_ptr(), self._p2.data_ptr(), s3.data_ptr(), B, s)
        _k("wide_conv3_dgrad", dc3.data_ptr(), self.w3d.data_ptr(), self._code2.data_ptr(),
                  dc2.data_ptr(), B, s)
        _k("wide_conv2_wgrad", dc2.data_ptr(), self._a1.data_ptr(), s2.data_ptr(), B, s)
        _k("wide_conv2_dgrad", dc2.data_ptr(), self.w2d.data_ptr(), self._a1.data_ptr(),
                  da1m.data_ptr(), B, s)
        _k("wide_conv1_wgrad", self._x.data_ptr(), da1m.data_ptr(), s1.data_ptr(), B, s)
        self._dc3, self._dc2, self._da1m = dc3, dc2, da1m
        return s1, s2, s3

    def _adam(self, lo, n, slabs):
        s = _stream(slabs)
        _k("adam_from_slabs", self.params[lo:].data_ptr(), self.grads[lo:].data_ptr(),
                  self.m[lo:].data_ptr(), self.v[lo:].data_ptr(), slabs.data_ptr(), slabs.shape[0], n,
                  float(self.lr), float(self.betas[0]), float(self.betas[1]), float(self.eps),
                  self.step_ctr.data_ptr(), s)

    def step_from_slabs(self, s1, s2, s3):
        """Adam on all client parameters from the three slab sets (ONE launch, bit-identical to one
        slk_adam_from_slabs per set), then shadows + step counter."""
        if self.fuse_adam:
            P, I = ctypes.c_void_p, ctypes.c_int
            segs = ((0, 1792, s1), (1792, 73856, s2), (75648, 295168, s3))
            arr = lambda ts: ctypes.cast((P * 3)(*ts), P)  # noqa: E731
            _k("adam_multi_from_slabs", arr([self.params[lo:].data_ptr() for lo, _, _ in segs]),
               arr([self.grads[lo:].data_ptr() for lo, _, _ in segs]),
               arr([self.m[lo:].data_ptr() for lo, _, _ in segs]), arr([self.v[lo:].data_ptr() for lo, _, _ in segs]),
               arr([sl.data_ptr() for _, _, sl in segs]), ctypes.cast((I * 3)(*[sl.shape[0] for _, _, sl in segs]), P),
               ctypes.cast((I * 3)(*[n for _, n, _ in segs]), P), 3, float(self.lr), float(self.betas[0]),
               float(self.betas[1]), float(self.eps), self.step_ctr.data_ptr(), _stream(self.params))
        else:
            self._adam(0, 1792, s1)
            self._adam(1792, 73856, s2)
            self._adam(75648, 295168, s3)
        self.refresh_shadows()
        _k("tick", self.step_ctr.data_ptr(), _stream(self.params))

    def backward_step(self, dcut: torch.Tensor):
        self.step_from_slabs(*self.backward_slabs(dcut))

    # --- multi-GPU (dist.WideHub): gradient into self.grads, all-reduced by the caller, then Adam
    cut_dtype = _BF

    @staticmethod
    def cut_shape(B: int):
        return (B,) + CUT_SHAPE

    def backward_grads(self, dcut: torch.Tensor, tag="", accumulate: bool = False):
        """activations.backward(grads) into the flat gradient block (fixed-order slab reduction);
        accumulate=True adds (micro-batches of one step)."""
        s1, s2, s3 = self.backward_slabs(dcut, tag)
        st = _stream(dcut)
        for lo, n, sl in ((0, 1792, s1), (1792, 73856, s2), (75648, 295168, s3)):
            with TIMER("reduce_slabs"):
                _lib.call("slk_reduce_slabs", sl.data_ptr(), sl.shape[0], n, self.grads[lo:].data_ptr(),
                          int(bool(accumulate)), st)

    def step_from_grads(self):
        """Adam from self.grads (e.g. after an all-reduce over the client ranks)."""
        g = self.grads
        _k("adam_from_slabs", self.params.data_ptr(), None, self.m.data_ptr(), self.v.data_ptr(), g.data_ptr(), 1,
           CLIENT_NPARAM, float(self.lr), float(self.betas[0]), float(self.betas[1]), float(self.eps),
           self.step_ctr.data_ptr(), _stream(g))
        self.refresh_shadows()
        _k("tick", self.step_ctr.data_ptr(), _stream(g))


class WideServerStage:
    """Server half: step_request(cut, labels, step) -> (dcut, loss_i): dropout + fc + CE forward and
    backward, Adam, loss logged to the device ring (server_part.py:38-58 for the widened model)."""

    def __init__(self, model: Optional[WideModelPartB] = None, device="cuda", lr=LR, betas=(BETA1, BETA2),
                 eps=EPS, seed: int = 0, loss_log: Optional[LossLog] = None):
        self.device = torch.device(device)
        self.model = (model if model is not None else WideModelPartB()).to(self.device)
        self.params, self.grads = _flat([self.model.fc.weight, self.model.fc.bias], self.device)
        assert self.params.numel() == SERVER_NPARAM
        self.m = torch.zeros_like(self.params)
        self.v = torch.zeros_like(self.params)
        self.step_ctr = torch.zeros(1, dtype=torch.int32, device=self.device)
        self.lr, self.betas, self.eps, self.seed = lr, betas, eps, int(seed)
        self.wf8 = torch.empty(163840, dtype=_F32, device=self.device)
        self.err_flag = torch.zeros(1, dtype=torch.int32, device=self.device)
        self.loss_log = loss_log if loss_log is not None else LossLog(self.device)
        self._buf = _Buffers()
        self.refresh_shadows()

    def _b(self, name, shape, dtype):
        return self._buf.get(name, shape, dtype, self.device)

    def refresh_shadows(self):
        _k("wide_fc_shadow", self.params.data_ptr(), self.wf8.data_ptr(), _stream(self.params))

    def forward_backward(self, cut, labels, grad_scale, dcut=None, b0: int = 0):
        B = cut.shape[0]
        _dev(cut, "cut", (B,) + CUT_SHAPE, _BF)
        _dev(labels, "labels", (B,), torch.int64)
        s = _stream(cut)
        logits = self._b("logits", (B, 10), _F32)
        loss_i = self._b("loss_i", (B,), _F32)
        dlogits = self._b("dlogits", (B, 10), _F32)
        dcut = dcut if dcut is not None else self._b("dcut", (B,) + CUT_SHAPE, _BF)
        _dev(dcut, "dcut", (B,) + CUT_SHAPE, _BF)
        sf = self._b("sf", (_q("slk_wide_head_nslab", B), SERVER_NPARAM), _F32)
        work = self._b("work", (_q("slk_wide_head_work", B),), _F32)
        _k("wide_head", cut.data_ptr(), self.wf8.data_ptr(), self.params[163840:].data_ptr(),
           labels.data_ptr(), self.step_ctr.data_ptr(), self.seed, KEEP_THRESHOLD, KEEP_SCALE,
           float(grad_scale), logits.data_ptr(), loss_i.data_ptr(), dlogits.data_ptr(), dcut.data_ptr(),
           sf.data_ptr(), work.data_ptr(), self.err_flag.data_ptr(), int(b0), B, s)
        self._logits, self._dlogits = logits, dlogits
        return dcut, loss_i, sf

    def step_from_slabs(self, sf):
        s = _stream(sf)
        _k("adam_from_slabs", self.params.data_ptr(), self.grads.data_ptr(), self.m.data_ptr(),
                  self.v.data_ptr(), sf.data_ptr(), sf.shape[0], SERVER_NPARAM, float(self.lr),
                  float(self.betas[0]), float(self.betas[1]), float(self.eps), self.step_ctr.data_ptr(), s)
        self.refresh_shadows()
        _k("tick", self.step_ctr.data_ptr(), s)

    def log_loss(self, loss_i, step=None):
        _k("loss_log", loss_i.data_ptr(), loss_i.numel(), 1.0 / loss_i.numel(),
                  self.loss_log.ring.data_ptr(), self.loss_log.ring.numel(), self.loss_log.counter.data_ptr(),
                  _stream(loss_i))
        if step is not None:
            self.loss_log.note_step(step)

    def step_request(self, cut, labels, step=None, dcut=None):
        """One /forward_pass for the widened model: returns (dcut, loss_i)."""
        B = cut.shape[0]
        dcut, loss_i, sf = self.forward_backward(cut, labels, 1.0 / B, dcut=dcut)
        self.log_loss(loss_i)
        self.step_from_slabs(sf)
        if step is not None:
            self.loss_log.note_step(step)
        return dcut, loss_i

    def check_labels(self):
        if int(self.err_flag.item()) != 0:
            raise IndexError("splitcnn: a label was out of range [0, 10)")

    # --- micro-batched / multi-client steps (dist.WideHub): accumulate, then one Adam step
    def accumulate(self, cut, labels, grad_scale: float, b0: int, k: int, nparts: int, dcut=None):
        """Head forward/backward for samples b0 .. b0+len(cut)-1 of the step's global batch (mean-loss
        scale grad_scale = 1/global batch); the fc gradient adds into self.grads (k = 0 starts it) and
        this part's loss sum lands in loss part k of nparts. Returns dcut."""
        dcut, loss_i, sf = self.forward_backward(cut, labels, grad_scale, dcut=dcut, b0=b0)
        s = _stream(sf)
        with TIMER("reduce_slabs"):
            _lib.call("slk_reduce_slabs", sf.data_ptr(), sf.shape[0], SERVER_NPARAM, self.grads.data_ptr(),
                      int(k > 0), s)
        parts = self._b("loss_parts", (nparts,), _F32)
        _lib.call("slk_loss_sum", loss_i.data_ptr(), loss_i.numel(), float(grad_scale), parts[k:].data_ptr(), s)
        return dcut

    def finish_step(self, nparts: int, step=None):
        """Adam from the accumulated gradient, loss logged (sum of the parts), step counter ticked."""
        g = self.grads
        s = _stream(g)
        _k("adam_from_slabs", self.params.data_ptr(), None, self.m.data_ptr(), self.v.data_ptr(), g.data_ptr(), 1,
           SERVER_NPARAM, float(self.lr), float(self.betas[0]), float(self.betas[1]), float(self.eps),
           self.step_ctr.data_ptr(), s)
        self.refresh_shadows()
        parts = self._b("loss_parts", (nparts,), _F32)
        _k("loss_log", parts.data_ptr(), nparts, 1.0, self.loss_log.ring.data_ptr(), self.loss_log.ring.numel(),
           self.loss_log.counter.data_ptr(), s)
        if step is not None:
            self.loss_log.note_step(step)
        _k("tick", self.step_ctr.data_ptr(), s)


class WideTrainer:
    """Both widened stages fused on one GPU, the whole step captured as one HIP graph (like
    engine.SplitTrainer): client fwd -> server dropout/fc/CE/bwd/Adam -> client bwd/Adam."""

    def __init__(self, client: Optional[WideModelPartA] = None, server: Optional[WideModelPartB] = None,
                 device="cuda", graph: bool = True, seed: int = 0):
        self.device = torch.device(device)
        self.client = WideClientStage(client, self.device)
        self.server = WideServerStage(server, self.device, seed=seed)
        self.graph = graph
        self._graphs = {}
        self.global_step = 0

    @property
    def loss_log(self) -> LossLog:
        return self.server.loss_log

    def _eager(self, x, y):
        cut = self.client.forward(x)
        dcut, _ = self.server.step_request(cut, y)
        self.client.backward_step(dcut)

    def _state(self):
        c, s = self.client, self.server
        return [c.params, c.m, c.v, c.step_ctr, s.params, s.m, s.v, s.step_ctr, s.loss_log.counter]

    def _graph_for(self, B):
        g = self._graphs.get(B)
        if g is not None:
            return g
        x = torch.zeros((B, 3, 32, 32), dtype=_F32, device=self.device)
        y = torch.zeros((B,), dtype=torch.int64, device=self.device)
        saved = [t.clone() for t in self._state()]
        st = torch.cuda.Stream(self.device)
        st.wait_stream(torch.cuda.current_stream(self.device))
        with torch.cuda.stream(st):
            self._eager(x, y)
        torch.cuda.current_stream(self.device).wait_stream(st)
        graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(graph):
            self._eager(x, y)
        for t, v in zip(self._state(), saved):
            t.copy_(v)
        self.client.refresh_shadows()
        self.server.refresh_shadows()
        g = {"graph": graph, "x": x, "y": y}
        self._graphs[B] = g
        return g

    def static_inputs(self, B):
        g = self._graph_for(B)
        return g["x"], g["y"]

    def step(self, x, y):
        B = x.shape[0]
        if self.graph:
            g = self._graph_for(B)
            if x.data_ptr() != g["x"].data_ptr():
                g["x"].copy_(x, non_blocking=True)
            if y.data_ptr() != g["y"].data_ptr():
                g["y"].copy_(y, non_blocking=True)
            g["graph"].replay()
        else:
            self._eager(x, y)
        self.server.loss_log.note_step(self.global_step)
        self.global_step += 1
