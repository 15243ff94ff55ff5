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
from .engine import TIMER, LossLog, _Buffers, register_graph_inputs, select_graph
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
# The module contract of src/model_def.py:5-71 for the widened network: the halves are differentiable
# (autograd Functions over the same kernels the stages launch), so the reference's own step code runs
# on them — client: activations = model(x); activations.backward(grads); optimizer.step()
# (src/client_part.py:112-133); server: client_activations.requires_grad_(True); outputs =
# model(client_activations); loss = criterion(outputs, labels); loss.backward(); optimizer.step();
# return client_activations.grad (src/server_part.py:45-57). The cut is bf16 in logical NCHW
# [B,256,8,8] at this boundary (the kernels use C8 internally). The stages (WideClientStage /
# WideServerStage / WideTrainer) are the fused fast path over the same kernels.
class WideModelPartA(nn.Module):
    """Client bottom stack: conv1 3->64 + ReLU, conv2 64->128 + ReLU + pool, conv3 128->256 + ReLU +
    pool -> cut bf16 [B,256,8,8]."""

    def __init__(self):
        super().__init__()
        self.conv1 = nn.Conv2d(3, 64, 3, 1, padding=1)
        self.conv2 = nn.Conv2d(64, 128, 3, 1, padding=1)
        self.conv3 = nn.Conv2d(128, 256, 3, 1, padding=1)
        self.relu = nn.ReLU()
        self.pool = nn.MaxPool2d(2)

    def forward(self, x):
        _require_cuda(x, "WideModelPartA")
        return _WideClientFn.apply(x, self.conv1.weight, self.conv1.bias, self.conv2.weight, self.conv2.bias,
                                   self.conv3.weight, self.conv3.bias)


class WideModelPartB(nn.Module):
    """Server top stack: Dropout(0.25) -> flatten -> Linear(16384, 10). In training mode each forward
    draws a fresh dropout mask (the hash of seed, forward count, sample, feature — the stages' mask
    at the same step); eval mode keeps every feature."""

    def __init__(self):
        super().__init__()
        self.dropout = nn.Dropout(P_DROP)
        self.flatten = nn.Flatten()
        self.fc = nn.Linear(256 * 8 * 8, 10)
        self.dropout_seed = 0
        self._drop_step = None   # device forward counter (not state: keeps the state_dict contract)

    def forward(self, x):
        _require_cuda(x, "WideModelPartB")
        if self._drop_step is None or self._drop_step.device != x.device:
            self._drop_step = torch.zeros(1, dtype=torch.int32, device=x.device)
        snap = self._drop_step.clone()
        thresh, scale = (KEEP_THRESHOLD, KEEP_SCALE) if self.training else (0, 1.0)
        logits = _WideHeadFn.apply(x, self.fc.weight, self.fc.bias, snap, self.dropout_seed, thresh, scale)
        if self.training:
            _lib.call("slk_tick", self._drop_step.data_ptr(), _stream(x))
        return logits


class WideFullModel(nn.Module):
    """The unsplit widened network; parameter names = A ∪ B (like FullModel, src/model_def.py:31-46)."""

    def __init__(self):
        super().__init__()
        a, b = WideModelPartA(), WideModelPartB()
        self.conv1, self.conv2, self.conv3 = a.conv1, a.conv2, a.conv3
        self.dropout, self.fc = b.dropout, b.fc
        self._head = [b]   # shares fc / dropout; kept out of the module tree (state_dict keys)

    def forward(self, x):
        _require_cuda(x, "WideFullModel")
        cut = _WideClientFn.apply(x, self.conv1.weight, self.conv1.bias, self.conv2.weight, self.conv2.bias,
                                  self.conv3.weight, self.conv3.bias)
        head = self._head[0]
        head.train(self.training)
        return head(cut)


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



def _require_cuda(x, who):
    if x.device.type != "cuda":
        raise RuntimeError(f"splitcnn.{who}: input is on {x.device}; the widened model runs on the MI355X HIP "
                           "kernels only (move the module and its inputs to a ROCm device). There is no CPU fallback.")


def _f32p(t, name, n):
    """Device pointer of an f32 parameter (contiguous, n elements)."""
    _dev(t, name)
    if t.numel() != n:
        raise ValueError(f"{name}: expected {n} elements, got {t.numel()}")
    return t.data_ptr()


def new_shadows(device):
    return {"w1b": torch.empty(64 * 32, dtype=_BF, device=device), "w2f": torch.empty(73728, dtype=_BF, device=device),
            "w2d": torch.empty(73728, dtype=_BF, device=device), "w3f": torch.empty(294912, dtype=_BF, device=device),
            "w3d": torch.empty(294912, dtype=_BF, device=device)}


def build_shadows(W1, W2, W3, sh, stream):
    """bf16 MFMA layouts of the conv weights from their f32 masters (slk_wide_shadows)."""
    _k("wide_shadows", _f32p(W1, "conv1.weight", 1728), _f32p(W2, "conv2.weight", 73728),
       _f32p(W3, "conv3.weight", 294912), sh["w1b"].data_ptr(), sh["w2f"].data_ptr(), sh["w2d"].data_ptr(),
       sh["w3f"].data_ptr(), sh["w3d"].data_ptr(), stream)


def client_forward_kernels(x, sh, b1, b2, b3, a1, p2, code2, cut, code3, a1bits=None):
    """conv1 + ReLU -> conv2 + ReLU + pool -> conv3 + ReLU + pool (the cut), C8 bf16. a1bits ([B, 1024]
    int64): conv1 also writes the ReLU word of every pixel (bit c = a1[c] > 0), conv2's dgrad mask."""
    B = x.shape[0]
    _dev(x, "x", (B, 3, 32, 32))
    s = _stream(x)
    b1p, b2p, b3p = _f32p(b1, "conv1.bias", 64), _f32p(b2, "conv2.bias", 128), _f32p(b3, "conv3.bias", 256)
    bits = _dev(a1bits, "a1bits", (B, 1024), torch.int64) if a1bits is not None else None
    _k("wide_conv1_fwd", x.data_ptr(), sh["w1b"].data_ptr(), b1p, a1.data_ptr(), bits, B, s)
    _k("wide_conv2_fwd", a1.data_ptr(), sh["w2f"].data_ptr(), b2p, p2.data_ptr(), code2.data_ptr(), B, s)
    _k("wide_conv3_fwd", p2.data_ptr(), sh["w3f"].data_ptr(), b3p, cut.data_ptr(), code3.data_ptr(), B, s)


def client_backward_slab_shapes(B):
    return ((_q("slk_wide_conv1_wgrad_nslab", B), 1728 + 64), (_q("slk_wide_conv2_wgrad_nslab", B), 73728 + 128),
            (_q("slk_wide_conv3_wgrad_nslab", B), 294912 + 256))


def client_backward_kernels(dcut, saved, w2d, w3d, scratch, s1, s2, s3):
    """activations.backward(dcut) of the client stack into three slab sets [dW | db] (conv1, conv2,
    conv3). saved = (x, a1, p2, code2, code3[, a1bits]) of the forward; scratch = (dp2, da1m). No
    unpooled gradient is stored: conv3's kernels route the pooled dcut by code3 while staging it, conv3's
    dgrad writes dp2 (the gradient of p2, 16 x 16) and conv2's kernels route dp2 by code2 the same way.
    conv2's dgrad masks by a1 > 0 from a1's ReLU words (slk_wide_conv1_fwd writes them; computed from a1
    here when the forward did not)."""
    x, a1, p2, code2, code3 = saved[:5]
    dp2, da1m = scratch
    B = x.shape[0]
    s = _stream(dp2)
    _dev(dcut, "dcut", (B,) + CUT_SHAPE, _BF)
    if len(saved) > 5 and saved[5] is not None:
        _dev(saved[5], "a1bits", (B, 1024), torch.int64)
        a1bits = saved[5]
    else:
        a1bits = torch.empty((B, 1024), dtype=torch.int64, device=dp2.device)
        _k("wide_relu_bits", a1.data_ptr(), a1bits.data_ptr(), B, s)
    _k("wide_conv3_wgrad", dcut.data_ptr(), code3.data_ptr(), p2.data_ptr(), s3.data_ptr(), B, s)
    _k("wide_conv3_dgrad", dcut.data_ptr(), code3.data_ptr(), w3d.data_ptr(), dp2.data_ptr(), B, s)
    _k("wide_conv2_wgrad", dp2.data_ptr(), code2.data_ptr(), a1.data_ptr(), s2.data_ptr(), B, s)
    _k("wide_conv2_dgrad", dp2.data_ptr(), code2.data_ptr(), w2d.data_ptr(), a1bits.data_ptr(), da1m.data_ptr(), B, s)
    _k("wide_conv1_wgrad", x.data_ptr(), da1m.data_ptr(), s1.data_ptr(), B, s)


def client_backward_scratch(B, get):
    """(dp2, da1m) via get(name, shape, dtype)."""
    return get("dp2", (B, 16, 16, 16, 8), _BF), get("da1m", (B, 8, 32, 32, 8), _BF)


def _reduce(slabs):
    out = torch.empty(slabs.shape[1], dtype=_F32, device=slabs.device)
    _lib.call("slk_reduce_slabs", slabs.data_ptr(), slabs.shape[0], slabs.shape[1], out.data_ptr(), 0, _stream(slabs))
    return out


class _WideClientFn(torch.autograd.Function):
    """cut = WideModelPartA(x) (bf16, logical NCHW); backward = the client stack's weight gradients."""

    @staticmethod
    def forward(ctx, x, W1, b1, W2, b2, W3, b3):
        x = x.contiguous()
        B, dev = x.shape[0], x.device
        Ws = [t.detach().contiguous() for t in (W1, b1, W2, b2, W3, b3)]
        sh = new_shadows(dev)
        build_shadows(Ws[0], Ws[2], Ws[4], sh, _stream(x))
        a1 = torch.empty((B, 8, 32, 32, 8), dtype=_BF, device=dev)
        p2 = torch.empty((B, 16, 16, 16, 8), dtype=_BF, device=dev)
        code2 = torch.empty((B, 16, 16, 16, 8), dtype=_U8, device=dev)
        cut = torch.empty((B,) + CUT_SHAPE, dtype=_BF, device=dev)
        code3 = torch.empty((B,) + CUT_SHAPE, dtype=_U8, device=dev)
        a1bits = torch.empty((B, 1024), dtype=torch.int64, device=dev)
        client_forward_kernels(x, sh, Ws[1], Ws[3], Ws[5], a1, p2, code2, cut, code3, a1bits)
        ctx.save_for_backward(x, a1, p2, code2, code3, a1bits, sh["w2d"], sh["w3d"])
        return c8_to_nchw(cut)

    @staticmethod
    def backward(ctx, g):
        if ctx.needs_input_grad[0]:
            raise NotImplementedError("splitcnn: gradient w.r.t. the client's input images is not part of the "
                                      "split step (src/client_part.py:110-114)")
        x, a1, p2, code2, code3, a1bits, w2d, w3d = ctx.saved_tensors
        B, dev = x.shape[0], x.device
        dcut = nchw_to_c8(g.to(_BF))
        scratch = client_backward_scratch(B, lambda n, sh_, dt: torch.empty(sh_, dtype=dt, device=dev))
        slabs = [torch.empty(sh_, dtype=_F32, device=dev) for sh_ in client_backward_slab_shapes(B)]
        client_backward_kernels(dcut, (x, a1, p2, code2, code3, a1bits), w2d, w3d, scratch, *slabs)
        g1, g2, g3 = (_reduce(sl) for sl in slabs)
        return (None, g1[:1728].view(64, 3, 3, 3), g1[1728:], g2[:73728].view(128, 64, 3, 3), g2[73728:],
                g3[:294912].view(256, 128, 3, 3), g3[294912:])


class _WideHeadFn(torch.autograd.Function):
    """logits = fc(dropout(flatten(cut))) — WideModelPartB.forward; backward gives the cut gradient
    (bf16, logical NCHW) and the fc weight gradient."""

    @staticmethod
    def forward(ctx, cut_nchw, Wf, bf, step, seed, thresh, scale):
        B, dev = cut_nchw.shape[0], cut_nchw.device
        if tuple(cut_nchw.shape[1:]) != (256, 8, 8):
            raise ValueError(f"cut: expected [B,256,8,8], got {tuple(cut_nchw.shape)}")
        cut = nchw_to_c8(cut_nchw.detach().to(_BF))
        Wf, bf = Wf.detach().contiguous(), bf.detach().contiguous()
        wf8 = torch.empty(163840, dtype=_F32, device=dev)
        s = _stream(cut)
        _k("wide_fc_shadow", _f32p(Wf, "fc.weight", 163840), wf8.data_ptr(), s)
        logits = torch.empty((B, 10), dtype=_F32, device=dev)
        _k("wide_head_fwd", cut.data_ptr(), wf8.data_ptr(), _f32p(bf, "fc.bias", 10), step.data_ptr(), int(seed),
           int(thresh), float(scale), logits.data_ptr(), 0, B, s)
        ctx.save_for_backward(cut, wf8, step)
        ctx.drop = (int(seed), int(thresh), float(scale))
        ctx.in_dtype = cut_nchw.dtype
        return logits

    @staticmethod
    def backward(ctx, dlogits):
        cut, wf8, step = ctx.saved_tensors
        seed, thresh, scale = ctx.drop
        B, dev = cut.shape[0], cut.device
        dlogits = dlogits.to(_F32).contiguous()
        dcut = torch.empty_like(cut)
        slabs = torch.empty((_q("slk_wide_head_nslab", B), SERVER_NPARAM), dtype=_F32, device=dev)
        _k("wide_head_bwd", cut.data_ptr(), wf8.data_ptr(), _dev(dlogits, "dlogits", (B, 10)), step.data_ptr(), seed,
           thresh, scale, dcut.data_ptr(), slabs.data_ptr(), 0, B, _stream(dlogits))
        g = _reduce(slabs)
        return (c8_to_nchw(dcut).to(ctx.in_dtype), g[:163840].view(10, 16384), g[163840:], None, None, None, None)

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
        self.sh = new_shadows(self.device)   # bf16 conv weight shadows (slk_wide_shadows layouts)
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
        build_shadows(self._p("W1", 1728), self._p("W2", 73728), self._p("W3", 294912), self.sh, _stream(self.params))

    def forward(self, x: torch.Tensor, out: Optional[torch.Tensor] = None, tag="") -> torch.Tensor:
        """cut = client forward of x; `tag` keeps separate saved tensors per micro-batch."""
        B = x.shape[0]
        _dev(x, "x", (B, 3, 32, 32))
        a1 = self._b(f"a1{tag}", (B, 8, 32, 32, 8), _BF)
        p2 = self._b(f"p2{tag}", (B, 16, 16, 16, 8), _BF)
        code2 = self._b(f"code2{tag}", (B, 16, 16, 16, 8), _U8)
        cut = out if out is not None else self._b(f"cut{tag}", (B,) + CUT_SHAPE, _BF)
        _dev(cut, "cut", (B,) + CUT_SHAPE, _BF)
        code3 = self._b(f"code3{tag}", (B,) + CUT_SHAPE, _U8)
        a1bits = self._b(f"a1bits{tag}", (B, 1024), torch.int64)
        client_forward_kernels(x, self.sh, self._p("b1", 64), self._p("b2", 128), self._p("b3", 256),
                               a1, p2, code2, cut, code3, a1bits)
        self._x, self._a1, self._p2, self._code2, self._code3 = x, a1, p2, code2, code3
        self._saved[tag] = (x, a1, p2, code2, code3, a1bits)
        return cut

    def backward_slabs(self, dcut: torch.Tensor, tag=""):
        """Client backward into three slab sets (conv1, conv2, conv3); returns them."""
        B = self._saved[tag][0].shape[0]
        self._x, self._a1, self._p2, self._code2, self._code3 = self._saved[tag][:5]
        scratch = client_backward_scratch(B, self._b)
        s1, s2, s3 = (self._b(n, shp, _F32) for n, shp in zip(("s1", "s2", "s3"), client_backward_slab_shapes(B)))
        client_backward_kernels(dcut, self._saved[tag], self.sh["w2d"], self.sh["w3d"], scratch, s1, s2, s3)
        self._dp2, self._da1m = scratch
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
        self.graph_inputs = 4   # caller input buffers captured directly (as engine.SplitTrainer)
        self._seen = {}
        self.global_step = 0

    @property
    def loss_log(self) -> LossLog:
        return self.server.loss_log

    def _eager(self, x, y):
        c = self.client
        dcut, _ = self.server.step_request(c.forward(x), y)
        c.backward_step(dcut)

    def _state(self):
        c, s = self.client, self.server
        return [c.params, c.m, c.v, c.step_ctr, s.params, s.m, s.v, s.step_ctr, s.loss_log.counter]

    def _graph_for(self, B, x=None, y=None):
        """The step's graph on the static inputs, or (x, y given) on those caller buffers."""
        key = B if x is None else (B, x.data_ptr(), y.data_ptr())
        g = self._graphs.get(key)
        if g is not None:
            return g
        if x is None:
            x = torch.zeros((B, 3, 32, 32), dtype=_F32, device=self.device)
            y = torch.zeros((B,), dtype=torch.int64, device=self.device)
        saved = [t.clone() for t in self._state()]
        st = torch.cuda.Stream(self.device)
        st.wait_stream(torch.cuda.current_stream(self.device))
        with torch.cuda.stream(st):
            self._eager(x, y)
        torch.cuda.current_stream(self.device).wait_stream(st)
        graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(graph, capture_error_mode="thread_local"):
            self._eager(x, y)
        for t, v in zip(self._state(), saved):
            t.copy_(v)
        self.client.refresh_shadows()
        self.server.refresh_shadows()
        g = {"graph": graph, "x": x, "y": y}
        self._graphs[key] = g
        return g

    def _own_buffers_ok(self, x, y) -> bool:
        return (x.device == self.device and y.device == self.device and x.dtype == _F32 and y.dtype == torch.int64
                and x.is_contiguous() and y.is_contiguous() and tuple(x.shape[1:]) == (3, 32, 32)
                and y.shape == (x.shape[0],))

    def register_inputs(self, x, y) -> bool:
        """Capture a graph on the caller's own (x, y) buffers now (engine.register_graph_inputs)."""
        return register_graph_inputs(self, x, y)

    def static_inputs(self, B):
        g = self._graph_for(B)
        return g["x"], g["y"]

    def step(self, x, y):
        B = x.shape[0]
        if self.graph:
            g = select_graph(self, x, y)
            if g is not None:
                g["graph"].replay()
                self.server.loss_log.note_step(self.global_step)
                self.global_step += 1
                return
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
