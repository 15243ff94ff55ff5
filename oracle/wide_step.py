"""ORACLE — TEST INFRASTRUCTURE ONLY. Never imported by the product path (splitcnn/).

CPU restatement (numpy, float64 accumulation) of the WIDENED split-CNN step, BASELINE.json config 5
("K5": widened split CNN, 64-256 channels, synthetic 3x32x32, deeper cut, bf16 MFMA implicit-GEMM
conv) with the north star's dropout and Adam. The reference has no such model:
its step contract (client_part.py:110-138 <-> server_part.py:25-58) is kept, the network is widened:

  client  conv1 3->64  3x3 pad 1 + ReLU                       (32x32)
          conv2 64->128 3x3 pad 1 + ReLU + maxpool 2           (-> 16x16)
          conv3 128->256 3x3 pad 1 + ReLU + maxpool 2          (-> 8x8: the cut, 16,384 per sample)
  server  Dropout(p=0.25) -> flatten (c*64 + y*8 + x) -> Linear(16384, 10) -> CrossEntropyLoss(mean)
  optim   torch.optim.Adam(lr=1e-3, betas=(0.9, 0.999), eps=1e-8) on both sides

Numerics of the bf16 path (what the GPU kernels compute, and therefore what this oracle restates):
every convolution (forward, dgrad, wgrad) multiplies bf16 operands — the input image rounded to
bf16, the weights as bf16 shadows of the f32 masters, activations and gradients as stored — with f32
accumulation (as torch autocast runs a bf16 conv); activations are stored as bf16
(round-to-nearest-even) after ReLU and after each pool, and so are the cut gradient and the
unpooled / ReLU-masked gradients; the max-pool argmax is taken on
the f32 pre-rounding values; the head, cross-entropy, Adam and all master weights are f32. With
bf16=False every rounding is skipped: that float64 form is what tests/test_wide_oracle.py pins
against torch autograd + torch.optim.Adam on the same modules (the reference has no fixtures for
this config: its parity anchor is torch's semantics, as for the dropout and Adam the north star adds).

Dropout mask: keep(b, f) = lowbias32(e*0x9E3779B1 + step*0x85EBCA77 + seed*0xC2B2AE3D) >= p * 2^32
with e = b*16384 + f (all uint32 arithmetic); kept values are scaled by 1/(1-p) in f32.
"""
from __future__ import annotations

import numpy as np

CUT_C, CUT_HW = 256, 8
CUT_F = CUT_C * CUT_HW * CUT_HW      # 16384
NCLS = 10
P_DROP = 0.25
LR, BETA1, BETA2, EPS = 1e-3, 0.9, 0.999, 1e-8
CODE_NONE = 4
PARAM_SHAPES = {
    "conv1.weight": (64, 3, 3, 3), "conv1.bias": (64,),
    "conv2.weight": (128, 64, 3, 3), "conv2.bias": (128,),
    "conv3.weight": (256, 128, 3, 3), "conv3.bias": (256,),
    "fc.weight": (NCLS, CUT_F), "fc.bias": (NCLS,),
}
CLIENT_KEYS = ["conv1.weight", "conv1.bias", "conv2.weight", "conv2.bias", "conv3.weight", "conv3.bias"]
SERVER_KEYS = ["fc.weight", "fc.bias"]


# ----------------------------------------------------------------------------- bf16 helpers
def bf16(a):
    """Round to the nearest bf16 (ties to even), returned as float32 values."""
    u = np.ascontiguousarray(a, dtype=np.float32).view(np.uint32).astype(np.uint64)
    u = ((u + 0x7FFF + ((u >> 16) & 1)) & 0xFFFF0000).astype(np.uint32)
    return u.view(np.float32)


def _r(a, on):
    return bf16(a).astype(np.float64) if on else a


# ----------------------------------------------------------------------------- conv / pool
def _pad1(x):
    return np.pad(x, ((0, 0), (0, 0), (1, 1), (1, 1)))


def _cols(xp, H, W):
    """xp [B,C,H+2,W+2] -> [B,C,3,3,H,W]."""
    B, C = xp.shape[:2]
    out = np.empty((B, C, 3, 3, H, W), dtype=xp.dtype)
    for ky in range(3):
        for kx in range(3):
            out[:, :, ky, kx] = xp[:, :, ky:ky + H, kx:kx + W]
    return out


def conv3x3p1(x, W, b=None):
    """conv2d(x, W, b, stride 1, padding 1): x [B,Ci,H,W], W [Co,Ci,3,3] -> [B,Co,H,W]."""
    H, Wd = x.shape[2:]
    y = np.einsum("bcklhw,ockl->bohw", _cols(_pad1(x), H, Wd), W, optimize=True)
    return y if b is None else y + b[None, :, None, None]


def conv3x3p1_wgrad(x, dy):
    """dW[o,c,ky,kx] = sum dy[b,o,h,w] * xpad[b,c,h+ky,w+kx]; db = sum dy."""
    H, Wd = x.shape[2:]
    dW = np.einsum("bohw,bcklhw->ockl", dy, _cols(_pad1(x), H, Wd), optimize=True)
    return dW, dy.sum(axis=(0, 2, 3))


def conv3x3p1_dgrad(dy, W):
    """dx = full correlation of dy with W, cropped back to the input size (padding 1)."""
    B, Co, H, Wd = dy.shape
    Ci = W.shape[1]
    dxp = np.zeros((B, Ci, H + 2, Wd + 2), dtype=dy.dtype)
    for ky in range(3):
        for kx in range(3):
            dxp[:, :, ky:ky + H, kx:kx + Wd] += np.einsum("bohw,oc->bchw", dy, W[:, :, ky, kx], optimize=True)
    return dxp[:, :, 1:H + 1, 1:Wd + 1]


def relu_pool_code(c):
    """maxpool2(relu(c)) with torch's first-max argmax; code = argmax position 0..3 (row-major in
    the window) where the pooled value is > 0, else 4 (the ReLU blocks the gradient)."""
    B, C, H, W = c.shape
    win = c.reshape(B, C, H // 2, 2, W // 2, 2).transpose(0, 1, 2, 4, 3, 5).reshape(B, C, H // 2, W // 2, 4)
    win = np.where(win > 0, win, 0.0)
    idx = np.zeros(win.shape[:-1], dtype=np.int64)
    best = win[..., 0].copy()
    for q in range(1, 4):
        better = win[..., q] > best
        best = np.where(better, win[..., q], best)
        idx = np.where(better, q, idx)
    return best, np.where(best > 0, idx, CODE_NONE)


def unpool(dp, code):
    """Route dp [B,C,h,w] to the argmax position given by code (4 -> nowhere): [B,C,2h,2w]."""
    B, C, h, w = dp.shape
    d = np.zeros((B, C, h, w, 4), dtype=dp.dtype)
    for q in range(4):
        d[..., q] = np.where(code == q, dp, 0.0)
    return d.reshape(B, C, h, w, 2, 2).transpose(0, 1, 2, 4, 3, 5).reshape(B, C, 2 * h, 2 * w)


# ----------------------------------------------------------------------------- dropout / loss / adam
def lowbias32(x):
    x = np.asarray(x, dtype=np.uint32)
    x = x ^ (x >> np.uint32(16))
    x = (x * np.uint32(0x7FEB352D)).astype(np.uint32)
    x = x ^ (x >> np.uint32(15))
    x = (x * np.uint32(0x846CA68B)).astype(np.uint32)
    return x ^ (x >> np.uint32(16))


def dropout_keep(seed, step, B, F=CUT_F, p=P_DROP, b0=0):
    """Boolean keep mask [B, F] for samples b0 .. b0+B-1 of a step (flatten order c*64+y*8+x)."""
    with np.errstate(over="ignore"):
        e = (np.arange(b0, b0 + B, dtype=np.uint64)[:, None] * F + np.arange(F, dtype=np.uint64)[None, :])
        h = (e * 0x9E3779B1 + np.uint64(step) * 0x85EBCA77 + np.uint64(seed) * 0xC2B2AE3D) & 0xFFFFFFFF
    thresh = np.uint32(int(round(p * 4294967296.0)))
    return lowbias32(h.astype(np.uint32)) >= thresh


def cross_entropy(logits, y):
    B = logits.shape[0]
    m = logits.max(axis=1, keepdims=True)
    lse = m + np.log(np.exp(logits - m).sum(axis=1, keepdims=True))
    logp = logits - lse
    loss_i = -logp[np.arange(B), y]
    onehot = np.zeros_like(logits)
    onehot[np.arange(B), y] = 1.0
    return loss_i.mean(), loss_i, (np.exp(logp) - onehot) / B


def adam(p, g, m, v, t, lr=LR, b1=BETA1, b2=BETA2, eps=EPS, f32=True):
    """torch.optim.Adam single-tensor update (torch/optim/adam.py `_single_tensor_adam`, default
    flags): exp_avg.lerp_(g, 1-b1); exp_avg_sq.mul_(b2).addcmul_(g, g, value=1-b2);
    denom = sqrt(v)/sqrt(1-b2^t) + eps; p.addcdiv_(exp_avg, denom, value=-lr/(1-b1^t)).
    The bias corrections are Python floats (float64); the tensor math is f32 when f32=True."""
    bc1 = 1.0 - b1 ** t
    bc2s = np.sqrt(1.0 - b2 ** t)
    step_size = lr / bc1
    if not f32:
        m = m + (1 - b1) * (g - m)
        v = v * b2 + (1 - b2) * g * g
        return p - step_size * m / (np.sqrt(v) / bc2s + eps), m, v
    f = np.float32
    p, g, m, v = (np.asarray(a, dtype=f) for a in (p, g, m, v))
    w = f(1 - b1)
    m = m + w * (g - m)                       # lerp with weight < 0.5
    v = v * f(b2) + g * g * f(1 - b2)
    denom = np.sqrt(v) / f(bc2s) + f(eps)
    p = p + f(-step_size) * (m / denom)
    return p, m, v


# ----------------------------------------------------------------------------- the step
def client_forward(P, x, bf=True):
    """Returns (cut, rec): cut = bf16(pool3) [B,256,8,8] and the saved tensors."""
    xb = _r(x, bf)
    a1 = _r(np.maximum(conv3x3p1(xb, _r(P["conv1.weight"], bf), P["conv1.bias"]), 0.0), bf)
    W2 = _r(P["conv2.weight"], bf)
    c2 = conv3x3p1(a1, W2, P["conv2.bias"])
    p2f, code2 = relu_pool_code(c2)
    p2 = _r(p2f, bf)
    W3 = _r(P["conv3.weight"], bf)
    c3 = conv3x3p1(p2, W3, P["conv3.bias"])
    p3f, code3 = relu_pool_code(c3)
    cut = _r(p3f, bf)
    return cut, dict(xb=xb, a1=a1, c2=c2, p2=p2, code2=code2, c3=c3, code3=code3, cut=cut, W2b=W2, W3b=W3)


def server_step(P, cut, y, keep, grad_scale_batch=None, bf=True):
    """Dropout -> fc -> CE fwd/bwd. Returns dict(loss, loss_i, logits, dlogits, dcut, dfc_w, dfc_b)."""
    B = cut.shape[0]
    flat = cut.reshape(B, -1)
    if bf:
        d = (flat.astype(np.float32) * np.float32(1.0 / (1.0 - P_DROP))).astype(np.float64) * keep
    else:
        d = flat * keep / (1.0 - P_DROP)
    logits = d @ P["fc.weight"].T + P["fc.bias"]
    loss, loss_i, dlogits = cross_entropy(logits, y)
    if grad_scale_batch is not None:
        dlogits = dlogits * B / grad_scale_batch
    dfc_w = dlogits.T @ d
    dfc_b = dlogits.sum(axis=0)
    dd = dlogits @ P["fc.weight"]
    dflat = dd * keep / (1.0 - P_DROP)
    if bf:
        dflat = (dd.astype(np.float32) * np.float32(1.0 / (1.0 - P_DROP))).astype(np.float64) * keep
    dcut = _r(dflat.reshape(cut.shape), bf)
    return dict(loss=loss, loss_i=loss_i, logits=logits, dlogits=dlogits, dcut=dcut,
                grads={"fc.weight": dfc_w, "fc.bias": dfc_b})


def client_backward(P, x, rec, dcut, bf=True):
    """act.backward(cut_grad) for the widened client: returns grads of conv1..conv3 and the
    intermediate gradients (dc3, dc2, da1m)."""
    dc3 = unpool(dcut, rec["code3"])
    dW3, db3 = conv3x3p1_wgrad(rec["p2"], dc3)
    dp2 = conv3x3p1_dgrad(dc3, rec["W3b"])
    dc2 = _r(unpool(dp2, rec["code2"]), bf)
    dW2, db2 = conv3x3p1_wgrad(rec["a1"], dc2)
    da1 = conv3x3p1_dgrad(dc2, rec["W2b"])
    da1m = _r(np.where(rec["a1"] > 0, da1, 0.0), bf)
    dW1, db1 = conv3x3p1_wgrad(rec["xb"], da1m)
    grads = {"conv1.weight": dW1, "conv1.bias": db1, "conv2.weight": dW2, "conv2.bias": db2,
             "conv3.weight": dW3, "conv3.bias": db3}
    return grads, dict(dc3=dc3, dc2=dc2, da1m=da1m)


def wide_step(P, opt, t, x, y, seed=0, bf=True, code_override=None):
    """One K5 split step at Adam step t (1-based). P: dict of float64 params; opt: dict name ->
    (m, v) (zeros at t=1). Returns (new_P, new_opt, record). code_override = (code2, code3)
    replaces the max-pool routing (e.g. by a GPU run's after a tie check)."""
    P = {k: np.asarray(v, dtype=np.float64) for k, v in P.items()}
    x = np.asarray(x, dtype=np.float64)
    y = np.asarray(y, dtype=np.int64)
    cut, rec = client_forward(P, x, bf)
    if code_override is not None:
        rec["code2"], rec["code3"] = (np.asarray(c).astype(np.int64) for c in code_override)
    keep = dropout_keep(seed, t - 1, x.shape[0])
    s = server_step(P, cut, y, keep, bf=bf)
    cg, crec = client_backward(P, x, rec, s["dcut"], bf)
    grads = dict(cg, **s["grads"])
    newP, newopt = {}, {}
    for k in P:
        m, v = opt.get(k, (np.zeros_like(P[k]), np.zeros_like(P[k])))
        p2, m2, v2 = adam(P[k], grads[k], m, v, t, f32=bf)
        newP[k] = np.asarray(p2, dtype=np.float64)
        newopt[k] = (m2, v2)
    s = {k: v for k, v in s.items() if k != "grads"}
    return newP, newopt, dict(rec, **crec, **s, grads=grads, keep=keep)

