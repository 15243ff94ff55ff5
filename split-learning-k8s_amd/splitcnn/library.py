"""torch.library registration of the split-CNN kernels (namespace ``splitcnn``).

Every op here is a functional wrapper over one libslk.so entry point (ops.py), registered with
``torch.library.custom_op`` so that the drop-in modules (model_def.py) are visible to the PyTorch
stack as opaque, differentiable operators rather than as Python autograd.Functions: each op has a
fake (meta) kernel, so ``torch.export`` / ``make_fx`` / ``torch.compile`` can trace a module without
running it, and the forward ops register their backward through other ``splitcnn`` ops, so the
traced backward graph is made of them too. The real kernels run only on a ROCm device (ops.py raises
otherwise); there is no CPU implementation.

The ops and the reference calls they replace (src/model_def.py, src/server_part.py):
  conv1_relu(x, W1, b1) -> act                              ModelPartA.forward (model_def.py:11-12)
  conv2_relu_pool(act, W2, b2) -> (pooled, code, amax, act16) model_def.py:25-26 (x3 kernels by default)
  linear(flat, W3, b3) -> logits                            fc1 (model_def.py:22,28)
  cross_entropy(logits, labels) -> loss                     nn.CrossEntropyLoss() (server_part.py:16,49)
and their backward helpers conv1_wgrad, row_amax, conv2_dgrad(_x3), conv2_wgrad(_x3), linear_dgrad,
linear_wgrad, cross_entropy_grad.
"""
from __future__ import annotations

import os
from typing import Optional, Tuple

import torch
from torch import Tensor

from . import ops

_NS = "splitcnn"


class _Memo:
    """A by-product one op's kernel wrote next to its output, remembered for the op that consumes that
    output in the same autograd pass: linear_dgrad's fused per-sample max |dpooled| (slk_fc_dgrad_amax)
    for the conv2 backward's x3 scales, cross_entropy's dlogits for its backward. A hit requires the very
    same storage (data pointer, element count) at the same version counter (views share it; any in-place
    write bumps it), so the by-product describes exactly the bytes the consumer sees; anything else (a
    miss, fake tensors under tracing) falls back to the op that recomputes it. One entry per kind; a hit
    consumes it."""

    def __init__(self):
        self._e = {}

    @staticmethod
    def _key(t):
        try:
            return (t.device, t.data_ptr(), t.numel(), t._version)
        except Exception:  # noqa: BLE001 (fake / functional tensors under tracing have no storage)
            return None

    def put(self, kind, t, value):
        k = self._key(t)
        if k is None:
            self._e.pop(kind, None)
        else:
            self._e[kind] = (k, t, value)   # t held until consumed or replaced (the next step's put)

    def take(self, kind, t) -> Optional[Tensor]:
        e = self._e.get(kind)
        k = self._key(t)
        if e is None or k is None or e[0] != k:
            return None
        del self._e[kind]
        return e[2]


_MEMO = _Memo()


# ----------------------------------------------------------------------------------- conv1 + ReLU
@torch.library.custom_op(f"{_NS}::conv1_relu", mutates_args=())
def conv1_relu(x: Tensor, W1: Tensor, b1: Tensor) -> Tensor:
    return ops.conv1_fwd(x.contiguous(), W1.contiguous(), b1.contiguous())


@conv1_relu.register_fake
def _(x, W1, b1):
    return x.new_empty((x.shape[0], 32, 26, 26))


@torch.library.custom_op(f"{_NS}::conv1_wgrad", mutates_args=())
def conv1_wgrad(x: Tensor, W1: Tensor, b1: Tensor, g: Tensor) -> Tensor:
    """[dW1 (288) | db1 (32)] of relu(conv1(x)) for the output gradient g. The ReLU mask act > 0 is
    recomputed from x, W1, b1 in conv1's own FMA order (bit-identical to the forward's), so act is neither
    saved nor read: x + g only (slk_conv1_wgrad_remask)."""
    return ops.reduce_slabs(ops.conv1_wgrad_remask_slabs(x.contiguous(), W1.contiguous(), b1.contiguous(),
                                                         g.contiguous()))


@conv1_wgrad.register_fake
def _(x, W1, b1, g):
    return x.new_empty((ops.CLIENT_NPARAM,))


def _conv1_setup(ctx, inputs, output):
    x, W1, b1 = inputs
    # W1 / b1 are saved for the mask: autograd's version check raises if they change before the backward
    ctx.save_for_backward(x, W1, b1)


def _conv1_backward(ctx, g, K=None):
    K = K or torch.ops.splitcnn
    x, W1, b1 = ctx.saved_tensors
    if ctx.needs_input_grad[0]:
        raise NotImplementedError(
            "splitcnn: gradient w.r.t. the client INPUT images is not part of the split step "
            "(the reference's data never requires grad, src/client_part.py:110-114)")
    flat = K.conv1_wgrad(x, W1, b1, g)
    return None, flat[:288].view(32, 1, 3, 3), flat[288:].view(32)


conv1_relu.register_autograd(_conv1_backward, setup_context=_conv1_setup)


# ----------------------------------------------------------------------------------- conv2 + ReLU + pool
# conv2 kernels of the drop-in modules: the engine's presets (engine.CONV_PRESETS), default "x3" — the f16
# MFMA with hi/lo-split fp32 operands for the forward, dgrad and wgrad, as in the fused trainer; "x3w"
# keeps the Winograd f32 wgrad, "f32" is Winograd on the f32 MFMA throughout. SLK_CONV selects.
_PRESETS = {"f32": ("wino", "wino", "wino"), "x3": ("x3", "x3", "x3"), "x3w": ("x3", "x3", "wino")}


def conv_impls() -> Tuple[str, str, str]:
    """(forward, dgrad, wgrad) kernels the conv2 ops run, from SLK_CONV (default "x3")."""
    p = os.environ.get("SLK_CONV", "x3")
    if p not in _PRESETS:
        raise ValueError(f"SLK_CONV must be one of {sorted(_PRESETS)}, got {p!r}")
    return _PRESETS[p]


@torch.library.custom_op(f"{_NS}::row_amax", mutates_args=())
def row_amax(x: Tensor) -> Tensor:
    """Per-row max |x| (the x3 kernels' per-sample operand scales)."""
    return ops.row_amax(x.contiguous())


@row_amax.register_fake
def _(x):
    return x.new_empty((x.shape[0],))


@torch.library.custom_op(f"{_NS}::conv2_relu_pool", mutates_args=())
def conv2_relu_pool(act: Tensor, W2: Tensor, b2: Tensor) -> Tuple[Tensor, Tensor, Tensor, Tensor]:
    """(pooled, code, act_amax, act16). With the x3 forward, act_amax = the per-sample max |act| (the
    kernels' scales; the received cut carries none, src/server_part.py:39-45) and, when the wgrad is x3
    too, act16 = the split input images the forward writes for it (the backward then saves these, not
    act). Otherwise both are empty."""
    fi, _di, wi = conv_impls()
    act = act.contiguous()
    B = act.shape[0]
    if fi != "x3":
        pooled, code = ops.conv2_fwd_pool(act, W2.contiguous(), b2.contiguous(), impl=fi)
        return pooled, code, act.new_empty((0,)), act.new_empty((0,), dtype=torch.uint8)
    a16 = act.new_empty((ops.conv2_act16_bytes(B) if wi == "x3" else 0,), dtype=torch.uint8)
    if wi == "x3" and act.data_ptr() % 16 == 0:
        # the forward computes the per-sample max itself (no separate 354 MB pass at B = 4096)
        amax = act.new_empty((B,))
        pooled, code = ops.conv2_fwd_pool(act, W2.contiguous(), b2.contiguous(), impl="x3", act16=a16,
                                          act_amax_out=amax)
        return pooled, code, amax, a16
    amax = ops.row_amax(act)
    pooled, code = ops.conv2_fwd_pool(act, W2.contiguous(), b2.contiguous(), impl="x3", act_amax=amax,
                                      act16=a16 if wi == "x3" else None)
    return pooled, code, amax, a16


@conv2_relu_pool.register_fake
def _(act, W2, b2):
    fi, _di, wi = conv_impls()
    B = act.shape[0]
    n16 = ops.conv2_act16_bytes(B) if (fi, wi) == ("x3", "x3") else 0
    return (act.new_empty((B, 64, 12, 12)), act.new_empty((B, 64, 12, 12), dtype=torch.uint8),
            act.new_empty((B if fi == "x3" else 0,)), act.new_empty((n16,), dtype=torch.uint8))


@torch.library.custom_op(f"{_NS}::conv2_dgrad", mutates_args=())
def conv2_dgrad(dpooled: Tensor, code: Tensor, W2: Tensor) -> Tensor:
    """Cut gradient: conv2 input gradient of the pool/ReLU-routed dpooled (Winograd f32)."""
    return ops.conv2_dgrad(dpooled.contiguous(), code.contiguous(), W2.contiguous())


@conv2_dgrad.register_fake
def _(dpooled, code, W2):
    return dpooled.new_empty((dpooled.shape[0], 32, 26, 26))


@torch.library.custom_op(f"{_NS}::conv2_dgrad_x3", mutates_args=())
def conv2_dgrad_x3(dpooled: Tensor, code: Tensor, W2: Tensor, dp_amax: Tensor) -> Tensor:
    """Cut gradient on the x3 kernel (dp_amax = per-sample max |dpooled|)."""
    return ops.conv2_dgrad(dpooled.contiguous(), code.contiguous(), W2.contiguous(), impl="x3", dp_amax=dp_amax)


@conv2_dgrad_x3.register_fake
def _(dpooled, code, W2, dp_amax):
    return dpooled.new_empty((dpooled.shape[0], 32, 26, 26))


@torch.library.custom_op(f"{_NS}::conv2_wgrad", mutates_args=())
def conv2_wgrad(act: Tensor, dpooled: Tensor, code: Tensor) -> Tensor:
    """[dW2 (18432) | db2 (64)] (Winograd f32)."""
    return ops.reduce_slabs(ops.conv2_wgrad_slabs(act.contiguous(), dpooled.contiguous(), code.contiguous()))


@conv2_wgrad.register_fake
def _(act, dpooled, code):
    return act.new_empty((ops.CONV2_SLAB,))


@torch.library.custom_op(f"{_NS}::conv2_wgrad_x3", mutates_args=())
def conv2_wgrad_x3(act16: Tensor, act_amax: Tensor, dpooled: Tensor, dp_amax: Tensor, code: Tensor) -> Tensor:
    """[dW2 | db2] on the x3 kernel from the forward's split input images (act itself is not needed)."""
    return ops.reduce_slabs(ops.conv2_wgrad_slabs(None, dpooled.contiguous(), code.contiguous(), impl="x3",
                                                  act_amax=act_amax, dp_amax=dp_amax, act16=act16))


@conv2_wgrad_x3.register_fake
def _(act16, act_amax, dpooled, dp_amax, code):
    return dpooled.new_empty((ops.CONV2_SLAB,))


def _conv2_setup(ctx, inputs, output):
    act, W2, _b2 = inputs
    _pooled, code, amax, a16 = output
    ctx.impls = conv_impls()
    # the x3 wgrad reads the forward's split images: keep those (same size as act), not act
    keep = (a16, amax) if ctx.impls[2] == "x3" else (act,)
    ctx.save_for_backward(code, W2, *keep)
    ctx.mark_non_differentiable(code, amax, a16)
    # the backward never reads the gradients of code / amax / act16: without this autograd fills a zero
    # tensor for each (act16 is as large as the cut: ~60 us of memset per step at B = 4096)
    ctx.set_materialize_grads(False)


def _conv2_backward(ctx, dpooled, _dcode, _damax, _da16, K=None):
    K = K or torch.ops.splitcnn
    if dpooled is None:   # pooled did not reach the loss (grads are not materialized, _conv2_setup)
        return None, None, None
    code, W2, *kept = ctx.saved_tensors
    _fi, di, wi = ctx.impls
    dpa = None
    if "x3" in (di, wi):
        # fc1's input gradient comes with its per-sample max (linear_dgrad, fused); recomputed otherwise
        dpa = _MEMO.take("dp_amax", dpooled)
        # a per-row max fits only the producer's row layout: a permuted / transposed view of the same storage
        # (same key) must recompute
        if dpa is not None and not (dpooled.is_contiguous() and dpooled.shape[0] == dpa.numel()):
            dpa = None
        if dpa is None:
            dpa = K.row_amax(dpooled)
    gact = None
    if ctx.needs_input_grad[0]:
        gact = (K.conv2_dgrad_x3(dpooled, code, W2, dpa) if di == "x3" else K.conv2_dgrad(dpooled, code, W2))
    dW2 = db2 = None
    if ctx.needs_input_grad[1] or ctx.needs_input_grad[2]:
        flat = (K.conv2_wgrad_x3(kept[0], kept[1], dpooled, dpa, code) if wi == "x3"
                else K.conv2_wgrad(kept[0], dpooled, code))
        dW2, db2 = flat[:18432].view(64, 32, 3, 3), flat[18432:].view(64)
    return gact, dW2, db2


conv2_relu_pool.register_autograd(_conv2_backward, setup_context=_conv2_setup)


# ----------------------------------------------------------------------------------- fc1
@torch.library.custom_op(f"{_NS}::linear", mutates_args=())
def linear(flat: Tensor, W3: Tensor, b3: Tensor) -> Tensor:
    return ops.fc_fwd(flat.contiguous(), W3.contiguous(), b3.contiguous())


@linear.register_fake
def _(flat, W3, b3):
    return flat.new_empty((flat.shape[0], 10))


@torch.library.custom_op(f"{_NS}::linear_dgrad", mutates_args=())
def linear_dgrad(dlogits: Tensor, W3: Tensor) -> Tensor:
    """fc1's input gradient; the kernel also writes its per-sample max |.| (slk_fc_dgrad_amax), kept for
    the conv2 backward's x3 scales (no separate row_amax pass over dpooled)."""
    dlogits = dlogits.contiguous()
    amax = dlogits.new_empty((dlogits.shape[0],))
    dflat = ops.fc_dgrad(dlogits, W3.contiguous(), dp_amax=amax)
    _MEMO.put("dp_amax", dflat, amax)
    return dflat


@linear_dgrad.register_fake
def _(dlogits, W3):
    return dlogits.new_empty((dlogits.shape[0], 9216))


@torch.library.custom_op(f"{_NS}::linear_wgrad", mutates_args=())
def linear_wgrad(dlogits: Tensor, flat: Tensor) -> Tensor:
    """[dW3 (92160) | db3 (10)]."""
    return ops.reduce_slabs(ops.fc_wgrad_slabs(dlogits.contiguous(), flat.contiguous()))


@linear_wgrad.register_fake
def _(dlogits, flat):
    return dlogits.new_empty((ops.FC_SLAB,))


def _linear_setup(ctx, inputs, output):
    flat, W3, _b3 = inputs
    ctx.save_for_backward(flat, W3)


def _linear_backward(ctx, dlogits, K=None):
    K = K or torch.ops.splitcnn
    flat, W3 = ctx.saved_tensors
    dW3 = db3 = None
    # the weight gradient first: it re-reads flat (151 MB at B = 4096) while the forward's copy is still in
    # the Infinity Cache; the input gradient's 151 MB write would evict it (the fused step's order too)
    if ctx.needs_input_grad[1] or ctx.needs_input_grad[2]:
        g = K.linear_wgrad(dlogits, flat)
        dW3, db3 = g[:92160].view(10, 9216), g[92160:].view(10)
    dflat = K.linear_dgrad(dlogits, W3) if ctx.needs_input_grad[0] else None
    return dflat, dW3, db3


linear.register_autograd(_linear_backward, setup_context=_linear_setup)


# ----------------------------------------------------------------------------------- cross-entropy
@torch.library.custom_op(f"{_NS}::cross_entropy", mutates_args=())
def cross_entropy(logits: Tensor, labels: Tensor) -> Tensor:
    """Mean cross-entropy (nn.CrossEntropyLoss(), integer labels) as a 0-d tensor."""
    logits, labels = logits.contiguous(), labels.contiguous()
    loss_i, dlogits = ops.xent_fwd_bwd(logits, labels, 1.0 / logits.shape[0])
    _MEMO.put("dlogits", logits, (labels, labels._version, dlogits))   # the backward's (softmax - onehot) / B
    return ops.loss_mean(loss_i).view(())


@cross_entropy.register_fake
def _(logits, labels):
    return logits.new_empty(())


@torch.library.custom_op(f"{_NS}::cross_entropy_grad", mutates_args=())
def cross_entropy_grad(logits: Tensor, labels: Tensor, gloss: Tensor) -> Tensor:
    """d loss / d logits = (softmax - onehot) / B * gloss (the fused kernel, then the upstream scale)."""
    logits, labels = logits.contiguous(), labels.contiguous()
    hit = _MEMO.take("dlogits", logits)
    if hit is not None and hit[0].data_ptr() == labels.data_ptr() and hit[1] == labels._version:
        dlogits = hit[2]
    else:
        _, dlogits = ops.xent_fwd_bwd(logits, labels, 1.0 / logits.shape[0])
    return dlogits * gloss


@cross_entropy_grad.register_fake
def _(logits, labels, gloss):
    return torch.empty_like(logits)


def _xent_setup(ctx, inputs, output):
    logits, labels = inputs
    ctx.save_for_backward(logits, labels)


def _xent_backward(ctx, gloss, K=None):
    K = K or torch.ops.splitcnn
    logits, labels = ctx.saved_tensors
    return K.cross_entropy_grad(logits, labels, gloss), None


cross_entropy.register_autograd(_xent_backward, setup_context=_xent_setup)


# ----------------------------------------------------------------------------------- eager fast path
# The same implementations and backward formulas as the ops above, as plain autograd.Functions, for eager
# calls on real tensors (the reference's own step code on the drop-in modules): a torch.library custom-op
# call costs ~65 us of Python dispatch (CustomOpDef -> autograd_impl -> redispatch -> backend_impl), an
# autograd.Function ~15 us, and after the step's loss.item() sync the client backward + the next client
# forward sit on the GPU's critical path. Tracing (make_fx / torch.export / torch.compile: a dispatch mode,
# fake or functional tensors) keeps the custom ops, so the traced graphs are unchanged; results are the same
# kernels, bit for bit (tests/test_gpu_parity.py). SLK_EAGER_OPS=0 turns the fast path off.
class _Direct:
    """The ops' bodies without torch.library dispatch (the backward formulas' K for eager calls)."""


for _n in ("conv1_wgrad", "row_amax", "conv2_dgrad", "conv2_dgrad_x3", "conv2_wgrad", "conv2_wgrad_x3",
           "linear_dgrad", "linear_wgrad", "cross_entropy_grad"):
    setattr(_Direct, _n, staticmethod(globals()[_n]._init_fn))
_EAGER = os.environ.get("SLK_EAGER_OPS", "1") != "0"


def eager(*ts) -> bool:
    """True for an eager call on plain tensors (no dispatch mode, not compiling): the fast path applies."""
    if not _EAGER or torch.compiler.is_compiling() or torch._C._len_torch_dispatch_stack() > 0:
        return False
    return all(type(t) in (torch.Tensor, torch.nn.Parameter) for t in ts)


class Conv1ReluFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, W1, b1):
        out = conv1_relu._init_fn(x, W1, b1)
        _conv1_setup(ctx, (x, W1, b1), out)
        return out

    @staticmethod
    def backward(ctx, g):
        return _conv1_backward(ctx, g, _Direct)


class Conv2ReluPoolFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, act, W2, b2):
        out = conv2_relu_pool._init_fn(act, W2, b2)
        _conv2_setup(ctx, (act, W2, b2), out)
        return out

    @staticmethod
    def backward(ctx, dpooled, dcode, damax, da16):
        return _conv2_backward(ctx, dpooled, dcode, damax, da16, _Direct)


class LinearFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, flat, W3, b3):
        out = linear._init_fn(flat, W3, b3)
        _linear_setup(ctx, (flat, W3, b3), out)
        return out

    @staticmethod
    def backward(ctx, dlogits):
        return _linear_backward(ctx, dlogits, _Direct)


class CrossEntropyFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, logits, labels):
        out = cross_entropy._init_fn(logits, labels)
        _xent_setup(ctx, (logits, labels), out)
        return out

    @staticmethod
    def backward(ctx, gloss):
        return _xent_backward(ctx, gloss, _Direct)
