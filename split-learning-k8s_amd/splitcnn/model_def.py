"""Drop-in replacement of the reference's module contract (src/model_def.py:1-71).

Same class names, attribute names, state_dict keys, parameter shapes, default initialisation and RNG
consumption order (conv1, conv2, fc1 — src/model_def.py:8,18,22), and the same `get_model(role)`
dispatch on LEARNING_MODE (src/model_def.py:49-71). What changes is where the arithmetic runs: every
forward and backward goes through the hand-written gfx950 kernels of libslk.so via the autograd
Functions below. The nn.Conv2d / nn.Linear submodules are kept ONLY as parameter containers (so
`model.conv1.weight`, `load_state_dict` and default init behave exactly as in the reference); their
own forward is never called. Modules must live on a ROCm device; CPU tensors raise.

Autograd behaves like the reference's: the server module is differentiable w.r.t. its input, so the
server's `client_activations.requires_grad_(True)` / `.grad` pattern (src/server_part.py:45,57) works,
and `activations.backward(grad)` on the client output (src/client_part.py:132) fills conv1's grads.
"""
from __future__ import annotations

import os

import torch
import torch.nn as nn

from . import ops


# ----------------------------------------------------------------------------- autograd functions
class Conv1ReLU(torch.autograd.Function):
    """act = relu(conv1(x)) — ModelPartA.forward (src/model_def.py:11-12)."""

    @staticmethod
    def forward(ctx, x, W1, b1):
        x = x.contiguous()
        act = ops.conv1_fwd(x, W1.detach(), b1.detach())
        ctx.save_for_backward(x, act)
        return act

    @staticmethod
    def backward(ctx, g):
        x, act = ctx.saved_tensors
        if ctx.needs_input_grad[0]:
            raise NotImplementedError(
                "splitcnn: gradient w.r.t. the client INPUT images is not part of the split step "
                "(the reference's data never requires grad, src/client_part.py:110-114)")
        flat = ops.reduce_slabs(ops.conv1_wgrad_slabs(x, act, g.contiguous()))
        return None, flat[:288].view(32, 1, 3, 3), flat[288:].view(32)


class Conv2ReLUPool(torch.autograd.Function):
    """pooled = maxpool2(relu(conv2(act))) — src/model_def.py:25-26."""

    @staticmethod
    def forward(ctx, act, W2, b2):
        act = act.contiguous()
        pooled, code = ops.conv2_fwd_pool(act, W2.detach(), b2.detach())
        ctx.save_for_backward(act, code, W2)
        ctx.mark_non_differentiable(code)
        return pooled, code

    @staticmethod
    def backward(ctx, dpooled, _dcode):
        act, code, W2 = ctx.saved_tensors
        dpooled = dpooled.contiguous()
        gact = ops.conv2_dgrad(dpooled, code, W2.detach()) if ctx.needs_input_grad[0] else None
        dW2 = db2 = None
        if ctx.needs_input_grad[1] or ctx.needs_input_grad[2]:
            flat = ops.reduce_slabs(ops.conv2_wgrad_slabs(act, dpooled, code))
            dW2, db2 = flat[:18432].view(64, 32, 3, 3), flat[18432:].view(64)
        return gact, dW2, db2


class Linear9216x10(torch.autograd.Function):
    """logits = flat @ W3^T + b3 — fc1 (src/model_def.py:22,28)."""

    @staticmethod
    def forward(ctx, flat, W3, b3):
        flat = flat.contiguous()
        logits = ops.fc_fwd(flat, W3.detach(), b3.detach())
        ctx.save_for_backward(flat, W3)
        return logits

    @staticmethod
    def backward(ctx, dlogits):
        flat, W3 = ctx.saved_tensors
        dlogits = dlogits.contiguous()
        dflat = ops.fc_dgrad(dlogits, W3.detach()) if ctx.needs_input_grad[0] else None
        dW3 = db3 = None
        if ctx.needs_input_grad[1] or ctx.needs_input_grad[2]:
            g = ops.reduce_slabs(ops.fc_wgrad_slabs(dlogits, flat))
            dW3, db3 = g[:92160].view(10, 9216), g[92160:].view(10)
        return dflat, dW3, db3


class CrossEntropyMean(torch.autograd.Function):
    """nn.CrossEntropyLoss() (mean, no label smoothing) — src/server_part.py:16,49."""

    @staticmethod
    def forward(ctx, logits, labels):
        logits = logits.contiguous()
        B = logits.shape[0]
        loss_i, dlogits = ops.xent_fwd_bwd(logits, labels, 1.0 / B)
        ctx.save_for_backward(dlogits)
        return ops.loss_mean(loss_i).view(())

    @staticmethod
    def backward(ctx, gloss):
        (dlogits,) = ctx.saved_tensors
        return dlogits * gloss, None


# ----------------------------------------------------------------------------- modules
def _require_device(x: torch.Tensor, who: str):
    if x.device.type != "cuda":
        raise RuntimeError(
            f"splitcnn.{who}: input is on {x.device}; these modules run on the MI355X HIP kernels "
            "only. Move the module and its inputs to a ROCm device (model.to('cuda')).")


class ModelPartA(nn.Module):
    """Client bottom stack: conv1(1->32, 3x3) + ReLU (src/model_def.py:5-12)."""

    def __init__(self):
        super().__init__()
        self.conv1 = nn.Conv2d(1, 32, 3, 1)  # parameter container (init + state_dict keys)
        self.relu = nn.ReLU()

    def forward(self, x):
        _require_device(x, "ModelPartA")
        return Conv1ReLU.apply(x, self.conv1.weight, self.conv1.bias)


class ModelPartB(nn.Module):
    """Server top stack: conv2 -> ReLU -> maxpool2 -> flatten -> fc1 (src/model_def.py:15-28)."""

    def __init__(self):
        super().__init__()
        self.conv2 = nn.Conv2d(32, 64, 3, 1)
        self.relu = nn.ReLU()
        self.pool = nn.MaxPool2d(2)
        self.flatten = nn.Flatten()
        self.fc1 = nn.Linear(9216, 10)

    def forward(self, x):
        _require_device(x, "ModelPartB")
        pooled, _code = Conv2ReLUPool.apply(x, self.conv2.weight, self.conv2.bias)
        return Linear9216x10.apply(pooled.view(pooled.shape[0], 9216), self.fc1.weight, self.fc1.bias)


class FullModel(nn.Module):
    """The unsplit network (src/model_def.py:31-46); same parameter names as A ∪ B."""

    def __init__(self):
        super().__init__()
        self.conv1 = nn.Conv2d(1, 32, 3, 1)
        self.conv2 = nn.Conv2d(32, 64, 3, 1)
        self.relu = nn.ReLU()
        self.pool = nn.MaxPool2d(2)
        self.flatten = nn.Flatten()
        self.fc1 = nn.Linear(9216, 10)

    def forward(self, x):
        _require_device(x, "FullModel")
        act = Conv1ReLU.apply(x, self.conv1.weight, self.conv1.bias)
        pooled, _code = Conv2ReLUPool.apply(act, self.conv2.weight, self.conv2.bias)
        return Linear9216x10.apply(pooled.view(pooled.shape[0], 9216), self.fc1.weight, self.fc1.bias)


class CrossEntropyLoss(nn.Module):
    """Drop-in for nn.CrossEntropyLoss() as the reference uses it (mean, integer class labels)."""

    def forward(self, logits, labels):
        _require_device(logits, "CrossEntropyLoss")
        return CrossEntropyMean.apply(logits, labels)


def get_model(role="client"):
    """Reference factory (src/model_def.py:49-71): LEARNING_MODE in {split, federated},
    case-insensitive, default "split"; anything else raises ValueError."""
    learning_mode = os.getenv("LEARNING_MODE", "split").lower()
    if learning_mode == "federated":
        return FullModel()
    elif learning_mode == "split":
        if role == "client":
            return ModelPartA()
        return ModelPartB()
    raise ValueError(f"Unknown LEARNING_MODE: {learning_mode}. Use 'split' or 'federated'.")
