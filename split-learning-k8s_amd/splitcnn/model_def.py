"""Drop-in replacement of the reference's module contract (src/model_def.py:1-71).

Same class names, attribute names, state_dict keys, parameter shapes, default initialisation and RNG
consumption order (conv1, conv2, fc1 — src/model_def.py:8,18,22), and the same `get_model(role)`
dispatch on LEARNING_MODE (src/model_def.py:49-71). What changes is where the arithmetic runs: every
forward and backward goes through the hand-written gfx950 kernels of libslk.so via the autograd
Functions below (eager calls: autograd.Functions over the same implementations, library.eager). The nn.Conv2d / nn.Linear submodules are kept ONLY as parameter containers (so
`model.conv1.weight`, `load_state_dict` and default init behave exactly as in the reference); their
own forward is never called. Modules must live on a ROCm device; CPU tensors raise. The ops are
registered with torch.library (library.py), with fake kernels, so the modules also trace under
torch.export / make_fx.

Autograd behaves like the reference's: the server module is differentiable w.r.t. its input, so the
server's `client_activations.requires_grad_(True)` / `.grad` pattern (src/server_part.py:45,57) works,
and `activations.backward(grad)` on the client output (src/client_part.py:132) fills conv1's grads.
"""
from __future__ import annotations

import os

import torch
import torch.nn as nn

from . import ops


# ----------------------------------------------------------------------------- operators
# The arithmetic of every forward and backward is a `splitcnn::` custom op (library.py: torch.library
# registrations with fake kernels and autograd formulas over libslk.so), so the modules trace under
# torch.export / make_fx as opaque differentiable operators.
from . import library  # noqa: E402,F401  (registers torch.ops.splitcnn.*)
from .library import Conv1ReluFn, Conv2ReluPoolFn, CrossEntropyFn, LinearFn, eager  # noqa: E402

_OPS = torch.ops.splitcnn


# eager calls on plain tensors take the same kernels through autograd.Functions (library.eager: less Python
# dispatch on the step's critical path); traced / exported / compiled calls go through the custom ops
def _conv1(x, W, b):
    return Conv1ReluFn.apply(x, W, b) if eager(x, W, b) else _OPS.conv1_relu(x, W, b)


def _conv2(x, W, b):
    return (Conv2ReluPoolFn.apply(x, W, b) if eager(x, W, b) else _OPS.conv2_relu_pool(x, W, b))[0]


def _linear(f, W, b):
    return LinearFn.apply(f, W, b) if eager(f, W, b) else _OPS.linear(f, W, b)


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
        return _conv1(x, self.conv1.weight, self.conv1.bias)


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
        pooled = _conv2(x, self.conv2.weight, self.conv2.bias)
        return _linear(pooled.view(pooled.shape[0], 9216), self.fc1.weight, self.fc1.bias)


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
        act = _conv1(x, self.conv1.weight, self.conv1.bias)
        pooled = _conv2(act, self.conv2.weight, self.conv2.bias)
        return _linear(pooled.view(pooled.shape[0], 9216), self.fc1.weight, self.fc1.bias)


class CrossEntropyLoss(nn.Module):
    """Drop-in for nn.CrossEntropyLoss() as the reference uses it (mean, integer class labels)."""

    def forward(self, logits, labels):
        _require_device(logits, "CrossEntropyLoss")
        return CrossEntropyFn.apply(logits, labels) if eager(logits, labels) else _OPS.cross_entropy(logits, labels)


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
