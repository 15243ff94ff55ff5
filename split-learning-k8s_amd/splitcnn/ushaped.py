"""Label-private U-shaped split.

The reference's README says the server holds the labels (README.md:5), but its client ships them
with every request (src/client_part.py:119). The U-shape keeps both ends of the network on the
client: the client runs conv1+ReLU AND the fc1 head + loss; the server runs only the conv2 trunk
(conv2+ReLU+max-pool). Per step:

    client:  act = relu(conv1(x))                      -> act          (cut 1, client -> server)
    server:  pooled, code = pool(relu(conv2(act)))     -> pooled       (cut 2, server -> client)
    client:  logits = fc1(pooled); CE(labels); dpooled; fc1 SGD; log loss
                                                        -> dpooled      (cut 2 grad, client -> server)
    server:  dW2/db2 + cut_grad from dpooled and code; conv2 SGD
                                                        -> cut_grad     (cut 1 grad, server -> client)
    client:  conv1 wgrad + SGD

Labels and logits never leave the client. Every gradient uses the pre-update weights, so the
result is exactly the reference's step (same oracle). The kernels are the split path's own:
conv2_fwd_pool / conv2_dgrad / conv2_wgrad on the server, fc_xent / fc_wgrad / conv1_* on the
client. `UShapedTrainer` runs both on one GPU; `dist.UShaped` puts them on two ranks.
"""
from typing import Optional

import torch

from . import ops
from .engine import CONV_DEFAULT, CONV_PRESETS, LR, TIMER, LossLog, _Buffers, _flatten_params
from .model_def import ModelPartA, ModelPartB


class UServerStage:
    """conv2 trunk of ModelPartB (model_def.py:18-20,24-26) + its SGD."""

    def __init__(self, model: Optional[ModelPartB] = None, lr: float = LR, device="cuda", conv: str = CONV_DEFAULT):
        self.device = torch.device(device)
        self.model = (model if model is not None else ModelPartB()).to(self.device)
        self.conv2 = self.model.conv2
        self.impl_fwd, self.impl_dgrad, self.impl_wgrad = CONV_PRESETS[conv]
        self.lr = lr
        self.params, self.grads = _flatten_params([self.conv2.weight, self.conv2.bias], self.device)
        self._buf = _Buffers()
        self._act = self._code = self._act16 = None

    def _b(self, name, shape, dtype=torch.float32):
        return self._buf.get(name, shape, dtype, self.device)

    def forward(self, act: torch.Tensor, pooled: Optional[torch.Tensor] = None) -> torch.Tensor:
        B = act.shape[0]
        W2, b2 = self.conv2.weight.detach(), self.conv2.bias.detach()
        amax = None
        if "x3" in (self.impl_fwd, self.impl_wgrad):
            amax = ops.row_amax(act, out=self._b("act_amax", (B,)))
        # x3 forward + x3 wgrad: the forward hands its split input images to the wgrad (as ServerStage)
        act16 = (self._b("act16", (ops.conv2_act16_bytes(B),), torch.uint8)
                 if (self.impl_fwd, self.impl_wgrad) == ("x3", "x3") else None)
        with TIMER("conv2_fwd_pool"):
            pooled, code = ops.conv2_fwd_pool(act, W2, b2,
                                              pooled=pooled if pooled is not None else self._b("pooled", (B, 64, 12, 12)),
                                              code=self._b("code", (B, 64, 12, 12), torch.uint8),
                                              impl=self.impl_fwd, act_amax=amax, act16=act16)
        self._act, self._code, self._amax, self._act16 = act, code, amax, act16
        return pooled

    def backward_step(self, dpooled: torch.Tensor, cut_grad: Optional[torch.Tensor] = None) -> torch.Tensor:
        """dpooled (cut-2 gradient) -> cut_grad (cut-1 gradient); then the conv2 SGD step."""
        act, code = self._act, self._code
        B = act.shape[0]
        W2 = self.conv2.weight.detach()
        cut_grad = cut_grad if cut_grad is not None else self._b("cut_grad", (B, 32, 26, 26))
        dpa = None
        if "x3" in (self.impl_dgrad, self.impl_wgrad):
            dpa = ops.row_amax(dpooled, out=self._b("dp_amax", (B,)))
        with TIMER("conv2_dgrad"):
            ops.conv2_dgrad(dpooled, code, W2, out=cut_grad, impl=self.impl_dgrad, dp_amax=dpa)
        with TIMER("conv2_wgrad"):
            s2 = ops.conv2_wgrad_slabs(act, dpooled, code,
                                       slabs=self._b("s2", (ops.conv2_wgrad_nslab(B, impl=self.impl_wgrad), ops.CONV2_SLAB)),
                                       impl=self.impl_wgrad, act_amax=self._amax, dp_amax=dpa, act16=self._act16)
        with TIMER("sgd_server"):
            ops.sgd_from_slabs(self.params, self.grads, s2, self.lr)
        return cut_grad


class UClientStage:
    """conv1 (ModelPartA) + the fc1 head of ModelPartB + CrossEntropyLoss + both SGDs + loss log."""

    def __init__(self, model_a: Optional[ModelPartA] = None, head: Optional[ModelPartB] = None,
                 lr: float = LR, device="cuda", loss_log: Optional[LossLog] = None):
        from .engine import ClientStage
        self.device = torch.device(device)
        self.conv = ClientStage(model_a, lr, self.device)
        head = head if head is not None else ModelPartB()
        self.fc1 = head.fc1.to(self.device)
        self.lr = lr
        self.params, self.grads = _flatten_params([self.fc1.weight, self.fc1.bias], self.device)
        self.loss_log = loss_log if loss_log is not None else LossLog(self.device)
        self.err_flag = torch.zeros(1, dtype=torch.int32, device=self.device)
        self._buf = _Buffers()

    def _b(self, name, shape, dtype=torch.float32):
        return self._buf.get(name, shape, dtype, self.device)

    def forward(self, x: torch.Tensor, out: Optional[torch.Tensor] = None) -> torch.Tensor:
        return self.conv.forward(x, out=out)

    def head_step(self, pooled: torch.Tensor, labels: torch.Tensor, step: Optional[int] = None,
                  dpooled: Optional[torch.Tensor] = None) -> torch.Tensor:
        """fc1 + CE (mean) + fc1 backward + fc1 SGD + loss log; returns dpooled (cut-2 gradient)."""
        B = pooled.shape[0]
        W3, b3 = self.fc1.weight.detach(), self.fc1.bias.detach()
        dpooled = dpooled if dpooled is not None else self._b("dpooled", (B, 64, 12, 12))
        with TIMER("fc_xent"):
            _, loss_i, dlogits, _ = ops.fc_xent(
                pooled, W3, b3, labels, 1.0 / B, logits=self._b("logits", (B, 10)),
                loss_i=self._b("loss_i", (B,)), dlogits=self._b("dlogits", (B, 10)),
                dpooled=dpooled, err_flag=self.err_flag)
        with TIMER("fc_wgrad"):
            s3 = ops.fc_wgrad_slabs(dlogits, pooled, slabs=self._b("s3", (ops.fc_wgrad_nslab(B), ops.FC_SLAB)))
        with TIMER("sgd_client"):
            ops.sgd_from_slabs(self.params, self.grads, s3, self.lr)
        with TIMER("loss_log"):
            ops.loss_log(loss_i, 1.0 / B, self.loss_log.ring, self.loss_log.counter)
        if step is not None:
            self.loss_log.note_step(step)
        return dpooled

    def backward_step(self, cut_grad: torch.Tensor) -> None:
        self.conv.backward_step(cut_grad)

    def check_labels(self):
        if int(self.err_flag.item()) != 0:
            raise IndexError("splitcnn: a label was out of range [0, 10)")


class UShapedTrainer:
    """Both U-shape halves on one GPU (cut tensors handed over in place)."""

    def __init__(self, model_a: Optional[ModelPartA] = None, model_b: Optional[ModelPartB] = None,
                 lr: float = LR, device="cuda", conv: str = CONV_DEFAULT):
        model_b = model_b if model_b is not None else ModelPartB()
        self.client = UClientStage(model_a, model_b, lr, device)
        self.server = UServerStage(model_b, lr, device, conv=conv)
        self.global_step = 0

    @property
    def loss_log(self) -> LossLog:
        return self.client.loss_log

    def step(self, x: torch.Tensor, y: torch.Tensor) -> None:
        act = self.client.forward(x)
        pooled = self.server.forward(act)
        dpooled = self.client.head_step(pooled, y, step=self.global_step)
        cut_grad = self.server.backward_step(dpooled)
        self.client.backward_step(cut_grad)
        self.global_step += 1
