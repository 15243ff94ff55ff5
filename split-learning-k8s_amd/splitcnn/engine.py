"""The split-CNN step engine: client stage, server stage and the 1-GPU fused trainer.

This is the MI355X-native form of the reference's step contract (src/client_part.py:110-138 <->
src/server_part.py:25-58):

    client:  zero_grad; act = model(x)                         (client_part.py:112-114)
             send {act.detach(), labels, step}                 (client_part.py:117-125)
    server:  act.requires_grad_(True); zero_grad; fwd; CE loss; backward; SGD step;
             log loss at step; return act.grad                 (server_part.py:45-58)
    client:  act.backward(cut_grad); SGD step; step += 1      (client_part.py:131-138)

API: ``ClientStage.forward(x) -> act``, ``ServerStage.step(act, labels, step) ->
(cut_grad, loss)``, ``ClientStage.backward_step(cut_grad)``. Each stage keeps its parameters in ONE
flat device block (the module's Parameters become views of it, so state_dict / load_state_dict keep
working) and its gradients in another; the weight-gradient slabs of the wgrad kernels are reduced in
fixed order inside the fused SGD launch. Nothing synchronises with the host: the loss goes to a
device ring (LossLog) flushed every N steps, replacing the per-step mlflow.log_metric REST call
(server_part.py:55). `SplitTrainer` runs both stages on one GPU and captures the whole step in a
HIP graph.
"""
from __future__ import annotations

import contextlib
from collections import defaultdict
from typing import Callable, Dict, List, Optional, Tuple

import torch
import torch.nn as nn

from . import ops
from .model_def import ModelPartA, ModelPartB

LR = 0.01  # optim.SGD(lr=0.01) on both sides (client_part.py:17, server_part.py:15)


class KernelTimer:
    """HIP-event timing of named launches on the launching (current) stream. Disabled by default;
    bench.py enables it for its per-kernel pass. Never enable inside graph capture."""

    def __init__(self):
        self.enabled = False
        self._ev: Dict[str, list] = defaultdict(list)

    @contextlib.contextmanager
    def __call__(self, name: str):
        if not self.enabled:
            yield
            return
        s = torch.cuda.Event(enable_timing=True)
        e = torch.cuda.Event(enable_timing=True)
        s.record()
        yield
        e.record()
        self._ev[name].append((s, e))

    def reset(self):
        self._ev.clear()

    def summary(self) -> Dict[str, Dict[str, float]]:
        torch.cuda.synchronize()
        out = {}
        for k, v in self._ev.items():
            ms = [s.elapsed_time(e) for s, e in v]
            out[k] = {"avg_ms": sum(ms) / len(ms), "min_ms": min(ms), "n": len(ms)}
        return out


TIMER = KernelTimer()


def _flatten_params(params: List[nn.Parameter], device) -> Tuple[torch.Tensor, torch.Tensor]:
    """Move `params` into one flat fp32 block; each Parameter becomes a view of it."""
    n = sum(p.numel() for p in params)
    flat = torch.empty(n, dtype=torch.float32, device=device)
    gflat = torch.zeros(n, dtype=torch.float32, device=device)
    off = 0
    for p in params:
        k = p.numel()
        flat[off:off + k].copy_(p.detach().reshape(-1).to(device=device, dtype=torch.float32))
        p.data = flat[off:off + k].view(p.shape)
        p.grad = gflat[off:off + k].view(p.shape)
        off += k
    return flat, gflat


class _Buffers:
    """Per-batch-size scratch owned by a stage (allocated once, reused every step).

    Keyed by (name, shape, dtype, device): a buffer is never replaced, so a HIP graph captured at one
    batch size keeps valid pointers after another size has run (a ragged loader alternates 64 / 32)."""

    def __init__(self):
        self._b = {}

    def get(self, name, shape, dtype, device):
        key = (name, tuple(shape), dtype, torch.device(device))
        t = self._b.get(key)
        if t is None:
            t = torch.empty(shape, dtype=dtype, device=device)
            self._b[key] = t
        return t


class LossLog:
    """Device-side loss log: one ring slot per server step, written by slk_loss_log (the device
    counter advances inside the kernel, so graph replays log too). `flush()` copies the ring to the
    host once and returns/sinks [(step, loss)] — the replacement of mlflow.log_metric("loss", ...,
    step=step) (src/server_part.py:55)."""

    def __init__(self, device, capacity: int = 4096, sink: Optional[Callable[[int, float], None]] = None):
        self.device = torch.device(device)
        self.capacity = capacity
        self.ring = torch.zeros(capacity, dtype=torch.float32, device=self.device)
        self.counter = torch.zeros(1, dtype=torch.int32, device=self.device)
        self.sink = sink
        self._flushed = 0            # number of entries already flushed
        self._steps: List[int] = []  # host-side step ids, in logging order (no device sync needed)
        self.history: List[Tuple[int, float]] = []

    def note_step(self, step: int):
        self._steps.append(int(step))

    def flush(self) -> List[Tuple[int, float]]:
        count = int(self.counter.item())
        new = count - self._flushed
        if new <= 0:
            return []
        if new > self.capacity:
            raise RuntimeError(f"LossLog overflow: {new} unflushed steps > capacity {self.capacity}")
        ring = self.ring.cpu()
        out = []
        for i in range(self._flushed, count):
            step = self._steps[i] if i < len(self._steps) else i
            loss = float(ring[i % self.capacity])
            out.append((step, loss))
            if self.sink is not None:
                self.sink(step, loss)
        self._flushed = count
        self.history.extend(out)
        if self.sink is not None and hasattr(self.sink, "flush"):
            self.sink.flush()  # batching sinks (splitcnn.sinks) send once per flush
        return out


# conv2 implementations per op (forward+pool, dgrad, wgrad): "f32" = the Winograd F(2x2,3x3) kernels
# on the f32 MFMA; "x3" = the f16-MFMA kernels with hi/lo-split f32 operands (csrc/slk_x3.hip) where
# are used for all three ("x3"), or for forward + dgrad with the Winograd wgrad ("x3w").
CONV_PRESETS = {"f32": ("wino", "wino", "wino"), "x3": ("x3", "x3", "x3"), "x3w": ("x3", "x3", "wino")}
CONV_DEFAULT = "x3"


class ClientStage:
    """Client half: ModelPartA on one device + SGD (src/client_part.py:16-17,112-133).

    forward(x) -> act; then either backward_step(cut_grad) (fused wgrad-slab reduce + SGD, the
    reference's `activations.backward(grads); optimizer.step()`), or backward(cut_grad,
    accumulate=...) into the flat gradient block followed by step() (micro-batched / all-reduced
    topologies)."""

    def __init__(self, model: Optional[ModelPartA] = None, lr: float = LR, device="cuda"):
        self.device = torch.device(device)
        self.model = (model if model is not None else ModelPartA()).to(self.device)
        self.lr = lr
        self.params, self.grads = _flatten_params(
            [self.model.conv1.weight, self.model.conv1.bias], self.device)
        self._buf = _Buffers()
        self._x = None
        self._act = None
        self._act_amax = None
        self._act16 = None
        self._relu_bits = None
        self.emit_amax = False  # forward also writes the per-sample max of act (x3 server kernels)
        # forward writes the x3 server operand (act16 images + act_amax) instead of the f32 act: the
        # fused single-GPU step, where the cut never leaves the device (forward then returns None)
        self.emit_act16 = False

    @property
    def W1(self):
        return self.model.conv1.weight

    @property
    def b1(self):
        return self.model.conv1.bias

    def bind_grads(self, view: torch.Tensor):
        """Use `view` (320 floats, e.g. a slice of an all-reduce bucket) as the gradient block."""
        view.copy_(self.grads)
        self.grads = view
        self.model.conv1.weight.grad = view[:288].view(32, 1, 3, 3)
        self.model.conv1.bias.grad = view[288:].view(32)

    def forward(self, x: torch.Tensor, out: Optional[torch.Tensor] = None) -> torch.Tensor:
        """act = relu(conv1(x)) (client_part.py:114). Keeps x/act for the backward."""
        B = x.shape[0]
        if self.emit_act16:
            amax = self._buf.get("act_amax", (B,), torch.float32, self.device)
            a16 = self._buf.get("act16", (ops.conv2_act16_bytes(B),), torch.uint8, self.device)
            bits = self._buf.get("relu_bits", (B, ops.RELU_BITS_WORDS), torch.int32, self.device)
            with TIMER("conv1_fwd"):
                act = ops.conv1_fwd_x3(x, self.W1.detach(), self.b1.detach(), amax, a16, act=out, relu_bits=bits)
            self._x, self._act, self._act_amax, self._act16, self._relu_bits = x, act, amax, a16, bits
            return act
        act = out if out is not None else self._buf.get("act", (B, 32, 26, 26), torch.float32, self.device)
        amax = self._buf.get("act_amax", (B,), torch.float32, self.device) if self.emit_amax else None
        with TIMER("conv1_fwd"):
            ops.conv1_fwd(x, self.W1.detach(), self.b1.detach(), out=act, act_amax=amax)
        self._x, self._act, self._act_amax = x, act, amax
        return act

    def forward_images(self, x: torch.Tensor, act16: torch.Tensor, act_amax: torch.Tensor) -> None:
        """act = relu(conv1(x)) (client_part.py:114) written as the server's x3 operand into caller
        buffers — act16 images (ops.conv2_act16_bytes(B) bytes) + the per-sample max — for the image
        exchange of dist.Hub (images=True). No f32 act and no ReLU bit map: this client's backward
        re-derives its mask from x."""
        with TIMER("conv1_fwd"):
            ops.conv1_fwd_x3(x, self.W1.detach(), self.b1.detach(), act_amax, act16)
        self._x, self._act, self._act_amax, self._act16 = x, None, act_amax, act16

    def _slabs(self, cut_grad, x, act, tag="slabs"):
        x = self._x if x is None else x
        act = self._act if act is None else act
        B = x.shape[0]
        slabs = self._buf.get(tag, (ops.conv1_wgrad_nslab(B), ops.CLIENT_NPARAM), torch.float32, self.device)
        with TIMER("conv1_wgrad"):
            # the mask act > 0 is recomputed from x and W1 (unchanged since the forward: the client
            # steps after its backward), so only x and cut_grad are read
            ops.conv1_wgrad_remask_slabs(x, self.W1.detach(), self.b1.detach(), cut_grad, slabs=slabs)
        return slabs

    def backward_step(self, cut_grad: torch.Tensor, x: Optional[torch.Tensor] = None,
                      act: Optional[torch.Tensor] = None) -> None:
        """act.backward(cut_grad); optimizer.step() (client_part.py:132-133): relu-bwd + conv1
        wgrad slabs, then ONE fused reduce+SGD launch over the 320 client parameters."""
        slabs = self._slabs(cut_grad, x, act)
        with TIMER("sgd_client"):
            ops.sgd_from_slabs(self.params, self.grads, slabs, self.lr)

    def step_from_slabs(self, slabs: torch.Tensor) -> None:
        """optimizer.step() from gradient slabs produced elsewhere (the server's fused x3 dgrad,
        ServerStage.forward_backward(client_fuse=...)): one fused reduce + SGD launch."""
        with TIMER("sgd_client"):
            ops.sgd_from_slabs(self.params, self.grads, slabs, self.lr)

    def backward(self, cut_grad: torch.Tensor, x: Optional[torch.Tensor] = None,
                 act: Optional[torch.Tensor] = None, accumulate: bool = False) -> None:
        """Weight gradient into self.grads (accumulate=True adds: micro-batches)."""
        slabs = self._slabs(cut_grad, x, act)
        ops.reduce_slabs(slabs, out=self.grads, accumulate=accumulate)

    def step(self):
        """SGD from the (already reduced / all-reduced) flat gradient block."""
        with TIMER("sgd_client"):
            ops.sgd(self.params, self.grads, self.lr)


class ServerStage:
    """Server half: ModelPartB + CrossEntropyLoss + SGD + loss log (src/server_part.py:14-16,25-58)."""

    def __init__(self, model: Optional[ModelPartB] = None, lr: float = LR, device="cuda",
                 loss_log: Optional[LossLog] = None, conv: str = CONV_DEFAULT):
        self.device = torch.device(device)
        self.conv = conv
        self.impl_fwd, self.impl_dgrad, self.impl_wgrad = CONV_PRESETS[conv]
        self.share_images = True  # x3: the forward's split input images feed the wgrad (act16)
        self.model = (model if model is not None else ModelPartB()).to(self.device)
        self.lr = lr
        m = self.model
        self.params, self.grads = _flatten_params(
            [m.conv2.weight, m.conv2.bias, m.fc1.weight, m.fc1.bias], self.device)
        self.loss_log = loss_log if loss_log is not None else LossLog(self.device)
        self.err_flag = torch.zeros(1, dtype=torch.int32, device=self.device)
        self.fuse_optim = True  # step_request: SGD of both slab kinds + the loss log in one launch
        # launch order knobs (profiling, tools/ab_trainers.py): fc1 wgrad right after the head (pooled
        # just read by it), conv2 wgrad before the dgrad. Defaults: the measured fastest order.
        self.fc_wgrad_early = False
        self.wgrad_first = False
        # the head as logits + cross-entropy, fc1 wgrad, then dpooled (+ dp_amax): fc1 wgrad re-reads
        # pooled while it is still in the Infinity Cache (the fused head's own 151 MB dpooled write
        # evicts it); same kernels, bit-identical results (tools/x3_ab.py --ops fcord --flush: 0.1010 ->
        # 0.0970 ms for head + fc1 wgrad from cold caches)
        self.fc_split = True
        # ... with its logits and cross-entropy in one launch (slk_fc_logits_xent, round 6; bitwise the two)
        self.fc_one_launch = True
        self._buf = _Buffers()

    def bind_grads(self, view: torch.Tensor):
        view.copy_(self.grads)
        self.grads = view
        m = self.model
        m.conv2.weight.grad = view[:18432].view(64, 32, 3, 3)
        m.conv2.bias.grad = view[18432:18496].view(64)
        m.fc1.weight.grad = view[18496:110656].view(10, 9216)
        m.fc1.bias.grad = view[110656:].view(10)

    def _b(self, name, shape, dtype=torch.float32):
        return self._buf.get(name, shape, dtype, self.device)

    def forward_backward(self, act: Optional[torch.Tensor], labels: torch.Tensor, grad_scale: float,
                         cut_grad: Optional[torch.Tensor] = None, act_amax: Optional[torch.Tensor] = None,
                         act16: Optional[torch.Tensor] = None, client_fuse=None, cut_pack=None):
        """Server forward + CE + backward WITHOUT the optimizer step. Returns (cut_grad, loss_i,
        conv2 slabs, fc slabs). grad_scale = 1/global_batch (mean loss). act_amax: the per-sample x3
        scale bound of act when the client produced it (ClientStage.emit_amax: conv1_cut_bound, >= max act;
        only its power of two is used); the x3 kernels compute the exact max otherwise.
        act16 (with act_amax, x3 forward + wgrad only): the client's split input images
        (ClientStage.emit_act16) — act is then not read and may be None. client_fuse = (x, relu_bits,
        slabs) (x3 dgrad only, single-GPU step): the dgrad also runs the client's ReLU backward +
        conv1 wgrad into `slabs` and the cut gradient is not materialised (returned as None).
        cut_pack = (parts, part_b) (x3 dgrad only; the codec exchange, dist.Hub): the cut gradient leaves
        packed at the positions of each part's received mask — parts = int64 device table [B / part_b, 3] of
        (mask, ranks, vals) pointers, one part per part_b samples (ops.conv2_dgrad_x3_pack_parts) — instead
        of dense; returned as None."""
        B = labels.shape[0]
        m = self.model
        W2, b2 = m.conv2.weight.detach(), m.conv2.bias.detach()
        W3, b3 = m.fc1.weight.detach(), m.fc1.bias.detach()
        fi, di, wi = self.impl_fwd, self.impl_dgrad, self.impl_wgrad
        if act16 is not None and ((fi, wi) != ("x3", "x3") or act_amax is None):
            raise ValueError("act16 input needs the x3 forward and wgrad (conv preset 'x3') and act_amax")
        if act_amax is None and "x3" in (fi, wi):
            with TIMER("act_amax"):
                act_amax = ops.row_amax(act, out=self._b("act_amax", (B,)))
        dp_amax = self._b("dp_amax", (B,)) if "x3" in (di, wi) else None
        pooled_b, code_b = self._b("pooled", (B, 64, 12, 12)), self._b("code", (B, 64, 12, 12), torch.uint8)
        if act16 is not None:
            with TIMER("conv2_fwd_pool"):
                pooled, code = ops.conv2_fwd_pool_x3i(act16, act_amax, W2, b2, pooled=pooled_b, code=code_b)
        else:
            # x3 forward + x3 wgrad: the forward hands its split input images to the wgrad (LDS-DMA copy)
            act16 = (self._b("act16", (ops.conv2_act16_bytes(B),), torch.uint8)
                     if fi == "x3" and wi == "x3" and self.share_images else None)
            with TIMER("conv2_fwd_pool"):
                pooled, code = ops.conv2_fwd_pool(act, W2, b2, pooled=pooled_b, code=code_b, impl=fi,
                                                  act_amax=act_amax, act16=act16)
        split = self.fc_split and dp_amax is not None
        if split:
            with TIMER("fc_xent"):
                if self.fc_one_launch:
                    _, loss_i, dlogits = ops.fc_logits_xent(
                        pooled, W3, b3, labels, grad_scale, logits=self._b("logits", (B, 10)),
                        loss_i=self._b("loss_i", (B,)), dlogits=self._b("dlogits", (B, 10)), err_flag=self.err_flag)
                else:
                    logits = ops.fc_fwd(pooled, W3, b3, out=self._b("logits", (B, 10)))
                    loss_i, dlogits = ops.xent_fwd_bwd(logits, labels, grad_scale, loss_i=self._b("loss_i", (B,)),
                                                       dlogits=self._b("dlogits", (B, 10)), err_flag=self.err_flag)
            with TIMER("fc_wgrad"):
                s3 = ops.fc_wgrad_slabs(dlogits, pooled, slabs=self._b("s3", (ops.fc_wgrad_nslab(B), ops.FC_SLAB)))
            dpooled = self._b("dpooled", (B, 64, 12, 12))
            with TIMER("fc_dgrad"):
                ops.fc_dgrad(dlogits, W3, out=dpooled.view(B, 9216), dp_amax=dp_amax)
        else:
            with TIMER("fc_xent"):
                _, loss_i, dlogits, dpooled = ops.fc_xent(
                    pooled, W3, b3, labels, grad_scale, logits=self._b("logits", (B, 10)),
                    loss_i=self._b("loss_i", (B,)), dlogits=self._b("dlogits", (B, 10)),
                    dpooled=self._b("dpooled", (B, 64, 12, 12)), err_flag=self.err_flag, dp_amax=dp_amax)
        # launch order dgrad -> wgrad -> fc wgrad (measured fastest: DESIGN.md §3a "Launch order")
        if self.fc_wgrad_early and not split:
            with TIMER("fc_wgrad"):
                s3 = ops.fc_wgrad_slabs(dlogits, pooled, slabs=self._b("s3", (ops.fc_wgrad_nslab(B), ops.FC_SLAB)))

        def wgrad():
            with TIMER("conv2_wgrad"):
                return ops.conv2_wgrad_slabs(act, dpooled, code,
                                             slabs=self._b("s2", (ops.conv2_wgrad_nslab(B, impl=wi), ops.CONV2_SLAB)),
                                             impl=wi, act_amax=act_amax, dp_amax=dp_amax, act16=act16)
        if self.wgrad_first:
            s2 = wgrad()
        if cut_pack is not None:
            if di != "x3":
                raise ValueError("cut_pack needs the x3 dgrad (conv preset 'x3' or 'x3w')")
            with TIMER("conv2_dgrad"):
                ops.conv2_dgrad_x3_pack_parts(dpooled, code, W2, dp_amax, *cut_pack)
            cut_grad = None
        elif client_fuse is not None:
            if di != "x3":
                raise ValueError("client_fuse needs the x3 dgrad (conv preset 'x3' or 'x3w')")
            cx, cbits, cslabs = client_fuse
            with TIMER("conv2_dgrad"):
                ops.conv2_dgrad_client_slabs(dpooled, code, W2, cx, cbits, dp_amax=dp_amax, slabs=cslabs)
            cut_grad = None
        else:
            if cut_grad is None:
                cut_grad = self._b("cut_grad", (B, 32, 26, 26))
            with TIMER("conv2_dgrad"):
                ops.conv2_dgrad(dpooled, code, W2, out=cut_grad, impl=di, dp_amax=dp_amax)
        if not self.wgrad_first:
            s2 = wgrad()
        if not self.fc_wgrad_early and not split:
            with TIMER("fc_wgrad"):
                s3 = ops.fc_wgrad_slabs(dlogits, pooled, slabs=self._b("s3", (ops.fc_wgrad_nslab(B), ops.FC_SLAB)))
        return cut_grad, loss_i, s2, s3

    def apply_grad_slabs(self, s2, s3):
        """optimizer.step() (server_part.py:52): two fused reduce+SGD launches, one per slab kind."""
        with TIMER("sgd_server"):
            ops.sgd_from_slabs(self.params[:ops.CONV2_SLAB], self.grads[:ops.CONV2_SLAB], s2, self.lr)
            ops.sgd_from_slabs(self.params[ops.CONV2_SLAB:], self.grads[ops.CONV2_SLAB:], s3, self.lr)

    def reduce_grads(self, s2, s3, accumulate: bool = False):
        """Reduce slabs into the flat gradient block without stepping (micro-batches, all-reduce)."""
        ops.reduce_slabs(s2, out=self.grads[:ops.CONV2_SLAB], accumulate=accumulate)
        ops.reduce_slabs(s3, out=self.grads[ops.CONV2_SLAB:], accumulate=accumulate)

    def compute(self, act, labels, grad_scale, accumulate=False, cut_grad=None, act_amax=None, act16=None,
                cut_pack=None):
        """forward_backward + reduce into self.grads; returns (cut_grad, loss_i)."""
        cut_grad, loss_i, s2, s3 = self.forward_backward(act, labels, grad_scale, cut_grad=cut_grad,
                                                         act_amax=act_amax, act16=act16, cut_pack=cut_pack)
        self.reduce_grads(s2, s3, accumulate=accumulate)
        return cut_grad, loss_i

    def step(self):
        with TIMER("sgd_server"):
            ops.sgd(self.params, self.grads, self.lr)

    def log_loss(self, values, scale: Optional[float] = None, step: Optional[int] = None):
        """Log scale*sum(values) (default: the mean of per-sample losses) for `step`."""
        scale = 1.0 / values.numel() if scale is None else scale
        with TIMER("loss_log"):
            ops.loss_log(values, scale, self.loss_log.ring, self.loss_log.counter)
        if step is not None:
            self.loss_log.note_step(step)

    def step_request(self, act: Optional[torch.Tensor], labels: torch.Tensor, step: Optional[int] = None,
                     cut_grad: Optional[torch.Tensor] = None, act_amax: Optional[torch.Tensor] = None,
                     act16: Optional[torch.Tensor] = None, client_fuse=None, extra_segments=()):
        """One /forward_pass request (server_part.py:38-58): returns (cut_grad, loss_i). The mean
        loss for `step` lands in the device loss log. `extra_segments`: further (param, grad, slabs)
        reduce+SGD segments at this stage's lr run in the same optimizer launch (the fused trainer's
        client update, whose slabs the dgrad wrote)."""
        B = labels.shape[0]
        cut_grad, loss_i, s2, s3 = self.forward_backward(act, labels, 1.0 / B, cut_grad=cut_grad,
                                                         act_amax=act_amax, act16=act16, client_fuse=client_fuse)
        if self.fuse_optim:
            # optimizer.step() + log_metric in ONE launch (bit-identical to the three below); measured
            # -10 us per step at B = 4096 (tools/ab_step.py). The client's SGD stays a separate launch
            # after its wgrad: moving that wgrad ahead of the server's update measured +25-35 us.
            k = ops.CONV2_SLAB
            with TIMER("sgd_server"):
                ops.sgd_multi_from_slabs([(self.params[:k], self.grads[:k], s2), (self.params[k:], self.grads[k:], s3),
                                          *extra_segments],
                                         self.lr, loss=(loss_i, 1.0 / B, self.loss_log.ring, self.loss_log.counter))
            if step is not None:
                self.loss_log.note_step(step)
        else:
            self.apply_grad_slabs(s2, s3)
            self.log_loss(loss_i, step=step)
            for prm, grd, sl in extra_segments:
                ops.sgd_from_slabs(prm, grd, sl, self.lr)
        return cut_grad, loss_i

    def check_labels(self):
        """Raise if any label seen so far was outside [0, 10) (torch raises IndexError there)."""
        if int(self.err_flag.item()) != 0:
            raise IndexError("splitcnn: a label was out of range [0, 10)")


def _n_caller_graphs(tr, B: int) -> int:
    return sum(1 for k in tr._graphs if isinstance(k, tuple) and k[0] == B)


def _is_static(tr, x, y) -> bool:
    st = tr._graphs.get(x.shape[0])
    return st is not None and x.data_ptr() == st["x"].data_ptr() and y.data_ptr() == st["y"].data_ptr()


def register_graph_inputs(tr, x, y) -> bool:
    """Capture trainer `tr`'s step graph on the caller's own (x, y) buffers now — a loader declaring its
    ring of batch buffers — so step() on them replays with no copy and no capture later. Counts toward
    `tr.graph_inputs`; False (nothing captured) when the buffers do not qualify or that budget is spent.
    Shared by SplitTrainer and wide.WideTrainer (`_graphs`, `_graph_for`, `_own_buffers_ok`)."""
    if not tr.graph or not tr._own_buffers_ok(x, y):
        return False
    B = x.shape[0]
    if _is_static(tr, x, y) or (B, x.data_ptr(), y.data_ptr()) in tr._graphs:
        return True
    if _n_caller_graphs(tr, B) >= tr.graph_inputs:
        return False
    tr._graph_for(B, x, y)
    return True


def select_graph(tr, x, y):
    """The graph step() replays directly on (x, y), or None (then it copies into the static inputs).
    The static inputs handed back (static_inputs(B)) replay their own graph; a caller buffer pair gets a
    graph of its own the SECOND time it is seen (a loader's ring), so a one-off fresh tensor goes
    through the static-input copy and is not kept alive by a graph."""
    if not tr._own_buffers_ok(x, y):
        return None
    if _is_static(tr, x, y):
        return tr._graphs[x.shape[0]]
    B = x.shape[0]
    key = (B, x.data_ptr(), y.data_ptr())
    g = tr._graphs.get(key)
    if g is None:
        n = tr._seen.get(key, 0) + 1
        tr._seen[key] = n
        if n >= 2 and _n_caller_graphs(tr, B) < tr.graph_inputs:
            g = tr._graph_for(B, x, y)
            del tr._seen[key]
    return g


class SplitTrainer:
    """Both stages fused on ONE GPU (BASELINE config 2): the cut tensor is handed over in place.

    `step(x, y)` = client fwd -> server fwd/loss/bwd/SGD -> client bwd/SGD, exactly one reference
    step. With `graph=True` the step is captured once per batch size into a HIP graph (static input
    buffers; `step` copies into them unless the caller hands in those very buffers)."""

    def __init__(self, client: Optional[ModelPartA] = None, server: Optional[ModelPartB] = None,
                 lr: float = LR, device="cuda", graph: bool = True, loss_log: Optional[LossLog] = None,
                 conv: str = CONV_DEFAULT, act16: bool = True, fuse_client_backward: bool = True,
                 graph_inputs: int = 4):
        self.device = torch.device(device)
        self.client = ClientStage(client, lr, self.device)
        self.server = ServerStage(server, lr, self.device, loss_log, conv=conv)
        # the cut's per-sample max rides along with the cut (fused into conv1) for the x3 kernels; with the
        # x3 forward AND wgrad the client writes the server's split input images directly (no f32 cut)
        self.client.emit_amax = "x3" in (self.server.impl_fwd, self.server.impl_wgrad)
        self.client.emit_act16 = (self.server.impl_fwd, self.server.impl_wgrad) == ("x3", "x3") and act16
        # the x3 dgrad also runs the client's ReLU backward + conv1 wgrad (no cut gradient in HBM)
        # (the client's ReLU mask comes from the bit map conv1_fwd_x3 writes next to the images)
        self.fuse_client_backward = self.server.impl_dgrad == "x3" and self.client.emit_act16 and fuse_client_backward
        self.graph = graph
        self._graphs = {}
        # graphs captured on a caller's own input buffers (a loader's ring of batch buffers): replaying
        # one reads its inputs where they already are, with no copy into the static inputs; at most
        # `graph_inputs` such buffer pairs per batch size, any others go through the static inputs
        self.graph_inputs = graph_inputs
        self._seen = {}   # (B, x ptr, y ptr) -> times a caller buffer pair went through the static inputs
        self.global_step = 0

    @property
    def loss_log(self) -> LossLog:
        return self.server.loss_log

    def _eager(self, x, y):
        act = self.client.forward(x)
        a16 = self.client._act16 if self.client.emit_act16 else None
        if self.fuse_client_backward:
            c = self.client
            slabs = c._buf.get("c1w_slabs", (ops.conv2_dgrad_c1w_nslab(x.shape[0]), ops.CLIENT_NPARAM),
                               torch.float32, self.device)
            # the client's update joins the server's optimizer launch (its slabs are complete once the
            # dgrad has run; bit-identical to step_from_slabs) when both stages step at one lr
            one = c.lr == self.server.lr
            self.server.step_request(act, y, act_amax=c._act_amax, act16=a16,
                                     client_fuse=(x, c._relu_bits, slabs),
                                     extra_segments=[(c.params, c.grads, slabs)] if one else ())
            if not one:
                c.step_from_slabs(slabs)
            return
        cut_grad, _ = self.server.step_request(act, y, act_amax=self.client._act_amax, act16=a16)
        self.client.backward_step(cut_grad)

    def static_inputs(self, B: int):
        g = self._graph_for(B)
        return g["x"], g["y"]

    def _graph_for(self, B: int, x: Optional[torch.Tensor] = None, y: Optional[torch.Tensor] = None):
        """The step's graph for batch size B on the static inputs, or (x, y given) on those buffers."""
        key = B if x is None else (B, x.data_ptr(), y.data_ptr())
        g = self._graphs.get(key)
        if g is not None:
            return g
        if x is None:
            x = torch.zeros((B, 1, 28, 28), dtype=torch.float32, device=self.device)
            y = torch.zeros((B,), dtype=torch.int64, device=self.device)
        # warm up on a side stream (allocations happen here, not during capture), then restore the
        # parameters and the loss log so the warm-up leaves no trace.
        saved_c, saved_s = self.client.params.clone(), self.server.params.clone()
        saved_ctr = self.server.loss_log.counter.clone()
        s = torch.cuda.Stream(self.device)
        s.wait_stream(torch.cuda.current_stream(self.device))
        with torch.cuda.stream(s):
            self._eager(x, y)
        torch.cuda.current_stream(self.device).wait_stream(s)
        graph = torch.cuda.CUDAGraph()
        # thread-local capture: another thread's CUDA calls (a process group's watchdog) cannot void it
        with torch.cuda.graph(graph, capture_error_mode="thread_local"):
            self._eager(x, y)
        self.client.params.copy_(saved_c)
        self.server.params.copy_(saved_s)
        self.server.loss_log.counter.copy_(saved_ctr)
        g = {"graph": graph, "x": x, "y": y}
        self._graphs[key] = g
        return g

    def _own_buffers_ok(self, x, y) -> bool:
        return (x.device == self.device and y.device == self.device and x.dtype == torch.float32
                and y.dtype == torch.int64 and x.is_contiguous() and y.is_contiguous()
                and tuple(x.shape[1:]) == (1, 28, 28) and y.shape == (x.shape[0],))

    def register_inputs(self, x: torch.Tensor, y: torch.Tensor) -> bool:
        """Capture a graph on the caller's own (x, y) buffers now (see `register_graph_inputs`)."""
        return register_graph_inputs(self, x, y)

    def step(self, x: torch.Tensor, y: torch.Tensor):
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
