"""Multi-GPU split-learning topologies over torch.distributed (backend "nccl" = RCCL over xGMI on
MI355X; "gloo" for the CPU protocol tests). One process per GPU.

The reference has exactly one exchange per step: the client POSTs the cut activations and labels,
the server answers with the cut gradient (src/client_part.py:117-131, src/server_part.py:38-58),
and its k8s Deployment runs one client (k8s/split-learning.yaml:49). Its HTTP transport becomes
device-resident exchange here:

  Replicated (default for N >= 2; "SplitFed-V1" on one node): every rank hosts one client and one
      server-side replica; the cut tensor is handed over in place on the GPU. After the backward,
      ONE all-reduce of the [client grads | server grads | loss] bucket (444 KB) averages both
      sides, so every rank applies the reference's SGD step for the concatenated global batch
      N*B (mean loss over N*B). Weak scaling: no data-path collective besides that bucket.
  Pipeline (N = 2): rank 0 = client stage, rank 1 = server stage. The batch is cut into m
      micro-batches; activations/labels go 0 -> 1 and cut gradients 1 -> 0 by send/recv while the
      other side computes; both sides accumulate gradients and step once per batch (= the
      reference step at batch B).
  Hub (N >= 3; SplitFed with N-1 client GPUs feeding ONE server GPU): each client sends its slice,
      the server runs every slice as it arrives (accumulating its gradient), returns each client
      its cut-gradient slice, and the clients all-reduce their 320-float gradient before stepping
      (= the reference step at batch (N-1)*B on the concatenated inputs).
  FedAvg (the reference's LEARNING_MODE=federated): full-model local training per
      rank, then one all-reduce of the sample-weighted parameters per round.

The first three are exactly the reference's step at their global batch (the mean loss scale 1/global is
applied inside the cross-entropy kernel), so they share the single-process oracle. The stage
objects only need: client.forward / backward / step / grads / bind_grads and server.compute / step /
grads / bind_grads / log_loss (engine.ClientStage / engine.ServerStage on GPU; oracle-backed
stages in the CPU tests).
"""
from __future__ import annotations

import time
from typing import Optional

import torch
import torch.distributed as dist

CLIENT_N = 320
SERVER_N = 110666


class _Staged:
    """A gloo point-to-point op on a device tensor, staged through host memory. Gloo moves only host
    buffers (the CPU protocol tests and the 1-GPU multi-rank rehearsal use it); RCCL ("nccl") moves
    device memory directly over xGMI, so with it these helpers are plain isend/irecv."""

    def __init__(self, work, host=None, dev=None):
        self.work, self.host, self.dev = work, host, dev

    def wait(self):
        self.work.wait()
        if self.dev is not None:
            self.dev.copy_(self.host)   # ordered on the current stream, before any consumer
        return True


def _host_staged(t, group) -> bool:
    return t.device.type == "cuda" and dist.get_backend(group) == "gloo"


def isend(t, dst, group=None):
    if _host_staged(t, group):
        h = t.detach().to("cpu")        # waits for the producer on the current stream
        return _Staged(dist.isend(h, dst, group=group), host=h)
    return dist.isend(t, dst, group=group)


def irecv(t, src, group=None):
    if _host_staged(t, group):
        h = torch.empty(t.shape, dtype=t.dtype)
        return _Staged(dist.irecv(h, src, group=group), host=h, dev=t)
    return dist.irecv(t, src, group=group)


def send(t, dst, group=None):
    isend(t, dst, group).wait()


def recv(t, src, group=None):
    irecv(t, src, group).wait()


def _loss_sum(values, scale, out):
    """scale*sum(values) -> out (the stage's own kernel when it has one)."""
    if values.device.type == "cuda":
        from . import ops
        ops.loss_sum(values, scale, out)
    else:
        out.copy_((values.double().sum() * scale).to(out.dtype).reshape(1))


def _pair_amax(client, server):
    """Same-device client/server pair: let the client's conv1 emit the cut's per-sample max when the
    server runs the x3 conv2 kernels (saves re-reading the cut)."""
    if "x3" in (getattr(server, "impl_fwd", None), getattr(server, "impl_wgrad", None)) and hasattr(client, "emit_amax"):
        client.emit_amax = True


def _compute(server, client, act, y, scale):
    amax = getattr(client, "_act_amax", None)
    if amax is not None:
        return server.compute(act, y, scale, act_amax=amax)
    return server.compute(act, y, scale)


def _fused_pair(client, server) -> bool:
    """Same-device engine stages with every conv2 kernel on x3: the replica can run the single-GPU
    fused step's kernels (client conv1 writes the server's split images, the client backward runs in
    the server's dgrad epilogue) — engine.SplitTrainer's launch sequence minus the optimizer."""
    return (getattr(server, "conv", None) == "x3" and hasattr(client, "emit_act16")
            and getattr(client, "device", None) is not None and client.device.type == "cuda"
            and client.device == server.device)


class Replicated:
    """Data-parallel replicas (SplitFed-V1 on one node). `fused` (default: whenever `_fused_pair`)
    runs the replica's compute as the single-GPU fused step (captured in one HIP graph per batch size
    when `graph`), the gradients land in the bucket by one reduce launch, ONE all-reduce of the
    bucket, then ONE launch steps both stages and logs the loss. At world 1 that is bit-identical to
    engine.SplitTrainer's step (same kernels, same slab order; the optimizer reads the reduced
    gradient instead of the slabs)."""

    def __init__(self, client, server, group=None, device=None, fused: Optional[bool] = None,
                 graph: bool = False):
        self.client, self.server = client, server
        self.fused = _fused_pair(client, server) if fused is None else fused
        if self.fused:
            if not _fused_pair(client, server):
                raise ValueError("Replicated(fused=True) needs same-device engine stages on the x3 conv preset")
            client.emit_act16 = True
        else:
            _pair_amax(client, server)
        self.group = group
        self.world = dist.get_world_size(group)
        dev = device if device is not None else client.grads.device
        self.bucket = torch.zeros(CLIENT_N + SERVER_N + 1, dtype=client.grads.dtype, device=dev)
        client.bind_grads(self.bucket[:CLIENT_N])
        server.bind_grads(self.bucket[CLIENT_N:CLIENT_N + SERVER_N])
        self.loss_slot = self.bucket[-1:]
        self.global_step = 0
        self.overlap = True   # split the all-reduce so the server's part overlaps the client backward
        self.graph = graph and self.fused
        self._graphs = {}

    # ---------------------------------------------------------------- fused replica (x3 stages)
    def _compute_fused(self, x, y):
        """Client forward -> server forward/loss/backward with the client backward in the dgrad
        epilogue -> every gradient slab reduced into the bucket + the scaled loss into its slot."""
        from . import ops
        c, s = self.client, self.server
        B = x.shape[0]
        scale = 1.0 / (self.world * B)
        c.forward(x)
        cslabs = c._buf.get("c1w_slabs", (ops.conv2_dgrad_c1w_nslab(B), ops.CLIENT_NPARAM), torch.float32, c.device)
        _, loss_i, s2, s3 = s.forward_backward(None, y, scale, act_amax=c._act_amax, act16=c._act16,
                                               client_fuse=(x, c.W1.detach(), c.b1.detach(), cslabs))
        k = ops.CONV2_SLAB
        ops.sgd_multi_from_slabs([(None, c.grads, cslabs), (None, s.grads[:k], s2), (None, s.grads[k:], s3)], 0.0)
        ops.loss_sum(loss_i, scale, self.loss_slot)

    def _graph_for(self, B):
        g = self._graphs.get(B)
        if g is not None:
            return g
        dev = self.bucket.device
        x = torch.zeros((B, 1, 28, 28), dtype=torch.float32, device=dev)
        y = torch.zeros((B,), dtype=torch.int64, device=dev)
        # warm up on a side stream (allocations happen here, not during capture); the compute segment
        # writes only scratch and the bucket, so the warm-up leaves no trace in the parameters
        st = torch.cuda.Stream(dev)
        st.wait_stream(torch.cuda.current_stream(dev))
        with torch.cuda.stream(st):
            self._compute_fused(x, y)
        torch.cuda.current_stream(dev).wait_stream(st)
        graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(graph):
            self._compute_fused(x, y)
        g = {"graph": graph, "x": x, "y": y}
        self._graphs[B] = g
        return g

    def _step_fused(self, x, y):
        from . import ops
        if self.graph:
            g = self._graph_for(x.shape[0])
            if x.data_ptr() != g["x"].data_ptr():
                g["x"].copy_(x, non_blocking=True)
            if y.data_ptr() != g["y"].data_ptr():
                g["y"].copy_(y, non_blocking=True)
            g["graph"].replay()
        else:
            self._compute_fused(x, y)
        dist.all_reduce(self.bucket, group=self.group)
        c, s, C = self.client, self.server, CLIENT_N
        ring, ctr = s.loss_log.ring, s.loss_log.counter
        segs = [(c.params, None, self.bucket[:C].view(1, C)), (s.params, None, self.bucket[C:C + SERVER_N].view(1, SERVER_N))]
        if c.lr == s.lr:
            ops.sgd_multi_from_slabs(segs, s.lr, loss=(self.loss_slot, 1.0, ring, ctr))
        else:
            ops.sgd_multi_from_slabs(segs[:1], c.lr)
            ops.sgd_multi_from_slabs(segs[1:], s.lr, loss=(self.loss_slot, 1.0, ring, ctr))
        s.loss_log.note_step(self.global_step)
        self.global_step += 1

    def step(self, x, y):
        if self.fused:
            return self._step_fused(x, y)
        B = x.shape[0]
        scale = 1.0 / (self.world * B)
        act = self.client.forward(x)
        cut, loss_i = _compute(self.server, self.client, act, y, scale)
        _loss_sum(loss_i, scale, self.loss_slot)
        if self.overlap:
            # the server gradients (+ loss) are final here: their all-reduce (442 KB) runs on the
            # collective stream while the client backward runs; the client's 1.28 KB follows it
            work = dist.all_reduce(self.bucket[CLIENT_N:], group=self.group, async_op=True)
            self.client.backward(cut)
            dist.all_reduce(self.bucket[:CLIENT_N], group=self.group)
            work.wait()
        else:
            self.client.backward(cut)
            dist.all_reduce(self.bucket, group=self.group)
        self.client.step()
        self.server.step()
        self.server.log_loss(self.loss_slot, scale=1.0, step=self.global_step)
        self.global_step += 1


class Pipeline:
    """2-rank client/server pipeline with m micro-batches. `role` is "client" or "server".

    compress (default on for CUDA tensors): the cut and its gradient travel through the lossless
    sparse codec (codec.py): per step one int32 header with the m micro-batches' nonzero counts, then
    per micro-batch the bit mask + the nonzero activations out and the gradient at those positions back.
    Results are bit-identical to the dense exchange; `exchange_bytes` counts what actually moved and
    `dense_bytes` what the dense exchange would have moved."""

    def __init__(self, stage, role: str, peer: int, micro: int = 4, group=None, compress: bool = True):
        assert role in ("client", "server")
        self.stage, self.role, self.peer, self.micro, self.group = stage, role, peer, micro, group
        self.compress = compress
        self.global_step = 0
        self._bufs = {}
        self.exchange_bytes = 0
        self.dense_bytes = 0
        self._codec = None

    def _use_codec(self, device):
        if not (self.compress and torch.device(device).type == "cuda"):
            return None
        if self._codec is None:
            from .codec import CutCodec
            self._codec = CutCodec()
        return self._codec

    def _buf(self, name, shape, dtype, device):
        t = self._bufs.get(name)
        if t is None or tuple(t.shape) != tuple(shape) or t.device != device:
            t = torch.empty(shape, dtype=dtype, device=device)
            self._bufs[name] = t
        return t

    def client_step(self, x, y):
        B = x.shape[0]
        m = self.micro
        assert B % m == 0, "batch must be divisible by the micro-batch count"
        mb = B // m
        c = self.stage
        dev = x.device
        acts = self._buf("acts", (B, 32, 26, 26), torch.float32, dev)
        cuts = self._buf("cuts", (B, 32, 26, 26), torch.float32, dev)
        codec = self._use_codec(dev)
        if codec is not None:
            return self._client_step_codec(codec, x, y, acts, cuts, m, mb)
        sends, recvs = [], []
        for k in range(m):
            sl = slice(k * mb, (k + 1) * mb)
            c.forward(x[sl], out=acts[sl])
            sends.append(isend(acts[sl], self.peer, group=self.group))
            sends.append(isend(y[sl], self.peer, group=self.group))
        for k in range(m):
            sl = slice(k * mb, (k + 1) * mb)
            recvs.append(irecv(cuts[sl], self.peer, group=self.group))
        for k in range(m):
            sl = slice(k * mb, (k + 1) * mb)
            recvs[k].wait()
            c.backward(cuts[sl], x=x[sl], act=acts[sl], accumulate=k > 0)
        for w in sends:
            w.wait()
        c.step()
        self.exchange_bytes = self.dense_bytes = 2 * acts.numel() * 4 + y.numel() * 8
        self.global_step += 1

    def _client_step_codec(self, codec, x, y, acts, cuts, m, mb):
        c = self.stage
        n = mb * 32 * 26 * 26
        bufs = []
        for k in range(m):
            sl = slice(k * mb, (k + 1) * mb)
            c.forward(x[sl], out=acts[sl])
            b = codec.buffers(("c", k), n, x.device)
            codec.encode(acts[sl], b)
            bufs.append(b)
        head = self._buf("head", (m,), torch.int32, x.device)
        for k in range(m):
            head[k:k + 1].copy_(bufs[k][3])
        totals = head.tolist()            # the one host sync of the step: sizes of the sparse payloads
        sends = [isend(head, self.peer, group=self.group)]
        for k in range(m):
            sl = slice(k * mb, (k + 1) * mb)
            sends.append(isend(bufs[k][0], self.peer, group=self.group))
            sends.append(isend(y[sl], self.peer, group=self.group))
            if totals[k]:
                sends.append(isend(bufs[k][4][:totals[k]], self.peer, group=self.group))
        gv = [self._buf(("gvals", k), (n,), torch.float32, x.device) for k in range(m)]
        recvs = [irecv(gv[k][:totals[k]], self.peer, group=self.group) if totals[k] else None for k in range(m)]
        for k in range(m):
            sl = slice(k * mb, (k + 1) * mb)
            if recvs[k] is not None:
                recvs[k].wait()
            codec.unpack(cuts[sl], bufs[k], vals=gv[k])
            c.backward(cuts[sl], x=x[sl], act=acts[sl], accumulate=k > 0)
        for w in sends:
            w.wait()
        c.step()
        self.exchange_bytes = m * 4 + sum(bufs[k][0].numel() * 4 + 2 * totals[k] * 4 for k in range(m)) + y.numel() * 8
        self.dense_bytes = 2 * acts.numel() * 4 + y.numel() * 8
        self.global_step += 1

    def server_step(self, B: int, device):
        m = self.micro
        mb = B // m
        s = self.stage
        acts = self._buf("acts", (B, 32, 26, 26), torch.float32, device)
        labels = self._buf("labels", (B,), torch.int64, device)
        cuts = self._buf("cuts", (B, 32, 26, 26), torch.float32, device)
        parts = self._buf("loss_parts", (m,), torch.float32, device)
        codec = self._use_codec(device)
        if codec is not None:
            return self._server_step_codec(codec, B, device, acts, labels, cuts, parts, m, mb)
        recvs = []
        for k in range(m):
            sl = slice(k * mb, (k + 1) * mb)
            recvs.append((irecv(acts[sl], self.peer, group=self.group),
                          irecv(labels[sl], self.peer, group=self.group)))
        sends = []
        for k in range(m):
            sl = slice(k * mb, (k + 1) * mb)
            recvs[k][0].wait()
            recvs[k][1].wait()
            _, loss_i = s.compute(acts[sl], labels[sl], 1.0 / B, accumulate=k > 0, cut_grad=cuts[sl])
            _loss_sum(loss_i, 1.0 / B, parts[k:k + 1])
            sends.append(isend(cuts[sl], self.peer, group=self.group))
        s.step()
        s.log_loss(parts, scale=1.0, step=self.global_step)
        for w in sends:
            w.wait()
        self.exchange_bytes = self.dense_bytes = 2 * acts.numel() * 4 + labels.numel() * 8
        self.global_step += 1

    def _server_step_codec(self, codec, B, device, acts, labels, cuts, parts, m, mb):
        s = self.stage
        n = mb * 32 * 26 * 26
        head = self._buf("head", (m,), torch.int32, device)
        irecv(head, self.peer, group=self.group).wait()
        totals = head.tolist()            # the one host sync of the step: sizes of the sparse payloads
        bufs, recvs = [], []
        for k in range(m):
            sl = slice(k * mb, (k + 1) * mb)
            b = codec.buffers(("s", k), n, device)
            bufs.append(b)
            rk = [irecv(b[0], self.peer, group=self.group), irecv(labels[sl], self.peer, group=self.group)]
            if totals[k]:
                rk.append(irecv(b[4][:totals[k]], self.peer, group=self.group))
            recvs.append(rk)
        sends = []
        for k in range(m):
            sl = slice(k * mb, (k + 1) * mb)
            for r in recvs[k]:
                r.wait()
            codec.offsets(n, bufs[k])
            codec.unpack(acts[sl], bufs[k])
            _, loss_i = s.compute(acts[sl], labels[sl], 1.0 / B, accumulate=k > 0, cut_grad=cuts[sl])
            _loss_sum(loss_i, 1.0 / B, parts[k:k + 1])
            gv = self._buf(("gvals", k), (n,), torch.float32, device)
            codec.pack(cuts[sl], bufs[k], vals=gv)
            if totals[k]:
                sends.append(isend(gv[:totals[k]], self.peer, group=self.group))
        s.step()
        s.log_loss(parts, scale=1.0, step=self.global_step)
        for w in sends:
            w.wait()
        self.exchange_bytes = m * 4 + sum(bufs[k][0].numel() * 4 + 2 * totals[k] * 4 for k in range(m)) + labels.numel() * 8
        self.dense_bytes = 2 * acts.numel() * 4 + labels.numel() * 8
        self.global_step += 1


class Hub:
    """N-1 client ranks (0..N-2) feed one server rank (N-1). `compress` as for Pipeline: per client
    and step one int32 header of the micro-batch nonzero counts, then mask + values each way."""

    def __init__(self, stage, rank: int, world: int, client_group=None, micro: int = 1, compress: bool = True):
        self.stage, self.rank, self.world = stage, rank, world
        self.server_rank = world - 1
        self.nclients = world - 1
        self.client_group = client_group
        self.micro = micro
        self.compress = compress
        self.global_step = 0
        self._bufs = {}
        self.exchange_bytes = 0
        self.dense_bytes = 0
        self._codec = None

    _use_codec = Pipeline._use_codec

    @property
    def is_server(self):
        return self.rank == self.server_rank

    def _buf(self, name, shape, dtype, device):
        t = self._bufs.get(name)
        if t is None or tuple(t.shape) != tuple(shape) or t.device != device:
            t = torch.empty(shape, dtype=dtype, device=device)
            self._bufs[name] = t
        return t

    def client_step(self, x, y):
        """Client k: forward each of `micro` micro-batches and send it (+ labels) while computing the
        next; back-propagate each returned cut-gradient slice as it lands; all-reduce; SGD."""
        c = self.stage
        B, m = x.shape[0], self.micro
        assert B % m == 0, "batch must be divisible by the micro-batch count"
        b = B // m
        act = self._buf("act", (B, 32, 26, 26), torch.float32, x.device)
        cut = self._buf("cut", (B, 32, 26, 26), torch.float32, x.device)
        codec = self._use_codec(x.device)
        if codec is not None:
            return self._client_step_codec(codec, x, y, act, cut, m, b)
        sends, recvs = [], []
        for k in range(m):
            sl = slice(k * b, (k + 1) * b)
            c.forward(x[sl], out=act[sl])
            sends.append(isend(act[sl], self.server_rank))
            sends.append(isend(y[sl], self.server_rank))
        for k in range(m):
            recvs.append(irecv(cut[k * b:(k + 1) * b], self.server_rank))
        for k in range(m):
            sl = slice(k * b, (k + 1) * b)
            recvs[k].wait()
            c.backward(cut[sl], x=x[sl], act=act[sl], accumulate=k > 0)
        for w in sends:
            w.wait()
        if self.nclients > 1:
            dist.all_reduce(c.grads, group=self.client_group)
        c.step()
        self.exchange_bytes = self.dense_bytes = 2 * act.numel() * 4 + y.numel() * 8
        self.global_step += 1

    def _client_step_codec(self, codec, x, y, act, cut, m, b):
        c = self.stage
        n = b * 32 * 26 * 26
        bufs = []
        for k in range(m):
            sl = slice(k * b, (k + 1) * b)
            c.forward(x[sl], out=act[sl])
            bk = codec.buffers(("c", k), n, x.device)
            codec.encode(act[sl], bk)
            bufs.append(bk)
        head = self._buf("head", (m,), torch.int32, x.device)
        for k in range(m):
            head[k:k + 1].copy_(bufs[k][3])
        totals = head.tolist()
        sends = [isend(head, self.server_rank)]
        for k in range(m):
            sl = slice(k * b, (k + 1) * b)
            sends.append(isend(bufs[k][0], self.server_rank))
            sends.append(isend(y[sl], self.server_rank))
            if totals[k]:
                sends.append(isend(bufs[k][4][:totals[k]], self.server_rank))
        gv = [self._buf(("gvals", k), (n,), torch.float32, x.device) for k in range(m)]
        recvs = [irecv(gv[k][:totals[k]], self.server_rank) if totals[k] else None for k in range(m)]
        for k in range(m):
            sl = slice(k * b, (k + 1) * b)
            if recvs[k] is not None:
                recvs[k].wait()
            codec.unpack(cut[sl], bufs[k], vals=gv[k])
            c.backward(cut[sl], x=x[sl], act=act[sl], accumulate=k > 0)
        for w in sends:
            w.wait()
        if self.nclients > 1:
            dist.all_reduce(c.grads, group=self.client_group)
        c.step()
        self.exchange_bytes = m * 4 + sum(bufs[k][0].numel() * 4 + 2 * totals[k] * 4 for k in range(m)) + y.numel() * 8
        self.dense_bytes = 2 * act.numel() * 4 + y.numel() * 8
        self.global_step += 1

    def server_step(self, B: int, device):
        """B = per-client batch; the server step covers (N-1)*B samples, consumed part by part in
        (micro-batch, client) order as they arrive, gradient accumulated, ONE SGD step."""
        s = self.stage
        m, nc = self.micro, self.nclients
        b, G = B // m, nc * B
        acts = self._buf("acts", (G, 32, 26, 26), torch.float32, device)
        labels = self._buf("labels", (G,), torch.int64, device)
        cuts = self._buf("cuts", (G, 32, 26, 26), torch.float32, device)
        parts = self._buf("loss_parts", (m * nc,), torch.float32, device)
        codec = self._use_codec(device)
        if codec is not None:
            return self._server_step_codec(codec, B, device, acts, labels, cuts, parts)
        reqs = {}
        for c in range(nc):
            for k in range(m):
                sl = slice(c * B + k * b, c * B + (k + 1) * b)
                reqs[c, k] = (irecv(acts[sl], c), irecv(labels[sl], c))
        sends, part = [], 0
        for k in range(m):
            for c in range(nc):
                sl = slice(c * B + k * b, c * B + (k + 1) * b)
                for r in reqs[c, k]:
                    r.wait()
                _, loss_i = s.compute(acts[sl], labels[sl], 1.0 / G, accumulate=part > 0, cut_grad=cuts[sl])
                _loss_sum(loss_i, 1.0 / G, parts[part:part + 1])
                sends.append(isend(cuts[sl], c))
                part += 1
        s.step()
        s.log_loss(parts, scale=1.0, step=self.global_step)
        for w in sends:
            w.wait()
        self.exchange_bytes = self.dense_bytes = 2 * acts.numel() * 4 + labels.numel() * 8
        self.global_step += 1

    def _server_step_codec(self, codec, B, device, acts, labels, cuts, parts):
        s = self.stage
        m, nc = self.micro, self.nclients
        b, G = B // m, nc * B
        n = b * 32 * 26 * 26
        heads = [self._buf(("head", c), (m,), torch.int32, device) for c in range(nc)]
        hreq = [irecv(heads[c], c) for c in range(nc)]
        totals = {}
        for c in range(nc):
            hreq[c].wait()
            for k, t in enumerate(heads[c].tolist()):
                totals[c, k] = t
        reqs, bufs = {}, {}
        for c in range(nc):
            for k in range(m):
                sl = slice(c * B + k * b, c * B + (k + 1) * b)
                bk = codec.buffers(("s", c, k), n, device)
                bufs[c, k] = bk
                rk = [irecv(bk[0], c), irecv(labels[sl], c)]
                if totals[c, k]:
                    rk.append(irecv(bk[4][:totals[c, k]], c))
                reqs[c, k] = rk
        sends, part = [], 0
        for k in range(m):
            for c in range(nc):
                sl = slice(c * B + k * b, c * B + (k + 1) * b)
                for r in reqs[c, k]:
                    r.wait()
                codec.offsets(n, bufs[c, k])
                codec.unpack(acts[sl], bufs[c, k])
                _, loss_i = s.compute(acts[sl], labels[sl], 1.0 / G, accumulate=part > 0, cut_grad=cuts[sl])
                _loss_sum(loss_i, 1.0 / G, parts[part:part + 1])
                gv = self._buf(("gvals", c, k), (n,), torch.float32, device)
                codec.pack(cuts[sl], bufs[c, k], vals=gv)
                if totals[c, k]:
                    sends.append(isend(gv[:totals[c, k]], c))
                part += 1
        s.step()
        s.log_loss(parts, scale=1.0, step=self.global_step)
        for w in sends:
            w.wait()
        self.exchange_bytes = (nc * m * 4 + sum(bufs[key][0].numel() * 4 + 2 * t * 4 for key, t in totals.items())
                               + labels.numel() * 8)
        self.dense_bytes = 2 * acts.numel() * 4 + labels.numel() * 8
        self.global_step += 1


class FedAvg:
    """Federated learning round: each rank trains the FULL model locally on its own
    batches (src/client_part.py:143-170: forward, CE, backward, SGD per batch — on one GPU that is the
    split step with the cut in place), then `aggregate()` replaces the reference's state_dict POST +
    identity `load_state_dict` (client_part.py:172-195, server_part.py:81-93) by ONE all-reduce of
    [n_k * params | n_k | n_k * mean local loss] and a device-side divide: sample-weighted FedAvg,
    no host sync. With one rank it is exactly the reference's single-client round.

    The aggregated client loss is logged for `step` like server_part.py:84 (mlflow.log_metric)."""

    def __init__(self, client, server, group=None, device=None):
        self.client, self.server = client, server
        _pair_amax(client, server)
        self.group = group
        dev = device if device is not None else client.params.device
        self.n = CLIENT_N + SERVER_N
        self.bucket = torch.zeros(self.n + 2, dtype=client.params.dtype, device=dev)
        self.loss_acc = torch.zeros(1, dtype=client.params.dtype, device=dev)
        self._loss_tmp = torch.zeros(1, dtype=client.params.dtype, device=dev)
        self.samples = 0   # n_k of the current round (host count: no sync)
        self.batches = 0

    def local_step(self, x, y):
        B = x.shape[0]
        act = self.client.forward(x)
        cut, loss_i = _compute(self.server, self.client, act, y, 1.0 / B)
        self.client.backward(cut)
        self.client.step()
        self.server.step()
        _loss_sum(loss_i, 1.0 / B, self._loss_tmp)
        self.loss_acc += self._loss_tmp     # epoch_loss += loss.item() without the per-step sync
        self.samples += B
        self.batches += 1

    def aggregate(self, step: Optional[int] = None, weight: Optional[float] = None):
        """All-reduce the sample-weighted parameters; every rank leaves with the FedAvg model."""
        w = float(self.samples if weight is None else weight)
        C = CLIENT_N
        b = self.bucket
        torch.mul(self.client.params, w, out=b[:C])
        torch.mul(self.server.params, w, out=b[C:self.n])
        b[self.n].fill_(w)
        torch.mul(self.loss_acc, w / max(self.batches, 1), out=b[self.n + 1:])
        dist.all_reduce(b, group=self.group)
        wsum = b[self.n:self.n + 1]
        torch.div(b[:C], wsum, out=self.client.params)
        torch.div(b[C:self.n], wsum, out=self.server.params)
        torch.div(b[self.n + 1:], wsum, out=self._loss_tmp)
        self.server.log_loss(self._loss_tmp, scale=1.0, step=step)
        self.loss_acc.zero_()
        self.samples = self.batches = 0


class UShaped:
    """Label-private U-shape on 2 ranks (splitcnn/ushaped.py): rank `client` holds conv1 + fc1 +
    labels, rank `server` the conv2 trunk. Four tensors cross per step — act and dpooled
    client -> server, pooled and cut_grad server -> client; labels never leave the client."""

    def __init__(self, stage, role: str, peer: int, group=None):
        assert role in ("client", "server")
        self.stage, self.role, self.peer, self.group = stage, role, peer, group
        self.global_step = 0
        self._bufs = {}
        self.exchange_bytes = 0

    def _buf(self, name, shape, dtype, device):
        t = self._bufs.get(name)
        if t is None or tuple(t.shape) != tuple(shape) or t.device != device:
            t = torch.empty(shape, dtype=dtype, device=device)
            self._bufs[name] = t
        return t

    def client_step(self, x, y):
        B, dev, c = x.shape[0], x.device, self.stage
        act = c.forward(x)
        send(act, self.peer, group=self.group)
        pooled = self._buf("pooled", (B, 64, 12, 12), act.dtype, dev)
        recv(pooled, self.peer, group=self.group)
        dpooled = c.head_step(pooled, y, step=self.global_step)
        send(dpooled, self.peer, group=self.group)
        cut = self._buf("cut", (B, 32, 26, 26), act.dtype, dev)
        recv(cut, self.peer, group=self.group)
        c.backward_step(cut)
        self.exchange_bytes = 2 * (act.numel() + pooled.numel()) * act.element_size()
        self.global_step += 1

    def server_step(self, B: int, device, dtype=torch.float32):
        s = self.stage
        act = self._buf("act", (B, 32, 26, 26), dtype, device)
        recv(act, self.peer, group=self.group)
        pooled = s.forward(act)
        send(pooled, self.peer, group=self.group)
        dpooled = self._buf("dpooled", (B, 64, 12, 12), dtype, device)
        recv(dpooled, self.peer, group=self.group)
        cut = s.backward_step(dpooled)
        send(cut, self.peer, group=self.group)
        self.exchange_bytes = 2 * (act.numel() + pooled.numel()) * act.element_size()
        self.global_step += 1


class WideHub:
    """SplitFed for the widened model (BASELINE config 5, splitcnn/wide.py): client ranks 0..N-2 run
    the conv stack (99.9 % of the step's FLOPs), the server rank N-1 the dropout/fc head. Each client
    cuts its batch into `micro` micro-batches: it sends micro-batch k's cut (bf16, 32 KB/sample) +
    labels while computing k+1, the server runs the head on every (micro-batch, client) part as it
    arrives — mean-loss scale and dropout indices of the concatenated (N-1)*B batch, fc gradient
    accumulated — and returns that part's cut gradient, which the client back-propagates while later
    parts are still in flight. Clients then all-reduce their weight gradient (370,816 f32) and take
    identical Adam steps: exactly the single-process widened step at batch (N-1)*B.
    Stages: client.forward(x, tag) / backward_grads(dcut, tag, accumulate) / step_from_grads / grads /
    cut_shape / cut_dtype; server.accumulate(cut, labels, scale, b0, k, nparts, dcut) / finish_step."""

    def __init__(self, stage, rank: int, world: int, client_group=None, micro: int = 1):
        self.stage, self.rank, self.world = stage, rank, world
        self.server_rank = world - 1
        self.nclients = world - 1
        self.client_group = client_group
        self.micro = micro
        self.global_step = 0
        self._bufs = {}
        self.exchange_bytes = 0

    def _buf(self, name, shape, dtype, device):
        t = self._bufs.get(name)
        if t is None or tuple(t.shape) != tuple(shape) or t.device != device or t.dtype != dtype:
            t = torch.empty(shape, dtype=dtype, device=device)
            self._bufs[name] = t
        return t

    def client_step(self, x, y):
        c = self.stage
        B, m = x.shape[0], self.micro
        assert B % m == 0, "batch must be divisible by the micro-batch count"
        b = B // m
        dcut = self._buf("dcut", c.cut_shape(B), c.cut_dtype, x.device)
        sends, recvs = [], []
        for k in range(m):
            sl = slice(k * b, (k + 1) * b)
            cut = c.forward(x[sl], tag=k)
            sends.append(isend(cut, self.server_rank))
            sends.append(isend(y[sl], self.server_rank))
        for k in range(m):
            recvs.append(irecv(dcut[k * b:(k + 1) * b], self.server_rank))
        for k in range(m):
            recvs[k].wait()
            c.backward_grads(dcut[k * b:(k + 1) * b], tag=k, accumulate=k > 0)
        for w in sends:
            w.wait()
        if self.nclients > 1:
            dist.all_reduce(c.grads, group=self.client_group)
        c.step_from_grads()
        self.exchange_bytes = 2 * dcut.numel() * dcut.element_size() + y.numel() * 8
        self.global_step += 1

    def server_step(self, B: int, device, cut_shape, cut_dtype):
        """B = per-client batch; cut_shape(n) / cut_dtype describe the client stage's cut tensor."""
        s = self.stage
        m, nc = self.micro, self.nclients
        b, G = B // m, nc * B
        cuts = self._buf("cuts", cut_shape(G), cut_dtype, device)
        dcuts = self._buf("dcuts", cut_shape(G), cut_dtype, device)
        labels = self._buf("labels", (G,), torch.int64, device)
        reqs = {}
        for c in range(nc):
            for k in range(m):
                sl = slice(c * B + k * b, c * B + (k + 1) * b)
                reqs[c, k] = (irecv(cuts[sl], c), irecv(labels[sl], c))
        sends, part = [], 0
        for k in range(m):
            for c in range(nc):
                sl = slice(c * B + k * b, c * B + (k + 1) * b)
                for r in reqs[c, k]:
                    r.wait()
                s.accumulate(cuts[sl], labels[sl], 1.0 / G, c * B + k * b, part, m * nc, dcut=dcuts[sl])
                sends.append(isend(dcuts[sl], c))
                part += 1
        s.finish_step(m * nc, step=self.global_step)
        for w in sends:
            w.wait()
        self.exchange_bytes = 2 * cuts.numel() * cuts.element_size() + labels.numel() * 8
        self.global_step += 1


def client_group_for(world: int):
    """The all-reduce group of the hub's client ranks (every rank must call this, in order)."""
    if world < 3:
        return None
    return dist.new_group(list(range(world - 1)))


def measure_p2p(nbytes: int, src: int, dst: int, device, iters: int = 5, group=None) -> Optional[float]:
    """One-directional send/recv bandwidth src -> dst in GB/s (rank-local timing on dst after a
    barrier-aligned start). Returns the value on dst, None elsewhere."""
    rank = dist.get_rank(group)
    n = nbytes // 4
    t = torch.empty(n, dtype=torch.float32, device=device)
    if rank == src:
        t.fill_(1.0)
    dist.barrier(group=group)
    for it in range(iters + 1):
        if it == 1:
            if device.type == "cuda":
                torch.cuda.synchronize(device)
            t0 = time.perf_counter()
        if rank == src:
            send(t, dst, group=group)
        elif rank == dst:
            recv(t, src, group=group)
    if device.type == "cuda":
        torch.cuda.synchronize(device)
    dt = time.perf_counter() - t0
    dist.barrier(group=group)
    return (iters * nbytes / dt / 1e9) if rank == dst else None
