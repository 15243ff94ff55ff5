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

import inspect
import time
import warnings
from typing import Optional

import torch
import torch.distributed as dist

CLIENT_N = 320
SERVER_N = 110666
# bytes per sample of the x3 split images (act16: 32 channels x 676 pixels x (hi, lo) f16) = the f32 cut's
# 32 x 26 x 26 x 4: the image exchange moves the same bytes (ops.conv2_act16_bytes(1), checked in the GPU tests)
IMG_BYTES = 2 * 2 * 32 * 26 * 26
CUT_ELEMS = 32 * 26 * 26


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
    the server's dgrad epilogue) — engine.SplitTrainer's launch sequence minus the optimizer. Decided
    from the server's three impl_* fields (not its preset name), read at every step."""
    impls = tuple(getattr(server, a, None) for a in ("impl_fwd", "impl_dgrad", "impl_wgrad"))
    return (impls == ("x3", "x3", "x3") and hasattr(client, "emit_act16")
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
                 graph: bool = False, overlap: Optional[bool] = None):
        self.client, self.server = client, server
        self.fused = _fused_pair(client, server) if fused is None else fused
        if self.fused and overlap:
            warnings.warn("Replicated: overlap applies to the unfused replica only (the fused replica's "
                          "client backward runs inside the server's dgrad; its bucket is all-reduced once)")
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
        # unfused replica: split the all-reduce so the server's part overlaps the client backward
        self.overlap = True if overlap is None else bool(overlap)
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
                                               client_fuse=(x, c._relu_bits, cslabs))
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
        # thread-local capture mode: ProcessGroupNCCL's watchdog thread queries the events of earlier
        # collectives while this thread captures; in the default global mode that query invalidates it
        with torch.cuda.graph(graph, capture_error_mode="thread_local"):
            self._compute_fused(x, y)
        g = {"graph": graph, "x": x, "y": y}
        self._graphs[B] = g
        return g

    def prepare(self, B: int) -> None:
        """Capture the replica's graph for batch size B now (bench.py does this after a synchronize +
        barrier and before the phase's first collective); otherwise the first step() captures it."""
        if self.fused and self.graph:
            self._graph_for(B)

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
            if not _fused_pair(self.client, self.server):
                raise RuntimeError("Replicated: the server's conv impls changed after construction; the fused "
                                   "replica needs x3 for the forward, dgrad and wgrad")
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


def exchange_groups():
    """Two process groups over every rank, one per exchange direction (collective: every rank calls
    this, in the same order).

    RCCL runs all point-to-point ops between two ranks of ONE group in issue order on one communicator
    stream, and a send larger than its staging buffer completes only once the peer's matching receive
    runs. The hub server interleaves per chunk (receive micro-batch k, send gradient k, receive k+1)
    while a client posts every micro-batch before its first gradient receive: on a single group the
    server's send of gradient k would wait for a receive queued behind the client's send of k+1, which
    waits for the server's receive of k+1, queued behind that send — a cycle. With the cut direction on
    one group and the gradient direction on the other, each stream carries one direction, issued in the
    same order by both sides (tests/test_p2p_order.py replays both sides under these semantics)."""
    ranks = list(range(dist.get_world_size()))
    return dist.new_group(ranks), dist.new_group(ranks)


class Hub:
    """N-1 client ranks (0..N-2) feed one server rank (N-1) — SplitFed, BASELINE config 4; with one
    client it is the 2-GPU client/server pipeline (config 3, `Pipeline`). Each client cuts its batch
    into `micro` micro-batches and sends micro-batch k's cut (+ labels, + its per-sample max when
    `ship_amax`, so the server's x3 kernels need not re-read the cut for their scales) while computing
    k+1.

    Server: its buffers are laid out [micro-batch k][client c][b] so that micro-batch k of EVERY client
    is one contiguous chunk of nc*b samples: the server runs one forward/loss/backward per chunk (not
    one per (client, micro-batch) part), captured once per chunk in a HIP graph (`graph`, default on
    GPUs; the exchange stays outside the graphs), accumulates its gradient across chunks, returns each
    part's cut gradient as soon as its chunk is done, and steps once: exactly the reference's step at
    the concatenated batch nc*B (src/server_part.py:47-52; the mean-loss scale 1/(nc*B) is applied in
    the cross-entropy kernel). Clients all-reduce their 320-float gradient and step.

    Transport: `groups` = (cut direction, gradient direction), one process group each
    (`exchange_groups()`, created here when not given; see there for why one group would deadlock).

    compress (default True): the cut and its gradient travel through the lossless sparse codec
    (codec.py, HIP kernels: CUDA tensors only): per micro-batch a 4-byte count, the bit mask and the
    nonzero activations out, the gradient at those positions back. The sizes RCCL's point-to-point
    calls need are learned per micro-batch (the client waits only for micro-batch k's encode before
    sending it, on a side stream, while k+1 computes; the server posts micro-batch k's receives once
    its count has landed), so no step-wide host sync holds the first send back. Results are
    bit-identical to the dense exchange. False = the dense fp32 exchange; a codec object (the
    CutCodec interface) is used as given.
    fuse_codec (default True; server, compress on, ship_amax on, an x3 engine stage): the received
    micro-batch is unpacked straight into the x3 input images (ops.cut_unpack_x3: no dense f32 cut) and
    the dgrad writes the cut gradient already packed at the mask's positions (ops.conv2_dgrad_x3_pack:
    no dense gradient, no pack pass); the server then computes exactly what the dense images exchange
    (images=True) computes, bit for bit. `compress` and `ship_amax` are constructor arguments that
    both sides must agree on — neither side infers them from its own device.
    `exchange_bytes` counts what moved on this rank's link(s), `dense_bytes` what the dense exchange
    would have moved."""

    def __init__(self, stage, rank: int, world: int, client_group=None, micro: int = 1, compress=True,
                 server_rank: Optional[int] = None, client_ranks=None, graph: bool = True, groups=None,
                 ship_amax: bool = True, images: bool = False, fuse_codec: bool = True):
        self.stage, self.rank, self.world = stage, rank, world
        self.fuse_codec = bool(fuse_codec)
        # images (dense exchange only): the client ships its x3 split images (act16, the same 86,528 B a
        # sample as the f32 cut) + per-sample max instead of the f32 act, and the server runs the image
        # forward (conv2_fwd_pool_x3i) instead of staging + splitting f32 rows in-kernel
        self.images = bool(images)
        if self.images and (compress not in (False, None) or not ship_amax):
            raise ValueError("images=True is the dense exchange with the per-sample max: compress=False, ship_amax=True")
        self.server_rank = world - 1 if server_rank is None else server_rank
        self.client_ranks = list(range(world - 1)) if client_ranks is None else list(client_ranks)
        self.nclients = len(self.client_ranks)
        self.client_group = client_group
        if groups is None:
            groups = exchange_groups() if dist.is_initialized() else (None, None)
        self.groups = tuple(groups)
        self.micro = micro
        self.compress = compress
        self.ship_amax = bool(ship_amax)
        self.graph = graph
        self.global_step = 0
        self._pool = {}
        self._bufs = {}
        self._graphs = {}
        self._side = None
        self.exchange_bytes = 0
        self.dense_bytes = 0
        self._codec = None
        # server: False after a step whose cut gradient left packed (fuse_codec): the dense `cuts` buffer
        # was not written; cuts_by_client scatters what went on the wire instead
        self.cut_dense = True
        # the server passes the shipped max on only to stages whose compute takes it (engine stages)
        self._amax_kw = "act_amax" in inspect.signature(stage.compute).parameters if hasattr(stage, "compute") else False
        if self.images and self.is_server:
            # fail here, not inside the first forward_backward while the clients block in their sends
            # (engine stages declare their conv kernels; a stage without impl_* — the CPU protocol tests'
            # oracle stage — only has to take the image bytes)
            takes = inspect.signature(stage.compute).parameters if hasattr(stage, "compute") else {}
            engine = hasattr(stage, "impl_fwd")
            impls = (getattr(stage, "impl_fwd", "x3"), getattr(stage, "impl_wgrad", "x3"))
            if "act16" not in takes or impls != ("x3", "x3") or (engine and not self._amax_kw):
                raise ValueError(f"Hub(images=True) needs a server stage on the x3 forward and wgrad whose compute "
                                 f"takes act16 and act_amax (got impl_fwd/impl_wgrad={impls}, act_amax={self._amax_kw})")

    @property
    def is_server(self):
        return self.rank == self.server_rank

    def _fused(self, codec) -> bool:
        """Server: the codec exchange runs through the fused kernels (see fuse_codec). Only for the
        CutCodec itself: the fused kernels read its mask / word-rank / values layout, so a codec object
        passed as `compress` (any other encode) always takes the unfused unpack / pack."""
        if codec is None or not (self.fuse_codec and self.ship_amax and self._amax_kw) or self.images:
            return False
        from .codec import CutCodec
        if type(codec) is not CutCodec:
            return False
        st = self.stage
        takes = inspect.signature(st.compute).parameters if hasattr(st, "compute") else {}
        impls = tuple(getattr(st, a, None) for a in ("impl_fwd", "impl_dgrad", "impl_wgrad"))
        return impls == ("x3", "x3", "x3") and "act16" in takes and "cut_pack" in takes

    def _use_codec(self, device):
        if self.compress is False or self.compress is None:
            return None
        if self._codec is None:
            if self.compress is not True:
                self._codec = self.compress          # a codec object (the CPU protocol tests)
            elif torch.device(device).type == "cuda":
                from .codec import CutCodec
                self._codec = CutCodec()
            else:
                raise ValueError("the cut codec runs as HIP kernels on CUDA tensors: pass compress=False "
                                 "(on BOTH sides) for CPU stages")
        return self._codec

    def _buf(self, name, shape, dtype, device, pin=False):
        """Scratch keyed by (name, shape, dtype, device): a buffer is never replaced, so the chunk graphs
        captured at one batch size keep valid pointers after another size has run."""
        pin = pin and torch.device(device).type == "cuda"
        key = (name, tuple(shape), dtype, "pinned" if pin else str(torch.device(device)))
        t = self._pool.get(key)
        if t is None:
            t = torch.empty(shape, dtype=dtype, pin_memory=True) if pin else torch.empty(shape, dtype=dtype, device=device)
            self._pool[key] = t
        self._bufs[name] = t   # the latest buffer of each name (introspection: tests, cuts_by_client)
        return t

    # streams / events: CUDA only; on the CPU every op is already ordered on the host
    def _side_stream(self, device):
        if torch.device(device).type != "cuda":
            return None
        if self._side is None:
            self._side = torch.cuda.Stream(device)
        return self._side

    @staticmethod
    def _record(device):
        if torch.device(device).type != "cuda":
            return None
        ev = torch.cuda.Event()
        ev.record()
        return ev

    def _p2p(self, op, t, peer, group, side=None):
        """isend / irecv on `side` (a CUDA stream: RCCL then orders the transfer after that stream's
        work only, not after everything queued on the current stream)."""
        if side is None:
            return op(t, peer, group)
        with torch.cuda.stream(side):
            return op(t, peer, group)

    def _recv_count(self, head, src, slot, pinned, side):
        """Receive a 1-element int32 count from `src` and return it on the host, without waiting for
        the compute queued on the current stream (side stream + pinned copy)."""
        w = self._p2p(irecv, head, src, self.groups[0], side)
        if isinstance(w, _Staged):
            # gloo: the count is already on the host; copying it to the device and reading it back
            # would wait for everything queued on the current stream (the previous chunk's graph)
            w.work.wait()
            return int(w.host.item())
        if side is None:
            w.wait()
            return int(head.item())
        with torch.cuda.stream(side):
            w.wait()
            pinned[slot:slot + 1].copy_(head, non_blocking=True)
            ev = torch.cuda.Event()
            ev.record(side)
        ev.synchronize()
        return int(pinned[slot].item())

    # ------------------------------------------------------------------------------ client
    def client_step(self, x, y):
        """Forward each micro-batch and send it while computing the next; back-propagate each returned
        cut-gradient slice as it lands; all-reduce the client gradient over the client ranks; SGD."""
        c = self.stage
        B, m = x.shape[0], self.micro
        assert B % m == 0, "batch must be divisible by the micro-batch count"
        b = B // m
        dev = x.device
        srv = self.server_rank
        fw, bw = self.groups
        act = None if self.images else self._buf("act", (B, 32, 26, 26), torch.float32, dev)
        img = self._buf("img", (B * IMG_BYTES,), torch.uint8, dev) if self.images else None
        cut = self._buf("cut", (B, 32, 26, 26), torch.float32, dev)
        ship = self.ship_amax
        amx = self._buf("amax", (B,), torch.float32, dev) if ship else None
        if ship and hasattr(c, "emit_amax"):
            c.emit_amax = True
        codec = self._use_codec(dev)
        n = b * 32 * 26 * 26
        side = self._side_stream(dev)
        if side is not None:
            # this step's receives land in buffers the previous step's backward read on the current stream
            side.wait_stream(torch.cuda.current_stream(dev))
        sends, bufs, evs = [], [], []
        counts = self._buf("counts_host", (m,), torch.int32, dev, pin=True) if codec is not None else None
        for k in range(m):
            sl = slice(k * b, (k + 1) * b)
            if img is not None:
                isl = img[k * b * IMG_BYTES:(k + 1) * b * IMG_BYTES]
                c.forward_images(x[sl], isl, amx[sl])
                sends += [isend(isl, srv, fw), isend(y[sl], srv, fw), isend(amx[sl], srv, fw)]
                continue
            c.forward(x[sl], out=act[sl])
            if ship:
                if getattr(c, "_act_amax", None) is not None:
                    amx[sl].copy_(c._act_amax)
                else:                                   # stages without a fused max (CPU protocol tests)
                    torch.amax(act[sl].reshape(b, -1), dim=1, out=amx[sl])
            if codec is None:
                sends += [isend(act[sl], srv, fw), isend(y[sl], srv, fw)] + ([isend(amx[sl], srv, fw)] if ship else [])
                continue
            bk = codec.buffers(("c", k), n, dev)
            codec.encode(act[sl], bk)
            bufs.append(bk)
            counts[k:k + 1].copy_(bk[3], non_blocking=True)
            evs.append(self._record(dev))
        totals = []
        if codec is not None:
            for k in range(m):
                sl = slice(k * b, (k + 1) * b)
                if evs[k] is not None:
                    evs[k].synchronize()          # micro-batch k's encode only: k+1.. keep computing
                    side.wait_event(evs[k])
                t = int(counts[k].item())
                totals.append(t)
                seq = [bufs[k][3], bufs[k][0], y[sl]] + ([amx[sl]] if ship else []) + ([bufs[k][4][:t]] if t else [])
                sends += [self._p2p(isend, u, srv, fw, side) for u in seq]
            gv = [self._buf(("gvals", k), (n,), torch.float32, dev) for k in range(m)]
            recvs = [self._p2p(irecv, gv[k][:totals[k]], srv, bw, side) if totals[k] else None for k in range(m)]
        else:
            recvs = [self._p2p(irecv, cut[k * b:(k + 1) * b], srv, bw, side) for k in range(m)]
        for k in range(m):
            sl = slice(k * b, (k + 1) * b)
            if recvs[k] is not None:
                recvs[k].wait()
            if codec is not None:
                codec.unpack(cut[sl], bufs[k], vals=gv[k])
            c.backward(cut[sl], x=x[sl], act=None if act is None else act[sl], accumulate=k > 0)
        for w in sends:
            w.wait()
        if self.nclients > 1:
            dist.all_reduce(c.grads, group=self.client_group)
        c.step()
        extra = y.numel() * 8 + (B * 4 if ship else 0)
        self.dense_bytes = 2 * cut.numel() * 4 + extra
        self.exchange_bytes = (self.dense_bytes if codec is None else
                               m * 4 + sum(bufs[k][0].numel() * 4 + 2 * totals[k] * 4 for k in range(m)) + extra)
        self.global_step += 1

    # ------------------------------------------------------------------------------ server
    def _chunk(self, k, B, device, codec):
        """Micro-batch k of every client as ONE server step part: [unpack] -> forward / loss / backward
        with the gradient accumulated over chunks -> scaled loss into its slot -> [pack]."""
        s = self.stage
        m, nc = self.micro, self.nclients
        b, G = B // m, nc * B
        CH = nc * b
        n = b * 32 * 26 * 26
        acts = self._inputs(G, device, codec)
        labels = self._buf("labels", (G,), torch.int64, device)
        fused = self._fused(codec)
        self.cut_dense = not fused
        # the fused codec path never writes a dense cut gradient (the dgrad packs it): no [G, 32, 26, 26]
        # buffer (1 GB at K4's 28,672 samples); cuts_by_client allocates it on demand
        cuts = None if fused else self._buf("cuts", (G, 32, 26, 26), torch.float32, device)
        parts = self._buf("loss_parts", (m,), torch.float32, device)
        ch = slice(k * CH, (k + 1) * CH)
        amx = self._buf("amax", (G,), torch.float32, device) if self.ship_amax else None
        if fused:
            # every client part of the chunk in ONE launch per pass (per-launch prologues x parts were most of
            # the codec's cost): count + scan + word ranks, unpack into the images, and (the dgrad) pack
            from . import ops
            t_off, t_unp, t_pack = self._part_tables(k, b, n, device, codec)
            ops.cut_offsets_ranks_parts(t_off, n)
            ops.cut_unpack_x3_parts(t_unp, b, amx[ch], acts[k * CH * IMG_BYTES:(k + 1) * CH * IMG_BYTES])
        elif codec is not None:
            for ci in range(nc):
                bk = codec.buffers(("s", ci, k), n, device)
                codec.offsets(n, bk)
                s0 = k * CH + ci * b
                codec.unpack(acts[s0:s0 + b], bk)
        kw = {}
        if self.ship_amax and self._amax_kw:
            kw["act_amax"] = amx[ch]
        if self.images or fused:
            kw["act16"] = acts[k * CH * IMG_BYTES:(k + 1) * CH * IMG_BYTES]
            if fused:
                kw["cut_pack"] = (t_pack, b)
            _, loss_i = s.compute(None, labels[ch], 1.0 / G, accumulate=k > 0,
                                  cut_grad=None if fused else cuts[ch], **kw)
        else:
            _, loss_i = s.compute(acts[ch], labels[ch], 1.0 / G, accumulate=k > 0, cut_grad=cuts[ch], **kw)
        _loss_sum(loss_i, 1.0 / G, parts[k:k + 1])
        if codec is not None and not fused:
            for ci in range(nc):
                bk = codec.buffers(("s", ci, k), n, device)
                codec.pack(cuts[k * CH + ci * b:k * CH + (ci + 1) * b], bk,
                           vals=self._buf(("gvals", ci, k), (n,), torch.float32, device))

    def _part_tables(self, k, b, n, device, codec):
        """Device pointer tables of chunk k's client parts for the fused codec kernels (int64 [nc, 5] / [nc, 3]
        / [nc, 3], see ops.cut_offsets_ranks_parts / cut_unpack_x3_parts / conv2_dgrad_x3_pack_parts). The
        buffers they point to are never replaced (keyed by size), so each table is written once per (k, b) —
        by the eager warm-up before a graph capture, never inside it."""
        nc = self.nclients
        key = ("tables", k, b)
        tabs = self._pool.get(key)
        if tabs is None:
            rows_off, rows_unp, rows_pack = [], [], []
            for ci in range(nc):
                mask, counts, offsets, total, vals = codec.buffers(("s", ci, k), n, device)
                rk = codec.ranks_buffer(("s", ci, k), n, device)
                gv = self._buf(("gvals", ci, k), (n,), torch.float32, device)
                rows_off.append([t.data_ptr() for t in (mask, counts, offsets, total, rk)])
                rows_unp.append([vals.data_ptr(), mask.data_ptr(), rk.data_ptr()])
                rows_pack.append([mask.data_ptr(), rk.data_ptr(), gv.data_ptr()])
            tabs = tuple(torch.tensor(r, dtype=torch.int64).to(device) for r in (rows_off, rows_unp, rows_pack))
            torch.cuda.current_stream(device).synchronize()
            self._pool[key] = tabs
        return tabs

    def _inputs(self, G, device, codec=None):
        """The server's input buffer of the cut: f32 act [G, 32, 26, 26], or the images' bytes (the dense
        images exchange receives them; the fused codec path unpacks into them)."""
        if self.images or self._fused(codec):
            return self._buf("imgs", (G * IMG_BYTES,), torch.uint8, device)
        return self._buf("acts", (G, 32, 26, 26), torch.float32, device)

    def _graphed(self, device) -> bool:
        return self.graph and torch.device(device).type == "cuda"

    def _prepare(self, B, device, codec):
        """Capture one HIP graph per chunk (first step at this batch size), BEFORE any receive is posted:
        the warm-up runs on zeroed inputs in the very buffers the receives fill later."""
        if not self._graphed(device) or all((k, B, codec is not None) in self._graphs for k in range(self.micro)):
            return
        G = self.nclients * B
        self._inputs(G, device, codec).zero_()
        self._buf("labels", (G,), torch.int64, device).zero_()
        if self.ship_amax:
            self._buf("amax", (G,), torch.float32, device).zero_()
        n = (B // self.micro) * 32 * 26 * 26
        st = torch.cuda.Stream(device)
        for k in range(self.micro):
            if codec is not None:
                for ci in range(self.nclients):
                    codec.buffers(("s", ci, k), n, device)[0].zero_()
            st.wait_stream(torch.cuda.current_stream(device))
            with torch.cuda.stream(st):
                self._chunk(k, B, device, codec)
            torch.cuda.current_stream(device).wait_stream(st)
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g, capture_error_mode="thread_local"):   # see Replicated._graph_for
                self._chunk(k, B, device, codec)
            self._graphs[k, B, codec is not None] = g
        torch.cuda.current_stream(device).synchronize()

    def prepare(self, B: int, device) -> None:
        """Server rank: capture the chunk graphs for per-client batch B now (bench.py does this after a
        synchronize + barrier and before the phase's first exchange); otherwise the first server_step
        captures them. No-op on client ranks (they run eagerly)."""
        if self.is_server:
            self._prepare(B, device, self._use_codec(device))

    def _run_chunk(self, k, B, device, codec):
        if self._graphed(device):
            self._graphs[k, B, codec is not None].replay()
        else:
            self._chunk(k, B, device, codec)

    def server_step(self, B: int, device):
        """B = per-client batch; the server step covers nc*B samples in `micro` chunks, ONE SGD step."""
        s = self.stage
        m, nc = self.micro, self.nclients
        assert B % m == 0, "batch must be divisible by the micro-batch count"
        b, G = B // m, nc * B
        CH = nc * b
        n = b * 32 * 26 * 26
        fw, bw = self.groups
        ship = self.ship_amax
        codec = self._use_codec(device)
        self.cut_dense = not self._fused(codec)
        acts = self._inputs(G, device, codec)
        labels = self._buf("labels", (G,), torch.int64, device)
        cuts = None if not self.cut_dense else self._buf("cuts", (G, 32, 26, 26), torch.float32, device)
        amx = self._buf("amax", (G,), torch.float32, device) if ship else None
        parts = self._buf("loss_parts", (m,), torch.float32, device)
        self._prepare(B, device, codec)
        part = lambda k, ci: slice(k * CH + ci * b, k * CH + (ci + 1) * b)  # noqa: E731
        side = self._side_stream(device)
        if side is not None:
            # receives on the side stream land in buffers the previous step's chunks read
            side.wait_stream(torch.cuda.current_stream(device))
        reqs = {}
        if codec is None:
            for ci, cr in enumerate(self.client_ranks):
                for k in range(m):
                    sl = part(k, ci)
                    asl = slice(sl.start * IMG_BYTES, sl.stop * IMG_BYTES) if self.images else sl
                    reqs[ci, k] = [irecv(acts[asl], cr, fw), irecv(labels[sl], cr, fw)]
                    if ship:
                        reqs[ci, k].append(irecv(amx[sl], cr, fw))
        else:
            pinned = self._buf("counts_host", (m * nc,), torch.int32, device, pin=True)
        totals = {}
        sends = []
        for k in range(m):
            if codec is not None:
                # per client, in its send order: the count, then mask / labels / max / values
                for ci, cr in enumerate(self.client_ranks):
                    sl = part(k, ci)
                    bk = codec.buffers(("s", ci, k), n, device)
                    t = self._recv_count(self._buf(("head", ci, k), (1,), torch.int32, device), cr, k * nc + ci,
                                         pinned, side)
                    totals[ci, k] = t
                    seq = [bk[0], labels[sl]] + ([amx[sl]] if ship else []) + ([bk[4][:t]] if t else [])
                    # on the side stream: the transfer need not wait for chunk k-1's compute
                    reqs[ci, k] = [self._p2p(irecv, u, cr, fw, side) for u in seq]
            for ci in range(nc):
                for r in reqs[ci, k]:
                    r.wait()
            self._run_chunk(k, B, device, codec)
            for ci, cr in enumerate(self.client_ranks):
                if codec is None:
                    sends.append(isend(cuts[part(k, ci)], cr, bw))
                elif totals[ci, k]:
                    gv = self._buf(("gvals", ci, k), (n,), torch.float32, device)
                    sends.append(isend(gv[:totals[ci, k]], cr, bw))
        s.step()
        s.log_loss(parts, scale=1.0, step=self.global_step)
        for w in sends:
            w.wait()
        extra = labels.numel() * 8 + (G * 4 if ship else 0)
        self.dense_bytes = 2 * G * CUT_ELEMS * 4 + extra
        self.exchange_bytes = (self.dense_bytes if codec is None else
                               nc * m * 4 + sum(codec.buffers(("s", ci, k), n, device)[0].numel() * 4 + 2 * t * 4
                                                for (ci, k), t in totals.items()) + extra)
        self.global_step += 1

    def cuts_by_client(self, B: int) -> torch.Tensor:
        """The last step's cut gradient in client order [client][B] (the server keeps [k][client][b]).
        After a fused-codec step (cut_dense False) that is what went on the wire, scattered: the gradient at
        the cut's nonzero positions, zeros elsewhere (positions the client's ReLU discards)."""
        m, nc = self.micro, self.nclients
        if not self.cut_dense:
            # the fused step wrote no dense buffer: scatter the packed gradient into one made here
            dev = self._bufs["labels"].device
            cuts = self._buf("cuts", (nc * B, 32, 26, 26), torch.float32, dev)
            b = B // m
            n = b * 32 * 26 * 26
            for k in range(m):
                for ci in range(nc):
                    s0 = (k * nc + ci) * b
                    self._codec.unpack(cuts[s0:s0 + b], self._codec.buffers(("s", ci, k), n, cuts.device),
                                       vals=self._buf(("gvals", ci, k), (n,), torch.float32, cuts.device))
        else:
            cuts = self._bufs["cuts"]
        return cuts.view(m, nc, B // m, *cuts.shape[1:]).transpose(0, 1).reshape(nc * B, *cuts.shape[1:])


class Pipeline(Hub):
    """2-rank client/server pipeline (BASELINE config 3) with m micro-batches: the hub with one client.
    `role` is "client" or "server", `peer` the other rank. Both sides accumulate their gradient over
    the micro-batches and step once per batch (= the reference step at batch B)."""

    def __init__(self, stage, role: str, peer: int, micro: int = 4, compress=True, graph: bool = True,
                 groups=None, ship_amax: bool = True, images: bool = False, fuse_codec: bool = True):
        assert role in ("client", "server")
        me = dist.get_rank()
        super().__init__(stage, me, dist.get_world_size(), None, micro, compress,
                         server_rank=peer if role == "client" else me,
                         client_ranks=[me] if role == "client" else [peer], graph=graph, groups=groups,
                         ship_amax=ship_amax, images=images, fuse_codec=fuse_codec)
        self.role, self.peer = role, peer


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

    def __init__(self, stage, rank: int, world: int, client_group=None, micro: int = 1, groups=None):
        self.stage, self.rank, self.world = stage, rank, world
        self.server_rank = world - 1
        self.nclients = world - 1
        self.client_group = client_group
        if groups is None:   # one group per direction, as for Hub (exchange_groups)
            groups = exchange_groups() if dist.is_initialized() else (None, None)
        self.groups = tuple(groups)
        self.micro = micro
        self.global_step = 0
        self._bufs = {}
        self.exchange_bytes = 0

    def _buf(self, name, shape, dtype, device):
        key = (name, tuple(shape), dtype, str(torch.device(device)))
        t = self._bufs.get(key)
        if t is None:
            t = torch.empty(shape, dtype=dtype, device=device)
            self._bufs[key] = t
        return t

    def client_step(self, x, y):
        c = self.stage
        B, m = x.shape[0], self.micro
        assert B % m == 0, "batch must be divisible by the micro-batch count"
        b = B // m
        dcut = self._buf("dcut", c.cut_shape(B), c.cut_dtype, x.device)
        fw, bw = self.groups
        sends, recvs = [], []
        for k in range(m):
            sl = slice(k * b, (k + 1) * b)
            cut = c.forward(x[sl], tag=k)
            sends.append(isend(cut, self.server_rank, fw))
            sends.append(isend(y[sl], self.server_rank, fw))
        for k in range(m):
            recvs.append(irecv(dcut[k * b:(k + 1) * b], self.server_rank, bw))
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
        fw, bw = self.groups
        reqs = {}
        for c in range(nc):
            for k in range(m):
                sl = slice(c * B + k * b, c * B + (k + 1) * b)
                reqs[c, k] = (irecv(cuts[sl], c, fw), irecv(labels[sl], c, fw))
        sends, part = [], 0
        for k in range(m):
            for c in range(nc):
                sl = slice(c * B + k * b, c * B + (k + 1) * b)
                for r in reqs[c, k]:
                    r.wait()
                s.accumulate(cuts[sl], labels[sl], 1.0 / G, c * B + k * b, part, m * nc, dcut=dcuts[sl])
                sends.append(isend(dcuts[sl], c, bw))
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
