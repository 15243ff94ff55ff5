"""Deadlock-freedom of the multi-GPU exchange protocols under RCCL's point-to-point semantics, with no
process group at all (CPU, threads).

RCCL (NCCL) runs every point-to-point op between two ranks of one process group in ISSUE order on one
communicator stream, and a send larger than its staging buffer completes only when the peer's matching
receive runs. gloo buffers sends and matches by tag, so a protocol whose two sides issue their ops in
incompatible orders passes every gloo test and hangs under RCCL (the codec hub's
server interleaved "recv micro-batch k, send gradient k, recv k+1" on the same group as a client that
posts all its sends first).

`_Fabric` replays each rank's ops as a thread against that model, made strict:
  * a channel is (group, unordered rank pair) — or (group) alone for `shared=True`, where a group's
    ops of one rank run on ONE stream whatever the peer (torch's eagerly initialised communicators);
  * every send is a rendezvous: it completes only when it and the peer's matching receive are both at
    the heads of their channel queues (sizes and dtypes must match, else the run fails);
  * `wait()` blocks the host until the op completed (stricter than RCCL's stream-level wait).
When every live thread waits on an op that can no longer complete, the run reports a deadlock. Early
completion only removes waits, so a protocol that drains here drains under RCCL's real buffering.

The stages are the CPU oracle stages (float64); the codec is `_TorchCodec`, a torch restatement of
csrc/slk_codec.hip's mask / values layout (test double only — the product codec is the HIP one), so
the codec path's op sequence runs on the CPU. Results are checked against oracle/split_step.py.
"""
import threading
from collections import defaultdict, deque

import numpy as np
import pytest
import torch

from conftest import PKG, ROOT, load_fixture  # noqa: F401

B = 4
STEPS = 2


class Deadlock(RuntimeError):
    pass


class _Op:
    def __init__(self, kind, rank, peer, t, group):
        self.kind, self.rank, self.peer, self.t, self.group = kind, rank, peer, t, group
        self.done = False


class _Work:
    def __init__(self, fab, op):
        self.fab, self.op = fab, op

    def wait(self):
        self.fab.wait(self.op)
        return True


class _Group:
    def __init__(self, name, ranks):
        self.name, self.ranks = name, list(ranks)

    def __repr__(self):
        return f"<group {self.name}>"


class _Fabric:
    """A fake torch.distributed for `nranks` threads (see the module docstring)."""

    def __init__(self, nranks, shared=False):
        self.n = nranks
        self.shared = shared
        self.cv = threading.Condition()
        self.q = defaultdict(deque)          # (channel, rank) -> ops in issue order
        self.waiting = {}                    # rank -> op it waits on
        self.live = nranks
        self.dead = None
        self.local = threading.local()
        self.ngroups = 0
        self.world = _Group("world", range(nranks))
        self.coll = {}                       # collective rendezvous state per (group, seq)
        self.coll_seq = defaultdict(int)
        self.log = defaultdict(list)

    # -- torch.distributed surface used by splitcnn.dist
    def is_initialized(self):
        return True

    def get_rank(self, group=None):
        return self.local.rank

    def get_world_size(self, group=None):
        return self.n if group is None else len(group.ranks)

    def get_backend(self, group=None):
        return "nccl"

    def new_group(self, ranks):
        # every rank calls it in the same order: name the k-th call of each rank alike
        k = self.local.__dict__.setdefault("ngroups", 0)
        self.local.ngroups = k + 1
        return _Group(f"g{k}", ranks)

    def _chan(self, group, a, b):
        g = (group or self.world).name
        return (g,) if self.shared else (g, min(a, b), max(a, b))

    def _post(self, kind, t, peer, group):
        me = self.local.rank
        op = _Op(kind, me, peer, t, group)
        with self.cv:
            self.q[self._chan(group, me, peer), me].append(op)
            self.log[me].append((kind, (group or self.world).name, peer, t.numel(), t.dtype))
            self._progress()
        return _Work(self, op)

    def isend(self, t, dst, group=None):
        return self._post("send", t, dst, group)

    def irecv(self, t, src, group=None):
        return self._post("recv", t, src, group)

    def _progress(self):
        moved = True
        while moved:
            moved = False
            for (chan, r), qu in list(self.q.items()):
                if not qu or qu[0].kind != "send":
                    continue
                s = qu[0]
                pq = self.q.get((chan, s.peer))
                if not pq:
                    continue
                rv = pq[0]
                if rv.kind != "recv" or rv.peer != r:
                    continue
                if rv.t.numel() != s.t.numel() or rv.t.dtype != s.t.dtype:
                    self.dead = AssertionError(f"size mismatch on {chan}: send {s.t.numel()} {s.t.dtype} "
                                               f"from {r}, recv {rv.t.numel()} {rv.t.dtype} on {s.peer}")
                    self.cv.notify_all()
                    return
                rv.t.copy_(s.t)
                qu.popleft()
                pq.popleft()
                s.done = rv.done = True
                moved = True
        self.cv.notify_all()

    def _stuck(self):
        return len(self.waiting) == self.live and all(not op.done for op in self.waiting.values())

    def wait(self, op):
        me = self.local.rank
        with self.cv:
            while not op.done:
                if self.dead is not None:
                    raise self.dead if isinstance(self.dead, AssertionError) else Deadlock(str(self.dead))
                self.waiting[me] = op
                if self._stuck():
                    heads = {f"{c}@{r}": (qq[0].kind, qq[0].peer, qq[0].t.numel()) for (c, r), qq in self.q.items() if qq}
                    self.dead = f"deadlock: every rank waits; channel heads {heads}"
                    self.cv.notify_all()
                    del self.waiting[me]
                    raise Deadlock(self.dead)
                self.cv.wait(timeout=30)
                self.waiting.pop(me, None)

    def all_reduce(self, t, group=None, op=None, async_op=False):
        g = group or self.world
        me = self.local.rank
        with self.cv:
            seq = self.coll_seq[g.name, me]
            self.coll_seq[g.name, me] += 1
            st = self.coll.setdefault((g.name, seq), {"sum": torch.zeros_like(t), "n": 0, "op": _Op("coll", me, -1, t, g)})
            st["sum"] += t
            st["n"] += 1
            if st["n"] == len(g.ranks):
                st["op"].done = True
                self.cv.notify_all()
        self.wait(st["op"])
        t.copy_(st["sum"])

    def barrier(self, group=None):
        self.all_reduce(torch.zeros(1), group)

    # -- thread driver
    def run(self, fns):
        errs = {}

        def body(r, fn):
            self.local.rank = r
            try:
                fn()
            except BaseException as e:  # noqa: BLE001
                errs[r] = e
                with self.cv:
                    if self.dead is None:
                        self.dead = f"rank {r} raised {e!r}"
                    self.cv.notify_all()
            finally:
                with self.cv:
                    self.live -= 1
                    self.waiting.pop(r, None)
                    if self.live and self._stuck() and self.dead is None:
                        self.dead = "deadlock after a rank finished"
                    self.cv.notify_all()
        th = [threading.Thread(target=body, args=(r, fn), daemon=True) for r, fn in enumerate(fns)]
        for t in th:
            t.start()
        for t in th:
            t.join(timeout=120)
        assert not any(t.is_alive() for t in th), "protocol threads did not finish"
        for r in sorted(errs):
            if isinstance(errs[r], Deadlock):
                raise errs[r]
        for r in sorted(errs):
            raise errs[r]


class _TorchCodec:
    """Test double of splitcnn.codec.CutCodec: the same buffer tuple (mask words, counts, offsets,
    total[1], vals[n]) and wire layout — bit k%32 of word k//32 set iff element k's bit pattern is
    nonzero, the values of the set elements in order — computed by torch on the CPU."""

    def __init__(self):
        self._b = {}

    def buffers(self, key, n, device):
        k = (key, n)
        if k not in self._b:
            self._b[k] = (torch.zeros((n + 31) // 32, dtype=torch.int32), torch.zeros(1, dtype=torch.int32),
                          torch.zeros(1, dtype=torch.int32), torch.zeros(1, dtype=torch.int32),
                          torch.zeros(n, dtype=torch.float32))
        return self._b[k]

    @staticmethod
    def _bits(mask, n):
        w = mask.to(torch.int64) & 0xFFFFFFFF
        return (((w.unsqueeze(1) >> torch.arange(32)) & 1).bool().reshape(-1))[:n]

    def encode(self, x, bufs):
        mask, _, _, total, vals = bufs
        flat = x.reshape(-1).to(torch.float32)
        nz = flat.view(torch.int32) != 0
        pad = torch.zeros(mask.numel() * 32, dtype=torch.int64)
        pad[:nz.numel()] = nz.to(torch.int64)
        words = (pad.view(-1, 32) << torch.arange(32)).sum(1)
        mask.copy_(((words + 2 ** 31) % 2 ** 32 - 2 ** 31).to(torch.int32))
        t = int(nz.sum())
        total.fill_(t)
        vals[:t] = flat[nz]

    def offsets(self, n, bufs):
        bufs[3].fill_(int(self._bits(bufs[0], n).sum()))

    def pack(self, x, bufs, vals=None):
        mask, _, _, _, v = bufs
        v = v if vals is None else vals
        sel = self._bits(mask, x.numel())
        t = int(sel.sum())
        v[:t] = x.reshape(-1)[sel].to(torch.float32)

    def unpack(self, out, bufs, vals=None):
        mask, _, _, _, v = bufs
        v = v if vals is None else vals
        sel = self._bits(mask, out.numel())
        flat = torch.zeros(out.numel(), dtype=out.dtype)
        flat[sel] = v[:int(sel.sum())].to(out.dtype)
        out.copy_(flat.view(out.shape))


def _setup():
    import sys
    sys.path[:0] = [PKG, ROOT]
    from oracle.stages import OracleClient, OracleServer
    from splitcnn import dist as sd
    from splitcnn.data import SyntheticMNIST
    fx = load_fixture("split_step_b4.npz")
    P = {k: fx["init_" + k].astype(np.float64) for k in ["W1", "b1", "W2", "b2", "W3", "b3"]}
    return sd, OracleClient, OracleServer, SyntheticMNIST, P


def _reference(P, batches):
    from oracle.split_step import split_step
    losses = []
    for x, y in batches:
        P, rec = split_step(P, x.numpy(), y.numpy())
        losses.append(rec["loss"])
    return P, losses


def _run_hub(monkeypatch, nclients, micro, codec, shared, ship_amax=True, images=False):
    sd, OC, OS, Data, P = _setup()
    world = nclients + 1
    fab = _Fabric(world, shared=shared)
    monkeypatch.setattr(sd, "dist", fab)
    d = Data(9)
    batches = [d.batch(nclients * B) for _ in range(STEPS)]
    out = {}

    def client(r):
        def fn():
            grp = sd.client_group_for(world)
            t = sd.Hub(OC(P), r, world, client_group=grp, micro=micro,
                       compress=_TorchCodec() if codec else False, ship_amax=ship_amax, images=images)
            for x, y in batches:
                sl = slice(r * B, (r + 1) * B)
                t.client_step(x[sl].contiguous(), y[sl].contiguous())
            out[r] = t.stage.named()
        return fn

    def server():
        grp = sd.client_group_for(world)
        t = sd.Hub(OS(P), world - 1, world, client_group=grp, micro=micro,
                   compress=_TorchCodec() if codec else False, ship_amax=ship_amax, images=images)
        for _ in batches:
            t.server_step(B, torch.device("cpu"))
        out["server"] = {**t.stage.named(), "losses": [l for _, l in t.stage.losses]}
    fab.run([client(r) for r in range(nclients)] + [server])
    return fab, out, _reference(P, batches)


def _check(out, ref, nclients):
    P, losses = ref
    for r in range(nclients):
        for k in ("W1", "b1"):
            np.testing.assert_allclose(out[r][k], P[k], rtol=0, atol=1e-6 * np.abs(P[k]).max())
    for k in ("W2", "b2", "W3", "b3"):
        np.testing.assert_allclose(out["server"][k], P[k], rtol=0, atol=1e-6 * np.abs(P[k]).max())
    np.testing.assert_allclose(out["server"]["losses"], losses, rtol=1e-6)


@pytest.mark.parametrize("shared", [False, True])
@pytest.mark.parametrize("nclients,micro,codec", [(1, 1, False), (1, 4, False), (1, 4, True), (3, 2, True),
                                                  (2, 1, True), (3, 2, False), (7, 2, True), (7, 4, False)])
def test_hub_drains_under_rccl_semantics(monkeypatch, nclients, micro, codec, shared):
    """K3 (1 client) and K4 (N-1 clients) with the dense exchange and the codec, micro-batched: both
    sides' op sequences drain under strict rendezvous FIFO semantics, and the result is the oracle's
    step at the concatenated batch."""
    fab, out, ref = _run_hub(monkeypatch, nclients, micro, codec, shared)
    _check(out, ref, nclients)
    # each group carries one direction: the cut group only client -> server, the gradient group only back
    for r, ops in fab.log.items():
        dirs = defaultdict(set)
        for kind, g, peer, _, _ in ops:
            if g != "world":
                dirs[g].add("up" if (kind == "send") == (r < nclients) else "down")
        assert all(len(v) == 1 for v in dirs.values()), (r, dict(dirs))


def test_single_group_hub_deadlocks_under_rccl_semantics(monkeypatch):
    """The round-3 layout (both directions on ONE group) with the codec and 2 micro-batches: the
    simulator must report the deadlock the advisor found — the check has teeth."""
    sd, *_ = _setup()
    real = sd.exchange_groups

    def one_group():
        g = real()
        return g[0], g[0]
    monkeypatch.setattr(sd, "exchange_groups", one_group)
    with pytest.raises(Deadlock):
        _run_hub(monkeypatch, 1, 2, True, False)


def test_codec_double_matches_dense(monkeypatch):
    """The CPU codec double moves exactly the bytes the dense exchange's results need: codec and dense
    hubs end bit-identical (as the HIP codec is, tests/test_dist_gpu.py)."""
    _, a, _ = _run_hub(monkeypatch, 2, 2, True, False)
    _, b, _ = _run_hub(monkeypatch, 2, 2, False, False)
    for k in a["server"]:
        np.testing.assert_array_equal(np.asarray(a["server"][k]), np.asarray(b["server"][k]))
    for r in range(2):
        for k in a[r]:
            np.testing.assert_array_equal(a[r][k], b[r][k])


@pytest.mark.parametrize("nclients,micro", [(1, 1), (1, 4), (3, 2)])
def test_image_exchange_drains_and_matches_dense(monkeypatch, nclients, micro):
    """The image exchange (Hub images=True: act16 bytes + per-sample max up, the cut gradient back) drains
    under strict RCCL semantics for K3 / K4 and ends bit-identical to the dense f32 exchange (the oracle
    stages carry the f32 act's bytes in the image buffer)."""
    sd, *_ = _setup()
    assert sd.IMG_BYTES == 32 * 26 * 26 * 4
    fab, a, ref = _run_hub(monkeypatch, nclients, micro, False, True, images=True)
    _check(a, ref, nclients)
    _, b, _ = _run_hub(monkeypatch, nclients, micro, False, True)
    for k in a["server"]:
        np.testing.assert_array_equal(np.asarray(a["server"][k]), np.asarray(b["server"][k]))
    for r in range(nclients):
        for k in a[r]:
            np.testing.assert_array_equal(a[r][k], b[r][k])
    with pytest.raises(ValueError):
        sd.Hub(None, 0, 2, compress=True, images=True, groups=(None, None))


def test_widehub_drains_under_rccl_semantics(monkeypatch):
    """dist.WideHub (config 5 SplitFed) op order, 2 clients x 2 micro-batches, shared-stream model."""
    import sys
    sys.path[:0] = [PKG, ROOT]
    from oracle.wide_stages import OracleWideClient, OracleWideServer
    from splitcnn import dist as sd
    from splitcnn.wide import SyntheticCIFAR, init_wide_models
    A, Bm = init_wide_models(seed=0)
    Pw = {k: v.detach().double().numpy() for k, v in list(A.state_dict().items()) + list(Bm.state_dict().items())}
    world, wb = 3, 2
    fab = _Fabric(world, shared=True)
    monkeypatch.setattr(sd, "dist", fab)
    d = SyntheticCIFAR(5)
    batches = [d.batch((world - 1) * wb) for _ in range(STEPS)]
    done = []

    def client(r):
        def fn():
            grp = sd.client_group_for(world)
            t = sd.WideHub(OracleWideClient(Pw), r, world, client_group=grp, micro=2)
            for x, y in batches:
                sl = slice(r * wb, (r + 1) * wb)
                t.client_step(x[sl].contiguous(), y[sl].contiguous())
            done.append(r)
        return fn

    def server():
        grp = sd.client_group_for(world)
        t = sd.WideHub(OracleWideServer(Pw), world - 1, world, client_group=grp, micro=2)
        for _ in batches:
            t.server_step(wb, torch.device("cpu"), OracleWideClient.cut_shape, OracleWideClient.cut_dtype)
        done.append("server")
    fab.run([client(r) for r in range(world - 1)] + [server])
    assert sorted(map(str, done)) == ["0", "1", "server"]


def test_hub_images_rejects_a_server_stage_that_cannot_take_images():
    """Hub(images=True) on the server rank raises at construction (not inside the first step, with the
    clients blocked in their sends) unless the stage runs the x3 forward and wgrad."""
    sd, *_ = _setup()
    from splitcnn.engine import ServerStage
    for conv in ("f32", "x3w"):
        with pytest.raises(ValueError, match="images=True"):
            sd.Hub(ServerStage(device="cpu", conv=conv), 1, 2, compress=False, images=True, groups=(None, None))
    sd.Hub(ServerStage(device="cpu", conv="x3"), 1, 2, compress=False, images=True, groups=(None, None))
    # a client rank is not checked (its stage is a client stage)
    sd.Hub(ServerStage(device="cpu", conv="f32"), 0, 2, compress=False, images=True, groups=(None, None))
