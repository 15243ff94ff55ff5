"""GPU parity of the multi-GPU topologies (BASELINE configs K3 / K4) on the real HIP stages.

The protocol classes of splitcnn/dist.py (Pipeline, Hub, Replicated) drive engine.ClientStage /
engine.ServerStage through call sequences the single-GPU trainer never uses:
  ServerStage.compute(accumulate=True, cut_grad=<slice>)      (micro-batches / client parts)
  ClientStage.backward(accumulate=True, x=<slice>, act=<slice>)
  slk_reduce_slabs(..., accumulate=1)
  bind_grads into an all-reduce bucket.
Each of them must reproduce the reference's ONE SGD step at the concatenated batch
(src/server_part.py:47-52, src/client_part.py:132-133), which the golden fixtures pin:
split_step_b12.npz is exactly "3 clients x 4 samples, concatenated", split_step_b14.npz "7 clients x 2
samples" (BASELINE config 4's client count), split_step_b4.npz three consecutive B = 4 steps.

Two layers:
  * loopback tests — the protocol's exact stage-call sequence in one process (no transport);
  * multi-process tests — the dist classes themselves, world 2-4, every rank on cuda:0 over gloo
    (gloo moves the device tensors through the host; RCCL cannot put two ranks on one GPU). Same
    fixtures, same bars: activations 1e-5, cut gradient / gradients 1e-4, loss 1e-5, post-step
    weights via weight_ok (1e-4 of the update).
"""
import os
import socket

import numpy as np
import pytest
import torch

from conftest import PARAMS, PKG, ROOT, load_fixture, rel_err, weight_ok

pytestmark = pytest.mark.gpu

C_OFF = {"W1": (0, 288), "b1": (288, 320)}
S_OFF = {"W2": (0, 18432), "b2": (18432, 18496), "W3": (18496, 110656), "b3": (110656, 110666)}
SHAPES = {"W1": (32, 1, 3, 3), "b1": (32,), "W2": (64, 32, 3, 3), "b2": (64,), "W3": (10, 9216), "b3": (10,)}


def _models(fx):
    from splitcnn.model_def import ModelPartA, ModelPartB
    a, b = ModelPartA(), ModelPartB()
    a.load_state_dict({"conv1.weight": torch.from_numpy(fx["init_W1"]), "conv1.bias": torch.from_numpy(fx["init_b1"])})
    b.load_state_dict({"conv2.weight": torch.from_numpy(fx["init_W2"]), "conv2.bias": torch.from_numpy(fx["init_b2"]),
                       "fc1.weight": torch.from_numpy(fx["init_W3"]), "fc1.bias": torch.from_numpy(fx["init_b3"])})
    return a, b


def _split(flat, offs):
    a = flat.detach().double().cpu().numpy()
    return {k: a[lo:hi].reshape(SHAPES[k]) for k, (lo, hi) in offs.items()}


def _check_step(fx, s, got_params, prev, got_grads=None, got_cut=None, got_act=None, loss=None, cut_dense=True):
    if got_act is not None:
        assert rel_err(got_act, fx[f"act_{s}"]) <= 1e-5
    if got_cut is not None:
        want = fx[f"cut_grad_{s}"]
        if not cut_dense:
            # the fused codec server returns the gradient at the cut's nonzero positions only (what the
            # wire carries; the client's ReLU backward discards the rest): zeros elsewhere
            keep = fx[f"act_{s}"] != 0
            assert not np.asarray(got_cut)[~keep].any()
            want = np.where(keep, want, 0)
        assert rel_err(got_cut, want) <= 1e-4
    if loss is not None:
        assert abs(loss - float(fx[f"loss_{s}"])) <= 1e-5 * abs(float(fx[f"loss_{s}"])), (loss, fx[f"loss_{s}"])
    if got_grads is not None and f"grad_W1_{s}" in fx:
        for k, g in got_grads.items():
            assert rel_err(g, fx[f"grad_{k}_{s}"]) <= 1e-4, (k, s)
    if f"post_W1_{s}" in fx:
        for k, v in got_params.items():
            assert weight_ok(v, fx[f"post_{k}_{s}"], prev[k]), (k, s)


# ----------------------------------------------------------------------------------------- loopback
@pytest.mark.parametrize("m", [1, 2, 4])
def test_pipeline_sequence_loopback(gpu, m):
    """dist.Pipeline's call order in one process: client fwd of every micro-batch into one act
    buffer, server compute(accumulate=k>0, cut_grad=slice) + loss part per micro-batch, ONE server
    SGD + loss log, client backward(accumulate=k>0, x=slice, act=slice), ONE client SGD — three
    consecutive B = 4 steps vs split_step_b4.npz."""
    from splitcnn import ops
    from splitcnn.engine import ClientStage, ServerStage
    fx = load_fixture("split_step_b4.npz")
    a, b = _models(fx)
    c, srv = ClientStage(a, device=gpu), ServerStage(b, device=gpu)
    B, mb = 4, 4 // m
    prev = {k: fx[f"init_{k}"] for k in PARAMS}
    for s in range(1, int(fx["nsteps"]) + 1):
        x = torch.from_numpy(fx[f"x_{s}"]).to(gpu)
        y = torch.from_numpy(fx[f"y_{s}"]).to(gpu)
        acts = torch.empty(B, 32, 26, 26, device=gpu)
        cuts = torch.empty(B, 32, 26, 26, device=gpu)
        parts = torch.empty(m, device=gpu)
        for k in range(m):
            sl = slice(k * mb, (k + 1) * mb)
            c.forward(x[sl], out=acts[sl])
        for k in range(m):
            sl = slice(k * mb, (k + 1) * mb)
            _, loss_i = srv.compute(acts[sl], y[sl], 1.0 / B, accumulate=k > 0, cut_grad=cuts[sl])
            ops.loss_sum(loss_i, 1.0 / B, parts[k:k + 1])
        server_grads = srv.grads.clone()
        srv.step()
        srv.log_loss(parts, scale=1.0, step=s)
        for k in range(m):
            sl = slice(k * mb, (k + 1) * mb)
            c.backward(cuts[sl], x=x[sl], act=acts[sl], accumulate=k > 0)
        client_grads = c.grads.clone()
        c.step()
        torch.cuda.synchronize()
        (step, loss), = srv.loss_log.flush()
        assert step == s
        got = {**_split(c.params, C_OFF), **_split(srv.params, S_OFF)}
        grads = {**_split(client_grads, C_OFF), **_split(server_grads, S_OFF)}
        _check_step(fx, s, got, prev, grads, cuts.cpu().numpy(), acts.cpu().numpy(), loss)
        prev = got


@pytest.mark.parametrize("nclients,m,fixture", [(3, 1, "split_step_b12.npz"), (3, 2, "split_step_b12.npz"),
                                                (2, 2, "split_step_b12.npz"), (7, 1, "split_step_b14.npz"),
                                                (7, 2, "split_step_b14.npz")])
def test_hub_sequence_loopback(gpu, nclients, m, fixture):
    """dist.Hub's call order in one process: each client (own ClientStage, same init) forwards its
    micro-batches; the server consumes (micro-batch, client) parts with mean scale 1/G, accumulating;
    clients back-propagate their slices with accumulate, their 320-float gradients are summed (the
    client all-reduce) and every client steps — vs split_step_b12.npz (12 samples = nclients x B) and,
    at K4's 7 clients, split_step_b14.npz."""
    from splitcnn import ops
    from splitcnn.engine import ClientStage, ServerStage
    fx = load_fixture(fixture)
    G = int(fx["B"])
    B = G // nclients
    b = B // m
    clients = []
    for _ in range(nclients):
        a, _b = _models(fx)
        clients.append(ClientStage(a, device=gpu))
    srv = ServerStage(_models(fx)[1], device=gpu)
    x = torch.from_numpy(fx["x_1"]).to(gpu)
    y = torch.from_numpy(fx["y_1"]).to(gpu)
    acts = torch.empty(G, 32, 26, 26, device=gpu)
    cuts = torch.empty(G, 32, 26, 26, device=gpu)
    parts = torch.empty(m * nclients, device=gpu)
    for ci, c in enumerate(clients):
        for k in range(m):
            sl = slice(ci * B + k * b, ci * B + (k + 1) * b)
            c.forward(x[sl], out=acts[sl])
    part = 0
    for k in range(m):
        for ci in range(nclients):
            sl = slice(ci * B + k * b, ci * B + (k + 1) * b)
            _, loss_i = srv.compute(acts[sl], y[sl], 1.0 / G, accumulate=part > 0, cut_grad=cuts[sl])
            ops.loss_sum(loss_i, 1.0 / G, parts[part:part + 1])
            part += 1
    server_grads = srv.grads.clone()
    srv.step()
    srv.log_loss(parts, scale=1.0, step=1)
    for ci, c in enumerate(clients):
        for k in range(m):
            sl = slice(ci * B + k * b, ci * B + (k + 1) * b)
            c.backward(cuts[sl], x=x[sl], act=acts[sl], accumulate=k > 0)
    total = sum(c.grads.clone() for c in clients)
    for c in clients:
        c.grads.copy_(total)
        c.step()
    torch.cuda.synchronize()
    (_, loss), = srv.loss_log.flush()
    prev = {k: fx[f"init_{k}"] for k in PARAMS}
    for c in clients:
        got = {**_split(c.params, C_OFF), **_split(srv.params, S_OFF)}
        grads = {**_split(c.grads, C_OFF), **_split(server_grads, S_OFF)}
        _check_step(fx, 1, got, prev, grads, cuts.cpu().numpy(), acts.cpu().numpy(), loss)


@pytest.mark.parametrize("nranks", [2, 3])
def test_replicated_bucket_loopback(gpu, nranks):
    """dist.Replicated: every replica binds its client and server gradients into ONE bucket
    [client 320 | server 110,666 | loss]; with the mean scale 1/(N*B) the summed bucket (the
    all-reduce, done here by hand) is the global-batch gradient; each replica steps from it."""
    from splitcnn import ops
    from splitcnn.dist import CLIENT_N, SERVER_N
    from splitcnn.engine import ClientStage, ServerStage
    fx = load_fixture("split_step_b12.npz")
    G = 12
    B = G // nranks
    x = torch.from_numpy(fx["x_1"]).to(gpu)
    y = torch.from_numpy(fx["y_1"]).to(gpu)
    reps = []
    for r in range(nranks):
        a, b = _models(fx)
        c, s = ClientStage(a, device=gpu), ServerStage(b, device=gpu)
        bucket = torch.zeros(CLIENT_N + SERVER_N + 1, device=gpu)
        c.bind_grads(bucket[:CLIENT_N])
        s.bind_grads(bucket[CLIENT_N:CLIENT_N + SERVER_N])
        # bind_grads must rewire the module's .grad views too (state_dict / optimizer users)
        assert c.model.conv1.weight.grad.data_ptr() == bucket.data_ptr()
        assert s.model.fc1.bias.grad.data_ptr() == bucket[CLIENT_N + 110656:].data_ptr()
        reps.append((c, s, bucket))
    cuts = []
    for r, (c, s, bucket) in enumerate(reps):
        sl = slice(r * B, (r + 1) * B)
        act = c.forward(x[sl].contiguous())
        cut, loss_i = s.compute(act, y[sl].contiguous(), 1.0 / G)
        cuts.append(cut.clone())
        c.backward(cut)
        ops.loss_sum(loss_i, 1.0 / G, bucket[-1:])
    total = sum(bk.clone() for _, _, bk in reps)
    for c, s, bucket in reps:
        bucket.copy_(total)
        c.step()
        s.step()
    torch.cuda.synchronize()
    loss = float(total[-1].item())
    prev = {k: fx[f"init_{k}"] for k in PARAMS}
    cut = torch.cat(cuts).cpu().numpy()
    for c, s, bucket in reps:
        got = {**_split(c.params, C_OFF), **_split(s.params, S_OFF)}
        grads = {**_split(bucket[:CLIENT_N], C_OFF), **_split(bucket[CLIENT_N:CLIENT_N + SERVER_N], S_OFF)}
        _check_step(fx, 1, got, prev, grads, cut, None, loss)


# ------------------------------------------------------------------------------ multi-process (gloo)
def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, topo, fixture, micro, outdir, compress=True):
    import sys
    sys.path[:0] = [PKG, ROOT, os.path.join(ROOT, "tests")]
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import torch.distributed as dist
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from splitcnn import dist as sd
    from splitcnn.engine import ClientStage, ServerStage
    dev = torch.device("cuda:0")
    torch.cuda.set_device(dev)
    fx = load_fixture(fixture)
    a, b = _models(fx)
    nsteps = int(fx["nsteps"])
    res = {}
    images = compress == "images"   # the dense exchange of the client's x3 images
    if images:
        compress = False
    try:
        if topo == "pipeline":
            if rank == 0:
                t = sd.Pipeline(ClientStage(a, device=dev), "client", 1, micro=micro, compress=compress, images=images)
            else:
                t = sd.Pipeline(ServerStage(b, device=dev), "server", 0, micro=micro, compress=compress, images=images)
            for s in range(1, nsteps + 1):
                x = torch.from_numpy(fx[f"x_{s}"]).to(dev)
                y = torch.from_numpy(fx[f"y_{s}"]).to(dev)
                if rank == 0:
                    t.client_step(x, y)
                    if not images:
                        res[f"act_{s}"] = t._bufs["act"].cpu().numpy()
                    res[f"params_{s}"] = t.stage.params.cpu().numpy()
                    res[f"grads_{s}"] = t.stage.grads.cpu().numpy()
                    res[f"bytes_{s}"] = np.array([t.exchange_bytes, t.dense_bytes])
                else:
                    t.server_step(x.shape[0], dev)
                    res[f"cut_{s}"] = t.cuts_by_client(x.shape[0]).cpu().numpy()
                    res["cut_dense"] = np.array(t.cut_dense)
                    res[f"params_{s}"] = t.stage.params.cpu().numpy()
                    res[f"grads_{s}"] = t.stage.grads.cpu().numpy()
            if rank == 1:
                torch.cuda.synchronize()
                res["losses"] = np.array([l for _, l in t.stage.loss_log.flush()])
        elif topo == "hub":
            grp = sd.client_group_for(world)
            nc = world - 1
            x = torch.from_numpy(fx["x_1"]).to(dev)
            y = torch.from_numpy(fx["y_1"]).to(dev)
            B = x.shape[0] // nc
            if rank < nc:
                t = sd.Hub(ClientStage(a, device=dev), rank, world, client_group=grp, micro=micro, compress=compress,
                           images=images)
                sl = slice(rank * B, (rank + 1) * B)
                t.client_step(x[sl].contiguous(), y[sl].contiguous())
                if not images:
                    res["act_1"] = t._bufs["act"].cpu().numpy()
            else:
                t = sd.Hub(ServerStage(b, device=dev), rank, world, client_group=grp, micro=micro, compress=compress,
                           images=images)
                t.server_step(B, dev)
                res["cut_1"] = t.cuts_by_client(B).cpu().numpy()
                res["cut_dense"] = np.array(t.cut_dense)
                torch.cuda.synchronize()
                res["losses"] = np.array([l for _, l in t.stage.loss_log.flush()])
            res["params_1"] = t.stage.params.cpu().numpy()
            res["grads_1"] = t.stage.grads.cpu().numpy()
            res["bytes_1"] = np.array([t.exchange_bytes, t.dense_bytes])
        elif topo == "replicated":
            x = torch.from_numpy(fx["x_1"]).to(dev)
            y = torch.from_numpy(fx["y_1"]).to(dev)
            B = x.shape[0] // world
            t = sd.Replicated(ClientStage(a, device=dev), ServerStage(b, device=dev), device=dev)
            sl = slice(rank * B, (rank + 1) * B)
            t.step(x[sl].contiguous(), y[sl].contiguous())
            torch.cuda.synchronize()
            res["cparams_1"] = t.client.params.cpu().numpy()
            res["sparams_1"] = t.server.params.cpu().numpy()
            res["bucket_1"] = t.bucket.cpu().numpy()
            res["losses"] = np.array([l for _, l in t.server.loss_log.flush()])
        elif topo == "widehub":
            from splitcnn.wide import SyntheticCIFAR, WideClientStage, WideServerStage, init_wide_models
            grp = sd.client_group_for(world)
            nc, WB = world - 1, 4
            x, y = SyntheticCIFAR(17).batch(nc * WB)
            x, y = x.to(dev), y.to(dev)
            wa, wb = init_wide_models(seed=0)
            if rank < nc:
                t = sd.WideHub(WideClientStage(wa, device=dev), rank, world, client_group=grp, micro=micro)
                sl = slice(rank * WB, (rank + 1) * WB)
                t.client_step(x[sl].contiguous(), y[sl].contiguous())
            else:
                t = sd.WideHub(WideServerStage(wb, device=dev), rank, world, client_group=grp, micro=micro)
                t.server_step(WB, dev, WideClientStage.cut_shape, WideClientStage.cut_dtype)
                torch.cuda.synchronize()
                res["losses"] = np.array([l for _, l in t.stage.loss_log.flush()])
            torch.cuda.synchronize()
            res["params_1"] = t.stage.params.cpu().numpy()
            res["grads_1"] = t.stage.grads.cpu().numpy()
        np.savez(os.path.join(outdir, f"r{rank}.npz"), **res)
    finally:
        dist.destroy_process_group()


def _spawn(world, topo, fixture, micro, outdir, compress=True):
    import torch.multiprocessing as mp
    os.makedirs(outdir, exist_ok=True)
    mp.spawn(_worker, args=(world, _port(), topo, fixture, micro, str(outdir), compress), nprocs=world, join=True)
    return [dict(np.load(os.path.join(outdir, f"r{r}.npz"))) for r in range(world)]


@pytest.mark.parametrize("micro", [4, 2])
def test_pipeline_two_ranks_vs_fixture(gpu, tmp_path, micro):
    """K3 protocol (client rank 0 <-> server rank 1, micro-batched send/recv, one step per batch),
    three B = 4 steps vs split_step_b4.npz."""
    fx = load_fixture("split_step_b4.npz")
    out = _spawn(2, "pipeline", "split_step_b4.npz", micro, tmp_path)
    prev = {k: fx[f"init_{k}"] for k in PARAMS}
    for s in range(1, int(fx["nsteps"]) + 1):
        got = {**_split(torch.from_numpy(out[0][f"params_{s}"]), C_OFF),
               **_split(torch.from_numpy(out[1][f"params_{s}"]), S_OFF)}
        grads = {**_split(torch.from_numpy(out[0][f"grads_{s}"]), C_OFF),
                 **_split(torch.from_numpy(out[1][f"grads_{s}"]), S_OFF)}
        _check_step(fx, s, got, prev, grads, out[1][f"cut_{s}"], out[0][f"act_{s}"], float(out[1]["losses"][s - 1]),
                    cut_dense=bool(out[1]["cut_dense"]))
        prev = got


@pytest.mark.parametrize("world,micro,fixture", [(4, 2, "split_step_b12.npz"), (3, 1, "split_step_b12.npz"),
                                                (8, 2, "split_step_b14.npz")])
def test_hub_vs_fixture(gpu, tmp_path, world, micro, fixture):
    """K4 protocol (N-1 client ranks -> 1 server rank, client all-reduce) vs split_step_b12.npz, and at
    BASELINE config 4's own world (7 client ranks + 1 server rank, 2 chunks) vs split_step_b14.npz."""
    fx = load_fixture(fixture)
    out = _spawn(world, "hub", fixture, micro, tmp_path)
    prev = {k: fx[f"init_{k}"] for k in PARAMS}
    srv = out[world - 1]
    act = np.concatenate([out[r]["act_1"] for r in range(world - 1)])
    for r in range(world - 1):
        got = {**_split(torch.from_numpy(out[r]["params_1"]), C_OFF), **_split(torch.from_numpy(srv["params_1"]), S_OFF)}
        grads = {**_split(torch.from_numpy(out[r]["grads_1"]), C_OFF), **_split(torch.from_numpy(srv["grads_1"]), S_OFF)}
        _check_step(fx, 1, got, prev, grads, srv["cut_1"], act, float(srv["losses"][0]), cut_dense=bool(srv["cut_dense"]))


@pytest.mark.parametrize("world", [3, 2])
def test_replicated_vs_fixture(gpu, tmp_path, world):
    """Data-parallel replicas (one all-reduce of the [client | server | loss] bucket) vs the
    concatenated-batch step of split_step_b12.npz; every rank ends with identical weights."""
    from splitcnn.dist import CLIENT_N, SERVER_N
    fx = load_fixture("split_step_b12.npz")
    out = _spawn(world, "replicated", "split_step_b12.npz", 1, tmp_path)
    prev = {k: fx[f"init_{k}"] for k in PARAMS}
    for r in range(world):
        o = out[r]
        got = {**_split(torch.from_numpy(o["cparams_1"]), C_OFF), **_split(torch.from_numpy(o["sparams_1"]), S_OFF)}
        bk = torch.from_numpy(o["bucket_1"])
        grads = {**_split(bk[:CLIENT_N], C_OFF), **_split(bk[CLIENT_N:CLIENT_N + SERVER_N], S_OFF)}
        _check_step(fx, 1, got, prev, grads, None, None, float(o["losses"][0]))
        assert np.array_equal(o["cparams_1"], out[0]["cparams_1"]) and np.array_equal(o["sparams_1"], out[0]["sparams_1"])


def test_widened_splitfed_hub_vs_fused_step(gpu, tmp_path):
    """K5 SplitFed protocol (dist.WideHub: 2 client ranks -> 1 server rank, 2 micro-batches each,
    client all-reduce) on the HIP stages vs the fused single-process widened step at the concatenated
    batch of 8: loss 1e-6, server and (all-reduced) client gradients 1e-6 of their max (summation
    order differs), clients identical, and every rank's Adam step = the torch formula on its gradient."""
    from oracle import wide_step as W
    from splitcnn.wide import SyntheticCIFAR, WideTrainer, init_wide_models
    out = _spawn(3, "widehub", "split_step_b4.npz", 2, tmp_path)
    x, y = SyntheticCIFAR(17).batch(8)
    ref = WideTrainer(*init_wide_models(seed=0), device=gpu, graph=False)
    ref.step(x.to(gpu), y.to(gpu))
    torch.cuda.synchronize()
    (_, ref_loss), = ref.loss_log.flush()
    assert abs(float(out[2]["losses"][0]) - ref_loss) <= 1e-6 * abs(ref_loss)

    def close(g, w):
        assert np.abs(g - w).max() <= 1e-6 * np.abs(w).max()
    close(out[0]["grads_1"].astype(np.float64), ref.client.grads.double().cpu().numpy())
    close(out[2]["grads_1"].astype(np.float64), ref.server.grads.double().cpu().numpy())
    assert np.array_equal(out[0]["params_1"], out[1]["params_1"]) and np.array_equal(out[0]["grads_1"], out[1]["grads_1"])
    wa, wb = init_wide_models(seed=0)
    for r, model in ((0, wa), (2, wb)):
        flat0 = np.concatenate([v.detach().double().numpy().ravel() for v in model.state_dict().values()])
        g = out[r]["grads_1"].astype(np.float64)
        want, _, _ = W.adam(flat0, g, np.zeros_like(g), np.zeros_like(g), 1)
        tol = 1e-6 * np.abs(want - flat0).max() + 2 * np.finfo(np.float32).eps * np.abs(want)
        assert (np.abs(out[r]["params_1"].astype(np.float64) - want) <= tol).all(), r


@pytest.mark.parametrize("topo,world,micro,fixture", [("pipeline", 2, 2, "split_step_b4.npz"),
                                                      ("hub", 3, 2, "split_step_b12.npz"),
                                                      ("hub", 8, 2, "split_step_b14.npz")])
def test_cut_codec_bit_identical_to_dense(gpu, tmp_path, topo, world, micro, fixture):
    """The sparse cut codec (the default on CUDA tensors) vs the dense exchange (compress=False):
    every rank's weights, gradients and losses are BIT-identical; the codec moved fewer bytes; the
    cut activations the client kept are the same."""
    dense = _spawn(world, topo, fixture, micro, tmp_path / "dense", compress=False)
    sparse = _spawn(world, topo, fixture, micro, tmp_path / "sparse", compress=True)
    srv = world - 1
    assert bool(dense[srv]["cut_dense"]) and not bool(sparse[srv]["cut_dense"])   # the server packs in its dgrad
    for r in range(world):
        for k in dense[r]:
            if k.startswith("bytes_") or k == "cut_dense":
                continue
            if k.startswith("cut_"):
                # what went on the wire: the dense gradient at the cut's nonzero positions, zeros elsewhere
                act = (np.concatenate([dense[c]["act_1"] for c in range(world - 1)]) if topo == "hub"
                       else dense[0]["act_" + k[4:]])
                assert np.array_equal(np.where(act != 0, dense[r][k], 0), sparse[r][k]), (r, k)
                continue
            assert np.array_equal(dense[r][k], sparse[r][k]), (r, k)
        for k in sparse[r]:
            if k.startswith("bytes_"):
                moved, full = sparse[r][k]
                assert dense[r][k][0] == dense[r][k][1] == full and 0 < moved < full, (r, k, moved, full)


@pytest.mark.parametrize("graph", [True, False])
def test_replicated_fused_world1_rccl_bitwise_vs_split_trainer(gpu, graph):
    """dist.Replicated's fused replica (the single-GPU step's kernels + the bucket all-reduce over RCCL,
    one rank) takes exactly SplitTrainer's steps: parameters and logged losses bitwise equal over four
    B = 256 steps, with and without the HIP graph (src/server_part.py:47-55, src/client_part.py:132-133)."""
    import torch.distributed as dist
    from splitcnn import dist as sd
    from splitcnn.data import SyntheticMNIST, init_models
    from splitcnn.engine import ClientStage, ServerStage, SplitTrainer
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(_port()))
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=gpu)
    try:
        data = SyntheticMNIST(5)
        batches = [tuple(t.to(gpu) for t in data.batch(256)) for _ in range(4)]
        tr = SplitTrainer(*init_models(seed=3), device=gpu, graph=True)
        a, b = init_models(seed=3)
        rep = sd.Replicated(ClientStage(a, device=gpu), ServerStage(b, device=gpu), graph=graph)
        assert rep.fused and rep.graph == graph
        for x, y in batches:
            tr.step(x, y)
            rep.step(x, y)
        torch.cuda.synchronize()
        assert torch.equal(tr.client.params, rep.client.params)
        assert torch.equal(tr.server.params, rep.server.params)
        assert tr.loss_log.flush() == rep.server.loss_log.flush()
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("codec", [False, True])
def test_hub_server_graphs_survive_batch_size_changes(gpu, codec):
    """the hub server's chunk graphs are captured per (chunk, B); after a step at
    another B they must still read the buffers the receives fill. B = 8 -> 4 -> 8 -> 4 with graphs
    must equal the eager server bit for bit (parameters and every cut gradient)."""
    from splitcnn import dist as sd
    from splitcnn.data import SyntheticMNIST, init_models
    from splitcnn.engine import ClientStage, ServerStage
    nc, m = 2, 2

    def make(graph):
        a, b = init_models(seed=0)
        return (sd.Hub(ServerStage(b, device=gpu), rank=nc, world=nc + 1, micro=m, compress=codec, graph=graph),
                ClientStage(a, device=gpu))
    runs = [make(True), make(False)]
    data = SyntheticMNIST(3)
    for B in (8, 4, 8, 4):
        b = B // m
        n = b * 32 * 26 * 26
        parts = [data.batch(b) for _ in range(m * nc)]
        cuts = []
        for hub, cl in runs:
            cl.emit_amax = True
            cdc = hub._use_codec(gpu)
            hub._prepare(B, gpu, cdc)      # (captures at a new B; zeroes the receive buffers)
            G = nc * B
            acts = hub._buf("acts", (G, 32, 26, 26), torch.float32, gpu)
            labels = hub._buf("labels", (G,), torch.int64, gpu)
            amx = hub._buf("amax", (G,), torch.float32, gpu)
            hub._buf("cuts", (G, 32, 26, 26), torch.float32, gpu)
            hub._buf("loss_parts", (m,), torch.float32, gpu)
            for k in range(m):
                for ci in range(nc):
                    sl = slice(k * nc * b + ci * b, k * nc * b + (ci + 1) * b)
                    x, y = parts[k * nc + ci]
                    cl.forward(x.to(gpu), out=acts[sl])     # what the receives would deliver
                    amx[sl].copy_(cl._act_amax)
                    labels[sl].copy_(y.to(gpu))
                    if cdc is not None:
                        cdc.encode(acts[sl], cdc.buffers(("s", ci, k), n, gpu))
            for k in range(m):
                hub._run_chunk(k, B, gpu, cdc)
            hub.stage.step()
            torch.cuda.synchronize()
            cuts.append(hub.cuts_by_client(B).clone() if cdc is None else
                        torch.cat([hub._buf(("gvals", ci, k), (n,), torch.float32, gpu).clone()
                                   for k in range(m) for ci in range(nc)]))
        torch.testing.assert_close(cuts[0], cuts[1], rtol=0, atol=0)
        torch.testing.assert_close(runs[0][0].stage.params, runs[1][0].stage.params, rtol=0, atol=0)


def test_hub_image_exchange_matches_f32_cut_bitwise(gpu):
    """dist.Hub(images=True): the server's chunk graphs fed with the client's x3 split images + maxima
    (ClientStage.forward_images, what the receives deliver) equal the same server fed with the f32 cut
    bit for bit — losses, every cut gradient and the parameters after the SGD step (the image forward
    reads the images conv2_fwd_pool_x3 itself splits from the f32 act). K4 shape: 3 clients x 2 chunks."""
    from splitcnn import dist as sd
    from splitcnn import ops
    from splitcnn.data import SyntheticMNIST, init_models
    from splitcnn.engine import ClientStage, ServerStage
    assert ops.conv2_act16_bytes(1) == sd.IMG_BYTES
    nc, m, B = 3, 2, 64
    b, G = B // m, nc * B
    data = SyntheticMNIST(5)
    parts = [data.batch(b) for _ in range(m * nc)]
    res = []
    for images in (False, True):
        a, s = init_models(seed=0)
        hub = sd.Hub(ServerStage(s, device=gpu), rank=nc, world=nc + 1, micro=m, compress=False, images=images)
        cl = ClientStage(a, device=gpu)
        cl.emit_amax = True
        hub._prepare(B, gpu, None)
        inp = hub._inputs(G, gpu)
        labels = hub._buf("labels", (G,), torch.int64, gpu)
        amx = hub._buf("amax", (G,), torch.float32, gpu)
        hub._buf("cuts", (G, 32, 26, 26), torch.float32, gpu)
        hub._buf("loss_parts", (m,), torch.float32, gpu)
        for k in range(m):
            for ci in range(nc):
                sl = slice(k * nc * b + ci * b, k * nc * b + (ci + 1) * b)
                x, y = parts[k * nc + ci]
                if images:
                    cl.forward_images(x.to(gpu), inp[sl.start * sd.IMG_BYTES:sl.stop * sd.IMG_BYTES], amx[sl])
                else:
                    cl.forward(x.to(gpu), out=inp[sl])
                    amx[sl].copy_(cl._act_amax)
                labels[sl].copy_(y.to(gpu))
        for k in range(m):
            hub._run_chunk(k, B, gpu, None)
        hub.stage.step()
        torch.cuda.synchronize()
        res.append((hub._bufs["loss_parts"].clone(), hub.cuts_by_client(B).clone(), hub.stage.params.clone()))
    for u, v in zip(*res):
        assert torch.equal(u, v)


@pytest.mark.parametrize("topo,world,micro,fixture", [("pipeline", 2, 2, "split_step_b4.npz"),
                                                      ("hub", 3, 2, "split_step_b12.npz"),
                                                      ("hub", 8, 2, "split_step_b14.npz")])
def test_image_exchange_bit_identical_to_dense(gpu, tmp_path, topo, world, micro, fixture):
    """The image exchange (images=True: the client's x3 split images + per-sample max up, the f32 cut
    gradient back) vs the dense f32 exchange, multi-process: every rank's weights, gradients, cut
    gradients and losses are BIT-identical and the same bytes moved."""
    dense = _spawn(world, topo, fixture, micro, tmp_path / "dense", compress=False)
    imgs = _spawn(world, topo, fixture, micro, tmp_path / "images", compress="images")
    for r in range(world):
        for k in imgs[r]:
            assert np.array_equal(dense[r][k], imgs[r][k]), (r, k)
        assert set(dense[r]) - set(imgs[r]) <= {k for k in dense[r] if k.startswith("act_")}
