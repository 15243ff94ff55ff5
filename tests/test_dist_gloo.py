"""Multi-rank protocols of splitcnn/dist.py on the CPU (gloo), driven with oracle-backed stages:
after two steps every topology must equal the single-process reference step at its global batch
(Replicated: N*B concatenated; Pipeline: B in micro-batches; Hub: (N-1)*B concatenated)."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from conftest import PKG, ROOT, load_fixture

B = 4
STEPS = 2


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _init_params():
    fx = load_fixture("split_step_b4.npz")
    return {k: fx["init_" + k].astype(np.float64) for k in ["W1", "b1", "W2", "b2", "W3", "b3"]}


def _batches(n_samples):
    import sys
    sys.path[:0] = [PKG, ROOT]
    from splitcnn.data import SyntheticMNIST
    d = SyntheticMNIST(9)
    return [d.batch(n_samples) for _ in range(STEPS)]


WB = 2  # per-client batch of the widened hub test


def _wide_init():
    import sys
    sys.path[:0] = [PKG, ROOT]
    from splitcnn.wide import init_wide_models
    A, Bm = init_wide_models(seed=0)
    return {k: v.detach().double().numpy() for k, v in list(A.state_dict().items()) + list(Bm.state_dict().items())}


def _wide_batches(n_samples):
    import sys
    sys.path[:0] = [PKG, ROOT]
    from splitcnn.wide import SyntheticCIFAR
    d = SyntheticCIFAR(5)
    return [d.batch(n_samples) for _ in range(STEPS)]


def _worker(rank, world, port, topo, outdir):
    import sys
    sys.path[:0] = [PKG, ROOT]
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    torch.set_num_threads(1)
    from oracle.stages import OracleClient, OracleServer
    from splitcnn import dist as sd
    P = _init_params()
    try:
        if topo == "replicated":
            batches = _batches(world * B)
            t = sd.Replicated(OracleClient(P), OracleServer(P), device=torch.device("cpu"))
            for x, y in batches:
                sl = slice(rank * B, (rank + 1) * B)
                t.step(x[sl].contiguous(), y[sl].contiguous())
            res = {**t.client.named(), **t.server.named(), "losses": [l for _, l in t.server.losses]}
        elif topo == "pipeline":
            batches = _batches(B)
            if rank == 0:
                t = sd.Pipeline(OracleClient(P), "client", 1, micro=2, compress=False)
                for x, y in batches:
                    t.client_step(x, y)
                res = t.stage.named()
            else:
                t = sd.Pipeline(OracleServer(P), "server", 0, micro=2, compress=False)
                for _ in batches:
                    t.server_step(B, torch.device("cpu"))
                res = {**t.stage.named(), "losses": [l for _, l in t.stage.losses]}
        elif topo == "ushaped":
            from oracle.stages import OracleUClient, OracleUServer
            batches = _batches(B)
            if rank == 0:
                t = sd.UShaped(OracleUClient(P), "client", 1)
                for x, y in batches:
                    t.client_step(x, y)
                res = {**t.stage.named(), "losses": [l for _, l in t.stage.losses]}
            else:
                t = sd.UShaped(OracleUServer(P), "server", 0)
                for _ in batches:
                    t.server_step(B, torch.device("cpu"), dtype=torch.float64)
                res = t.stage.named()
        elif topo in ("hub", "hub_m2"):
            batches = _batches((world - 1) * B)
            grp = sd.client_group_for(world)
            micro = 2 if topo == "hub_m2" else 1
            if rank < world - 1:
                t = sd.Hub(OracleClient(P), rank, world, client_group=grp, micro=micro, compress=False)
                for x, y in batches:
                    sl = slice(rank * B, (rank + 1) * B)
                    t.client_step(x[sl].contiguous(), y[sl].contiguous())
                res = t.stage.named()
            else:
                t = sd.Hub(OracleServer(P), rank, world, client_group=grp, micro=micro, compress=False)
                for _ in batches:
                    t.server_step(B, torch.device("cpu"))
                res = {**t.stage.named(), "losses": [l for _, l in t.stage.losses]}
        elif topo == "widehub":
            from oracle.wide_stages import OracleWideClient, OracleWideServer
            Pw = _wide_init()
            batches = _wide_batches((world - 1) * WB)
            grp = sd.client_group_for(world)
            if rank < world - 1:
                t = sd.WideHub(OracleWideClient(Pw), rank, world, client_group=grp, micro=2)
                for x, y in batches:
                    sl = slice(rank * WB, (rank + 1) * WB)
                    t.client_step(x[sl].contiguous(), y[sl].contiguous())
                res = t.stage.named()
            else:
                t = sd.WideHub(OracleWideServer(Pw), rank, world, client_group=grp, micro=2)
                for _ in batches:
                    t.server_step(WB, torch.device("cpu"), OracleWideClient.cut_shape, OracleWideClient.cut_dtype)
                res = {**t.stage.named(), "losses": [l for _, l in t.stage.losses]}
        np.savez(os.path.join(outdir, f"r{rank}.npz"), **{k: np.asarray(v) for k, v in res.items()})
    finally:
        dist.destroy_process_group()


def _reference(global_batch):
    import sys
    sys.path[:0] = [PKG, ROOT]
    from oracle.split_step import split_step
    P = _init_params()
    losses = []
    for x, y in _batches(global_batch):
        P, rec = split_step(P, x.numpy(), y.numpy())
        losses.append(rec["loss"])
    return P, losses


@pytest.mark.parametrize("topo,world,gb", [("replicated", 2, 2 * B), ("pipeline", 2, B), ("hub", 3, 2 * B),
                                           ("hub_m2", 4, 3 * B), ("ushaped", 2, B)])
def test_topology_equals_single_process_step(tmp_path, topo, world, gb):
    mp.spawn(_worker, args=(world, _port(), topo, str(tmp_path)), nprocs=world, join=True)
    P, losses = _reference(gb)
    outs = [dict(np.load(tmp_path / f"r{r}.npz")) for r in range(world)]
    if topo == "ushaped":   # labels, fc1 and the loss live on the client (rank 0)
        want = {0: ["W1", "b1", "W3", "b3", "losses"], 1: ["W2", "b2"]}
    else:
        client_ranks = range(world) if topo == "replicated" else range(world - 1)  # hub: server = last
        server_ranks = range(world) if topo == "replicated" else [world - 1]
        want = {r: [] for r in range(world)}
        for r in client_ranks:
            want[r] += ["W1", "b1"]
        for r in server_ranks:
            want[r] += ["W2", "b2", "W3", "b3", "losses"]
    for r, keys in want.items():
        for k in keys:
            if k == "losses":
                np.testing.assert_allclose(outs[r]["losses"], losses, rtol=1e-6)
            else:
                np.testing.assert_allclose(outs[r][k], P[k], rtol=0, atol=1e-6 * np.abs(P[k]).max())

def test_widened_splitfed_hub_equals_single_process_step(tmp_path):
    """dist.WideHub (BASELINE config 5 SplitFed: 2 client ranks -> 1 server rank, client all-reduce)
    equals oracle/wide_step.py's single-process widened step at the concatenated batch, step by step."""
    import sys
    sys.path[:0] = [PKG, ROOT]
    from oracle import wide_step as Wd
    world = 3
    mp.spawn(_worker, args=(world, _port(), "widehub", str(tmp_path)), nprocs=world, join=True)
    P, opt, losses = _wide_init(), {}, []
    for t, (x, y) in enumerate(_wide_batches((world - 1) * WB), start=1):
        P, opt, rec = Wd.wide_step(P, opt, t, x.double().numpy(), y.numpy(), seed=0, bf=False)
        losses.append(rec["loss"])
    outs = [dict(np.load(tmp_path / f"r{r}.npz")) for r in range(world)]
    for r in range(world - 1):
        for k in Wd.CLIENT_KEYS:
            np.testing.assert_allclose(outs[r][k], P[k], rtol=0, atol=1e-9 * np.abs(P[k]).max(), err_msg=k)
    for k in Wd.SERVER_KEYS:
        np.testing.assert_allclose(outs[world - 1][k], P[k], rtol=0, atol=1e-9 * np.abs(P[k]).max(), err_msg=k)
    np.testing.assert_allclose(outs[world - 1]["losses"], losses, rtol=1e-10)


FED_B = (4, 2)     # unequal local batches: FedAvg weights must follow the sample counts
FED_ROUNDS = (2, 1)  # local steps per round


def _fed_batches(rank):
    import sys
    sys.path[:0] = [PKG, ROOT]
    from splitcnn.data import SyntheticMNIST
    d = SyntheticMNIST(100 + rank)
    return [d.batch(FED_B[rank]) for _ in range(sum(FED_ROUNDS))]


def _fed_worker(rank, world, port, outdir):
    import sys
    sys.path[:0] = [PKG, ROOT]
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    torch.set_num_threads(1)
    from oracle.stages import OracleClient, OracleServer
    from splitcnn import dist as sd
    try:
        P = _init_params()
        fed = sd.FedAvg(OracleClient(P), OracleServer(P), device=torch.device("cpu"))
        it = iter(_fed_batches(rank))
        step = 0
        for r, nloc in enumerate(FED_ROUNDS):
            for _ in range(nloc):
                fed.local_step(*next(it))
                step += 1
            fed.aggregate(step=step - 1)
        res = {**fed.client.named(), **fed.server.named(), "losses": [l for _, l in fed.server.losses],
               "steps": [s for s, _ in fed.server.losses]}
        np.savez(os.path.join(outdir, f"r{rank}.npz"), **{k: np.asarray(v) for k, v in res.items()})
    finally:
        dist.destroy_process_group()


def test_fedavg_round_equals_weighted_average_of_local_training(tmp_path):
    """client_part.py:143-195 per rank (full-model local SGD), then sample-weighted averaging in
    place of server_part.py:81's identity load_state_dict; equal to the oracle run rank by rank."""
    import sys
    sys.path[:0] = [PKG, ROOT]
    from oracle.split_step import split_step
    world = 2
    mp.spawn(_fed_worker, args=(world, _port(), str(tmp_path)), nprocs=world, join=True)
    P = _init_params()
    data = [iter(_fed_batches(r)) for r in range(world)]
    want_losses = []
    for nloc in FED_ROUNDS:
        locals_, lsum = [], 0.0
        for r in range(world):
            Q = dict(P)
            ls = []
            for _ in range(nloc):
                x, y = next(data[r])
                Q, rec = split_step(Q, x.numpy(), y.numpy())
                ls.append(rec["loss"])
            locals_.append(Q)
            lsum += FED_B[r] * nloc * np.mean(ls)
        wts = np.array([FED_B[r] * nloc for r in range(world)], dtype=np.float64)
        P = {k: sum(w * Q[k] for w, Q in zip(wts, locals_)) / wts.sum() for k in P}
        want_losses.append(lsum / wts.sum())
    outs = [dict(np.load(tmp_path / f"r{r}.npz")) for r in range(world)]
    for r in range(world):
        for k in P:
            np.testing.assert_allclose(outs[r][k], P[k], rtol=0, atol=1e-9 * np.abs(P[k]).max())
        np.testing.assert_allclose(outs[r]["losses"], want_losses, rtol=1e-9)
        assert list(outs[r]["steps"]) == [FED_ROUNDS[0] - 1, sum(FED_ROUNDS) - 1]
