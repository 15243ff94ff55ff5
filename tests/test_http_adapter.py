"""The HTTP-compatible server adapter (splitcnn/http_server.py) against the reference's
wire contract: pickled {"activations","labels","step"} in, pickled cut gradient out
(src/client_part.py:117-133, src/server_part.py:25-58), 400 in the wrong LEARNING_MODE, /health,
/aggregate_weights (server_part.py:60-93). The GPU test drives it with the reference client's step
code (torch-CPU ModelPartA = Conv2d(1,32,3)+ReLU, model_def.py:5-12) over a real uvicorn socket."""
import os
import pickle
import threading
import time

import numpy as np
import pytest
import torch

from conftest import load_fixture, rel_err, weight_ok


def client_payload(act, labels, step):
    # client_part.py:117-122, byte for byte the same construction
    return pickle.dumps({"activations": act.clone().detach(), "labels": labels, "step": step})


def test_safe_unpickler_accepts_reference_payloads_and_refuses_code():
    from splitcnn.http_server import safe_loads
    act = torch.randn(3, 32, 26, 26)
    y = torch.tensor([1, 2, 3])
    got = safe_loads(client_payload(act, y, 7))
    assert torch.equal(got["activations"], act) and torch.equal(got["labels"], y) and got["step"] == 7
    sd = torch.nn.Linear(4, 2).state_dict()
    got = safe_loads(pickle.dumps({"model_state": sd, "epoch": 1, "loss": 0.5, "step": 3}))
    assert all(torch.equal(got["model_state"][k], sd[k]) for k in sd)

    class Evil:
        def __reduce__(self):
            return (os.system, ("echo pwned",))

    with pytest.raises(pickle.UnpicklingError, match="refused"):
        safe_loads(pickle.dumps({"activations": Evil()}))


def _client(mode):
    from fastapi.testclient import TestClient
    from splitcnn.http_server import make_app
    return TestClient(make_app(device="cpu", learning_mode=mode))


def test_health_and_mode_errors_match_reference():
    c = _client("split")
    assert c.get("/health").json() == {"status": "healthy", "mode": "split", "model_type": "ModelPartB"}
    r = c.post("/aggregate_weights", content=b"x")
    assert r.status_code == 400 and b"only for federated learning mode. Current mode: split" in r.content
    f = _client("federated")
    assert f.get("/health").json()["model_type"] == "FullModel"
    r = f.post("/forward_pass", content=client_payload(torch.zeros(1, 32, 26, 26), torch.zeros(1, dtype=torch.long), 0))
    assert r.status_code == 400 and b"only for split learning mode. Current mode: federated" in r.content


def test_bad_payloads_rejected_before_any_launch():
    c = _client("split")  # device="cpu": any launch would raise, so these must return first
    assert c.post("/forward_pass", content=b"not a pickle").status_code == 400
    r = c.post("/forward_pass", content=client_payload(torch.zeros(2, 32, 26, 25), torch.zeros(2, dtype=torch.long), 0))
    assert r.status_code == 400
    r = c.post("/forward_pass", content=client_payload(torch.zeros(2, 32, 26, 26), torch.tensor([0, 10]), 0))
    assert r.status_code == 500 and b"out of bounds" in r.content


def test_federated_single_client_identity_aggregation():
    """server_part.py:81-93: with one client the returned state is the client's state."""
    from splitcnn.data import init_models
    seen = []
    from fastapi.testclient import TestClient
    from splitcnn.http_server import make_app
    c = TestClient(make_app(device="cpu", learning_mode="federated", sink=lambda s, l: seen.append((s, l))))
    sd = init_models(seed=3, full=True).state_dict()
    r = c.post("/aggregate_weights", content=pickle.dumps({"model_state": sd, "epoch": 2, "loss": 1.25, "step": 9}))
    assert r.status_code == 200
    back = pickle.loads(r.content)
    assert set(back) == set(sd) and all(torch.equal(back[k], sd[k]) for k in sd)
    assert seen == [(9, 1.25)]


def _serve(app):
    import socket

    import uvicorn
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    server = uvicorn.Server(uvicorn.Config(app, host="127.0.0.1", port=port, log_level="warning"))
    th = threading.Thread(target=server.run, daemon=True)
    th.start()
    for _ in range(200):
        if server.started:
            break
        time.sleep(0.05)
    assert server.started
    return server, th, f"http://127.0.0.1:{port}"


@pytest.mark.gpu
def test_reference_client_over_http_matches_golden(gpu):
    """The reference client's loop (client_part.py:110-133) on CPU, over a real socket, against the
    GPU-backed server: cut gradients, the client's SGD result and the logged losses match the fixture."""
    import requests
    from splitcnn.data import init_models
    from splitcnn.engine import LossLog, ServerStage
    from splitcnn.http_server import make_app

    fx = load_fixture("split_step_b4.npz")
    _, model_b = init_models(seed=0)
    server = ServerStage(model_b, device=gpu, loss_log=LossLog(gpu))
    srv, th, url = _serve(make_app(server=server, learning_mode="split"))
    try:
        # the reference ModelPartA (model_def.py:5-12) in stock torch on the CPU, reference init
        conv = torch.nn.Conv2d(1, 32, 3, 1)
        with torch.no_grad():
            conv.weight.copy_(torch.from_numpy(fx["init_W1"]))
            conv.bias.copy_(torch.from_numpy(fx["init_b1"]))
        model = torch.nn.Sequential(conv, torch.nn.ReLU())
        opt = torch.optim.SGD(model.parameters(), lr=0.01)
        for step in range(1, int(fx["nsteps"]) + 1):
            data = torch.from_numpy(fx[f"x_{step}"])
            target = torch.from_numpy(fx[f"y_{step}"])
            opt.zero_grad()
            activations = model(data)
            response = requests.post(url + "/forward_pass", data=client_payload(activations, target, step - 1))
            assert response.status_code == 200, response.content
            server_grads = pickle.loads(response.content)
            assert rel_err(server_grads.numpy(), fx[f"cut_grad_{step}"]) <= 1e-4, step
            activations.backward(server_grads)
            opt.step()
        n = int(fx["nsteps"])
        assert weight_ok(conv.weight.detach().numpy(), fx[f"post_W1_{n}"], fx["init_W1"])
        assert weight_ok(conv.bias.detach().numpy(), fx[f"post_b1_{n}"], fx["init_b1"])
        assert weight_ok(model_b.fc1.weight.detach().cpu().numpy(), fx[f"post_W3_{n}"], fx["init_W3"])
        losses = requests.get(url + "/losses").json()["losses"]
        assert [s for s, _ in losses] == list(range(n))
        want = [float(fx[f"loss_{i}"]) for i in range(1, n + 1)]
        assert np.allclose([l for _, l in losses], want, rtol=1e-5)
    finally:
        srv.should_exit = True
        th.join(timeout=10)


def test_federated_round_averages_k_clients():
    """fed_clients=2: both POSTs wait for the round and get the mean state."""
    import asyncio

    import httpx
    from splitcnn.data import init_models
    from splitcnn.http_server import make_app
    app = make_app(device="cpu", learning_mode="federated", fed_clients=2)
    sds = [init_models(seed=s, full=True).state_dict() for s in (1, 2)]

    async def run():
        transport = httpx.ASGITransport(app=app)
        async with httpx.AsyncClient(transport=transport, base_url="http://t") as c:
            rs = await asyncio.gather(*[
                c.post("/aggregate_weights", content=pickle.dumps(
                    {"model_state": sd, "epoch": 1, "loss": 1.0 + i, "step": 5})) for i, sd in enumerate(sds)])
        return rs

    rs = asyncio.run(run())
    assert all(r.status_code == 200 for r in rs)
    outs = [pickle.loads(r.content) for r in rs]
    for k in sds[0]:
        want = (sds[0][k] + sds[1][k]) / 2
        assert torch.allclose(outs[0][k], want, rtol=0, atol=1e-7) and torch.equal(outs[0][k], outs[1][k])


def test_federated_round_refuses_duplicate_client_and_times_out():
    """A client id posting twice into one open round gets 409 (not counted twice); a round that
    never fills answers 504 after fed_timeout and the next post starts a fresh round. The epoch is
    logged next to the loss (server_part.py:86-87)."""
    import asyncio

    import httpx
    from splitcnn.data import init_models
    from splitcnn.http_server import make_app
    from splitcnn.sinks import JsonlSink

    class Rec(JsonlSink):
        def __init__(self):
            super().__init__(path="/dev/null")
            self.seen = []

        def log_metric(self, key, value, step):
            self.seen.append((key, value, step))

    rec = Rec()
    app = make_app(device="cpu", learning_mode="federated", fed_clients=2, fed_timeout=0.5, sink=rec)
    sd = init_models(seed=1, full=True).state_dict()
    body = lambda cid, loss=1.0: pickle.dumps({"model_state": sd, "epoch": 3, "loss": loss, "step": 7,  # noqa: E731
                                               "client_id": cid})

    async def run():
        transport = httpx.ASGITransport(app=app)
        async with httpx.AsyncClient(transport=transport, base_url="http://t") as c:
            first = asyncio.create_task(c.post("/aggregate_weights", content=body("a")))
            await asyncio.sleep(0.05)
            dup = await c.post("/aggregate_weights", content=body("a"))
            timed_out = await first
            fresh = await asyncio.gather(c.post("/aggregate_weights", content=body("a", 1.0)),
                                         c.post("/aggregate_weights", content=body("b", 3.0)))
        return dup, timed_out, fresh

    dup, timed_out, fresh = asyncio.run(run())
    assert dup.status_code == 409
    assert timed_out.status_code == 504
    assert [r.status_code for r in fresh] == [200, 200]
    assert rec.seen == [("loss", 2.0, 7), ("epoch", 3.0, 7)]


def test_federated_round_abandon_and_failure_release_every_waiter():
    """A round abandoned by one waiter's timeout releases every other waiter of that round at once
    (504, not after its own timeout), and an aggregation that raises answers every waiter 500 at once."""
    import asyncio
    import time

    import httpx
    from splitcnn.data import init_models
    from splitcnn.http_server import make_app
    sd = init_models(seed=1, full=True).state_dict()
    body = lambda cid, state=sd: pickle.dumps({"model_state": state, "epoch": 1, "loss": 1.0, "step": 3,  # noqa: E731
                                               "client_id": cid})

    async def abandon():
        app = make_app(device="cpu", learning_mode="federated", fed_clients=3, fed_timeout=1.0)
        transport = httpx.ASGITransport(app=app)
        async with httpx.AsyncClient(transport=transport, base_url="http://t") as c:
            t0 = time.monotonic()
            a = asyncio.create_task(c.post("/aggregate_weights", content=body("a")))
            await asyncio.sleep(0.6)
            b = asyncio.create_task(c.post("/aggregate_weights", content=body("b")))
            ra = await a
            rb = await b
            return ra, rb, time.monotonic() - t0

    ra, rb, dt = asyncio.run(abandon())
    assert ra.status_code == 504 and rb.status_code == 504
    assert dt < 1.5, dt   # b was released with a (t = 1.0), not at its own timeout (t = 1.6)

    async def failing():
        app = make_app(device="cpu", learning_mode="federated", fed_clients=2, fed_timeout=30.0)
        bad = {k + "_x": v for k, v in sd.items()}   # keys FullModel does not have: load_state_dict raises
        transport = httpx.ASGITransport(app=app)
        async with httpx.AsyncClient(transport=transport, base_url="http://t") as c:
            t0 = time.monotonic()
            rs = await asyncio.gather(c.post("/aggregate_weights", content=body("a", bad)),
                                      c.post("/aggregate_weights", content=body("b", bad)))
            return rs, time.monotonic() - t0

    rs, dt = asyncio.run(failing())
    assert [r.status_code for r in rs] == [500, 500] and dt < 10, ([r.status_code for r in rs], dt)


def test_mlflow_sink_keeps_metrics_until_posted(monkeypatch):
    """MlflowRestSink.flush drops a chunk only after the tracking server accepted it: a failed post
    raises and the next flush re-sends the same metrics."""
    from splitcnn import sinks

    class Resp:
        def __init__(self, ok):
            self.ok = ok
            self.status_code = 200 if ok else 503

        def raise_for_status(self):
            if not self.ok:
                raise RuntimeError("503")

    posts = []
    outcomes = iter([False, True])

    def fake_api(self, method, path, **kw):
        posts.append([m["step"] for m in kw["json"]["metrics"]])
        return Resp(next(outcomes))

    monkeypatch.setattr(sinks.MlflowRestSink, "_api", fake_api)
    s = sinks.MlflowRestSink.__new__(sinks.MlflowRestSink)
    s.key, s.run_id, s._pending = "loss", "r", []
    s(1, 0.5)
    s(2, 0.4)
    with pytest.raises(RuntimeError):
        s.flush()
    s.flush()
    assert posts == [[1, 2], [1, 2]] and s._pending == []
