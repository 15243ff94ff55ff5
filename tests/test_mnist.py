"""Real-MNIST input path: IDX parsing, the HBM-resident loader kernel
(slk_mnist_batch) bit-identical to ToTensor+Normalize (client_part.py:61-64), the DataLoader
contract (client_part.py:98: batch 64, shuffle, ragged last batch) and the MLflow-compatible loss
sink (server_part.py:55). No MNIST download exists offline: the IDX files are synthetic, written by
the same format the real files use."""
import json
import os
import threading
import time

import numpy as np
import pytest
import torch

from conftest import weight_ok


def _synthetic(n, seed=0):
    r = np.random.default_rng(seed)
    img = r.integers(0, 256, size=(n, 28, 28), dtype=np.uint8)
    img[0] = 0
    img[1] = 255
    return img, r.integers(0, 10, size=n, dtype=np.uint8)


def _write(root, img, lbl, gz=False, train=True):
    from splitcnn.mnist import write_idx
    a, b = ("train-images-idx3-ubyte", "train-labels-idx1-ubyte") if train else \
        ("t10k-images-idx3-ubyte", "t10k-labels-idx1-ubyte")
    ext = ".gz" if gz else ""
    write_idx(os.path.join(root, a + ext), img)
    write_idx(os.path.join(root, b + ext), lbl)


@pytest.mark.parametrize("gz", [False, True])
def test_idx_roundtrip_and_dataset(tmp_path, gz):
    from splitcnn.mnist import MnistIDX, read_idx
    img, lbl = _synthetic(37)
    raw = tmp_path / "MNIST" / "raw"
    raw.mkdir(parents=True)
    _write(str(raw), img, lbl, gz=gz)
    ds = MnistIDX(str(tmp_path), train=True)      # torchvision layout root/MNIST/raw
    assert len(ds) == 37 and np.array_equal(ds.images, img) and np.array_equal(ds.labels, lbl)
    # header: magic 0x00000803, dims big-endian
    p = raw / ("train-images-idx3-ubyte" + (".gz" if gz else ""))
    assert read_idx(str(p)).shape == (37, 28, 28)
    with pytest.raises(FileNotFoundError):
        MnistIDX(str(tmp_path), train=False)


def test_idx_rejects_garbage(tmp_path):
    from splitcnn.mnist import read_idx
    p = tmp_path / "bad"
    p.write_bytes(b"\x01\x02\x03\x04hello")
    with pytest.raises(ValueError, match="not an IDX"):
        read_idx(str(p))
    p.write_bytes(bytes([0, 0, 8, 1]) + (5).to_bytes(4, "big") + b"abc")
    with pytest.raises(ValueError, match="data bytes"):
        read_idx(str(p))


def test_oracle_equals_torch_op_sequence():
    """Pin: torchvision 0.17 ToTensor = .to(float32).div(255); Normalize = .sub_(mean).div_(std)."""
    from oracle.mnist import transform
    img, _ = _synthetic(64)
    t = torch.from_numpy(img).unsqueeze(1).to(torch.float32).div(255)
    t = t.sub_(torch.as_tensor([0.1307], dtype=torch.float32).view(-1, 1, 1)).div_(
        torch.as_tensor([0.3081], dtype=torch.float32).view(-1, 1, 1))
    assert np.array_equal(transform(img), t.numpy())


def test_loader_batches_like_reference_dataloader(tmp_path):
    from splitcnn.mnist import DeviceLoader, MnistIDX
    img, lbl = _synthetic(150)
    _write(str(tmp_path), img, lbl)
    ld = DeviceLoader(MnistIDX(str(tmp_path)), batch_size=64, seed=5, device="cpu")
    assert len(ld) == 3                                    # 64, 64, 22 (drop_last=False)
    o1 = ld.order()
    assert sorted(o1.tolist()) == list(range(150))
    ld2 = DeviceLoader(MnistIDX(str(tmp_path)), batch_size=64, seed=5, device="cpu")
    assert torch.equal(ld2.order(), o1)
    assert len(DeviceLoader(MnistIDX(str(tmp_path)), batch_size=64, device="cpu", drop_last=True)) == 2


def _fake_mlflow():
    from fastapi import FastAPI, Request
    app = FastAPI()
    st = {"exps": {}, "runs": {}, "metrics": []}

    @app.get("/api/2.0/mlflow/experiments/get-by-name")
    async def get_by_name(experiment_name: str):
        from fastapi.responses import JSONResponse
        if experiment_name not in st["exps"]:
            return JSONResponse({"error_code": "RESOURCE_DOES_NOT_EXIST"}, status_code=404)
        return {"experiment": {"experiment_id": st["exps"][experiment_name]}}

    @app.post("/api/2.0/mlflow/experiments/create")
    async def create(req: Request):
        body = await req.json()
        st["exps"][body["name"]] = str(len(st["exps"]) + 1)
        return {"experiment_id": st["exps"][body["name"]]}

    @app.post("/api/2.0/mlflow/runs/create")
    async def run_create(req: Request):
        body = await req.json()
        rid = f"run{len(st['runs'])}"
        st["runs"][rid] = body
        return {"run": {"info": {"run_id": rid}}}

    @app.post("/api/2.0/mlflow/runs/log-batch")
    async def log_batch(req: Request):
        body = await req.json()
        st["metrics"] += [(body["run_id"], m["key"], m["step"], m["value"]) for m in body["metrics"]]
        return {}

    return app, st


def test_mlflow_rest_sink_batches_losslog_flush():
    import socket

    import uvicorn
    from splitcnn.engine import LossLog
    from splitcnn.sinks import MlflowRestSink
    app, st = _fake_mlflow()
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    srv = uvicorn.Server(uvicorn.Config(app, host="127.0.0.1", port=port, log_level="warning"))
    th = threading.Thread(target=srv.run, daemon=True)
    th.start()
    try:
        for _ in range(200):
            if srv.started:
                break
            time.sleep(0.05)
        sink = MlflowRestSink(f"http://127.0.0.1:{port}", mode="split")
        assert st["exps"] == {"Split_Learning_Sim": "1"}
        assert st["runs"]["run0"]["run_name"] == "Split_Training"
        log = LossLog("cpu", capacity=8, sink=sink)
        # stand in for three slk_loss_log launches (the ring/counter protocol of the device kernel)
        for i, v in enumerate([2.5, 2.25, 2.0]):
            log.ring[i] = v
            log.note_step(10 + i)
        log.counter[0] = 3
        assert st["metrics"] == []
        log.flush()
        assert st["metrics"] == [("run0", "loss", 10, 2.5), ("run0", "loss", 11, 2.25), ("run0", "loss", 12, 2.0)]
        MlflowRestSink(f"http://127.0.0.1:{port}", mode="split")   # existing experiment is reused
        assert len(st["exps"]) == 1 and len(st["runs"]) == 2
    finally:
        srv.should_exit = True
        th.join(timeout=10)


def test_jsonl_sink(tmp_path):
    from splitcnn.sinks import JsonlSink
    p = tmp_path / "loss.jsonl"
    s = JsonlSink(str(p))
    s(0, 1.5)
    s(1, 1.25)
    s.flush()
    rows = [json.loads(l) for l in p.read_text().splitlines()]
    assert [(r["step"], r["value"]) for r in rows] == [(0, 1.5), (1, 1.25)]


@pytest.mark.gpu
def test_mnist_batch_kernel_bit_exact(gpu, tmp_path):
    from oracle.mnist import batch
    from splitcnn import ops
    img, lbl = _synthetic(1000, seed=3)
    dimg = torch.from_numpy(img).to(gpu)
    dlbl = torch.from_numpy(lbl).to(gpu)
    for B in (1, 3, 64, 999, 1000):
        idx = np.random.default_rng(B).permutation(1000)[:B]
        x, y = ops.mnist_batch(dimg, dlbl, torch.from_numpy(idx).to(gpu))
        wx, wy = batch(img, lbl, idx)
        assert np.array_equal(x.cpu().numpy(), wx), B     # bit-identical to ToTensor + Normalize
        assert np.array_equal(y.cpu().numpy(), wy), B
    err = torch.zeros(1, dtype=torch.int32, device=gpu)
    ops.mnist_batch(dimg, dlbl, torch.tensor([5, 1000, -1], device=gpu), err_flag=err)
    assert int(err.item()) == 1


@pytest.mark.gpu
def test_device_loader_epoch_and_training_step(gpu, tmp_path):
    """One epoch visits every sample once (ragged tail included); a trainer step on a loader batch
    equals the oracle step on the same (bit-identical) inputs."""
    from oracle.mnist import batch
    from oracle.split_step import split_step
    from splitcnn.data import init_models
    from splitcnn.engine import SplitTrainer
    from splitcnn.mnist import DeviceLoader, MnistIDX
    img, lbl = _synthetic(300, seed=4)
    _write(str(tmp_path), img, lbl, gz=True)
    ld = DeviceLoader(MnistIDX(str(tmp_path)), batch_size=64, seed=1, device=gpu)
    order = ld.order()
    ld.gen.manual_seed(1)
    seen, sizes = [], []
    for x, y in ld:
        sizes.append(x.shape[0])
        seen.append((x.cpu().numpy(), y.cpu().numpy()))
    assert sizes == [64, 64, 64, 64, 44]
    wx, wy = batch(img, lbl, order.numpy())
    assert np.array_equal(np.concatenate([s[0] for s in seen]), wx)
    assert np.array_equal(np.concatenate([s[1] for s in seen]), wy)
    a, b = init_models(seed=0)
    P = {"W1": a.conv1.weight, "b1": a.conv1.bias, "W2": b.conv2.weight, "b2": b.conv2.bias,
         "W3": b.fc1.weight, "b3": b.fc1.bias}
    P = {k: v.detach().double().numpy() for k, v in P.items()}
    tr = SplitTrainer(a, b, device=gpu, graph=False)
    x, y = next(iter(ld))
    xs, ys = x.cpu().numpy(), y.cpu().numpy()
    tr.step(x, y)
    Q, rec = split_step(P, xs.astype(np.float64), ys)
    tr.server.loss_log.flush()
    (_, loss), = tr.server.loss_log.history
    assert abs(loss - rec["loss"]) <= 1e-5 * rec["loss"]
    assert weight_ok(a.conv1.weight.detach().cpu().numpy(), Q["W1"], P["W1"])
    assert weight_ok(b.fc1.weight.detach().cpu().numpy(), Q["W3"], P["W3"])
