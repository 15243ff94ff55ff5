"""Label-private U-shaped variant (splitcnn/ushaped.py) on the GPU: same step as the
reference (fixture), and bit-identical to the standard split trainer (same kernels, same inputs,
only the placement of fc1 + loss differs)."""
import numpy as np
import pytest
import torch

from conftest import load_fixture, rel_err, weight_ok

KEYS = {"W1": ("conv1", "weight"), "b1": ("conv1", "bias"), "W2": ("conv2", "weight"),
        "b2": ("conv2", "bias"), "W3": ("fc1", "weight"), "b3": ("fc1", "bias")}


def _params(a, b):
    m = {"conv1": a.conv1, "conv2": b.conv2, "fc1": b.fc1}
    return {k: getattr(m[mod], attr).detach().cpu().numpy() for k, (mod, attr) in KEYS.items()}


@pytest.mark.gpu
def test_ushaped_matches_fixture(gpu):
    from splitcnn.data import init_models
    from splitcnn.ushaped import UShapedTrainer
    fx = load_fixture("split_step_b4.npz")
    a, b = init_models(seed=0)
    tr = UShapedTrainer(a, b, device=gpu)
    n = int(fx["nsteps"])
    for k in range(1, n + 1):
        tr.step(torch.from_numpy(fx[f"x_{k}"]).to(gpu), torch.from_numpy(fx[f"y_{k}"]).to(gpu))
        if k == 1:
            assert rel_err(tr.server._act.cpu().numpy(), fx["act_1"]) <= 1e-5
    got = _params(a, b)
    for key in KEYS:
        assert weight_ok(got[key], fx[f"post_{key}_{n}"], fx[f"init_{key}"]), key
    losses = [l for _, l in tr.loss_log.flush()]
    want = [float(fx[f"loss_{k}"]) for k in range(1, n + 1)]
    assert np.allclose(losses, want, rtol=1e-5)
    tr.client.check_labels()


@pytest.mark.gpu
def test_ushaped_bit_identical_to_split_trainer(gpu):
    from splitcnn.data import SyntheticMNIST, init_models
    from splitcnn.engine import SplitTrainer
    from splitcnn.ushaped import UShapedTrainer
    d = SyntheticMNIST(7)
    batches = [tuple(t.to(gpu) for t in d.batch(256)) for _ in range(3)]
    a1, b1 = init_models(seed=1)
    a2, b2 = init_models(seed=1)
    u = UShapedTrainer(a1, b1, device=gpu)
    # the U-shaped client runs its conv1 wgrad as its own launch: compare with the unfused SplitTrainer
    # (the fused one sums the client gradient in another order; tests/test_x3_gpu.py covers that)
    s = SplitTrainer(a2, b2, device=gpu, graph=False, fuse_client_backward=False)
    for x, y in batches:
        u.step(x, y)
        s.step(x, y)
    p1, p2 = _params(a1, b1), _params(a2, b2)
    for k in KEYS:
        assert np.array_equal(p1[k], p2[k]), k
    assert [l for _, l in u.loss_log.flush()] == [l for _, l in s.loss_log.flush()]
