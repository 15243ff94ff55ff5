"""CPU pins of the widened-model oracle (oracle/wide_step.py, BASELINE config 5).

The reference has no widened model and no fixtures for it (it has no tests at all), so
the oracle's anchor is torch's own semantics, as the north star states for this config: with the bf16
roundings switched off, one oracle step must equal, in float64, torch autograd through nn.Conv2d /
ReLU / MaxPool2d / the same dropout mask / nn.Linear / CrossEntropyLoss followed by torch.optim.Adam
on the very modules splitcnn.wide builds (same seeded init). The bf16 rounding helper is pinned
against torch's own float32 -> bfloat16 cast."""
import numpy as np
import pytest
import torch
import torch.nn.functional as F

from oracle import wide_step as W


def _torch_step(A, Bm, x, y, keep, steps=1):
    """Reference semantics in float64 torch: split forward, CE, backward, Adam (lr 1e-3)."""
    A = A.double()
    Bm = Bm.double()
    opt = torch.optim.Adam(list(A.parameters()) + list(Bm.parameters()), lr=1e-3)
    for t in range(steps):
        opt.zero_grad()
        h = F.relu(A.conv1(x))
        h = F.max_pool2d(F.relu(A.conv2(h)), 2)
        cut = F.max_pool2d(F.relu(A.conv3(h)), 2)
        act = cut.detach().requires_grad_(True)            # the cut hand-off (server_part.py:45)
        d = act.reshape(act.shape[0], -1) * keep[t] / (1 - W.P_DROP)
        loss = F.cross_entropy(Bm.fc(d), y)
        loss.backward()
        cut.backward(act.grad)                            # client_part.py:132
        opt.step()
    return A, Bm, loss.item(), act.grad


def test_oracle_f64_equals_torch_autograd_and_adam():
    from splitcnn.wide import init_wide_models, SyntheticCIFAR
    A, Bm = init_wide_models(seed=0)
    x, y = SyntheticCIFAR(42).batch(3)
    P = {k: v.detach().double().numpy() for k, v in list(A.state_dict().items()) + list(Bm.state_dict().items())}
    opt = {}
    keeps = []
    for t in (1, 2):
        keep = W.dropout_keep(0, t - 1, 3)
        keeps.append(torch.from_numpy(keep.astype(np.float64)))
        P, opt, rec = W.wide_step(P, opt, t, x.double().numpy(), y.numpy(), seed=0, bf=False)
    A2, B2, loss, dcut = _torch_step(A, Bm, x.double(), y, keeps, steps=2)
    assert abs(loss - rec["loss"]) <= 1e-12 * abs(loss)
    np.testing.assert_allclose(rec["dcut"], dcut.numpy(), rtol=0, atol=1e-14)
    got = dict(A2.state_dict(), **B2.state_dict())
    for k, v in got.items():
        np.testing.assert_allclose(P[k], v.numpy(), rtol=0, atol=1e-12, err_msg=k)


def test_oracle_adam_f32_matches_torch_adam():
    rng = np.random.default_rng(0)
    p0 = rng.standard_normal(1000).astype(np.float32)
    tp = torch.nn.Parameter(torch.from_numpy(p0.copy()))
    opt = torch.optim.Adam([tp], lr=1e-3)
    p, m, v = p0, np.zeros_like(p0), np.zeros_like(p0)
    for t in range(1, 6):
        g = rng.standard_normal(1000).astype(np.float32)
        tp.grad = torch.from_numpy(g.copy())
        opt.step()
        p, m, v = W.adam(p, g, m, v, t)
    # same formula, f32 tensor math: agreement to a few ulp
    np.testing.assert_allclose(p, tp.detach().numpy(), rtol=0, atol=4e-7)


def test_bf16_rounding_matches_torch_cast():
    rng = np.random.default_rng(1)
    a = np.concatenate([rng.standard_normal(10000).astype(np.float32) * 10.0 ** rng.integers(-8, 8, 10000),
                        np.array([0.0, -0.0, 1.0, 1.00390625, 1.01171875, 3e-39], np.float32)])
    want = torch.from_numpy(a).to(torch.bfloat16).float().numpy()
    assert np.array_equal(W.bf16(a), want)


def test_dropout_mask_statistics_and_determinism():
    k1 = W.dropout_keep(7, 3, 8)
    k2 = W.dropout_keep(7, 3, 8)
    assert k1.shape == (8, W.CUT_F) and np.array_equal(k1, k2)
    assert abs(k1.mean() - 0.75) < 0.01
    assert not np.array_equal(k1, W.dropout_keep(7, 4, 8))
    assert not np.array_equal(k1, W.dropout_keep(8, 3, 8))
    # sample offset = the same mask rows (SplitFed slices of one concatenated batch)
    assert np.array_equal(W.dropout_keep(7, 3, 8)[5:], W.dropout_keep(7, 3, 3, b0=5))


def test_relu_pool_code_semantics():
    c = np.zeros((1, 1, 2, 4))
    c[0, 0] = [[1.0, 3.0, -1.0, -2.0], [3.0, 2.0, -3.0, 0.0]]
    p, code = W.relu_pool_code(c)
    assert p[0, 0, 0].tolist() == [3.0, 0.0]
    assert code[0, 0, 0].tolist() == [1, W.CODE_NONE]   # tie 3.0/3.0: first max (position 1)
    up = W.unpool(np.ones_like(p), code)
    assert up[0, 0].tolist() == [[0, 1, 0, 0], [0, 0, 0, 0]]


def test_c8_layout_helpers_round_trip():
    from splitcnn.wide import c8_to_nchw, nchw_to_c8
    t = torch.arange(2 * 16 * 3 * 5, dtype=torch.float32).reshape(2, 16, 3, 5)
    c8 = nchw_to_c8(t)
    assert c8.shape == (2, 2, 3, 5, 8)
    assert c8[1, 1, 2, 4, 3] == t[1, 11, 2, 4]
    assert torch.equal(c8_to_nchw(c8), t)


def test_wide_module_contract():
    from splitcnn.wide import WideFullModel, WideModelPartA, WideModelPartB, get_wide_model
    a, b, f = WideModelPartA(), WideModelPartB(), WideFullModel()
    shapes = {k: tuple(v.shape) for k, v in list(a.state_dict().items()) + list(b.state_dict().items())}
    assert shapes == W.PARAM_SHAPES
    assert set(f.state_dict()) == set(shapes)
    assert sum(v.numel() for v in a.parameters()) == 370816
    assert sum(v.numel() for v in b.parameters()) == 163850
    with pytest.raises(RuntimeError, match="HIP kernels"):
        a(torch.zeros(1, 3, 32, 32))
    assert isinstance(get_wide_model("server"), WideModelPartB)
