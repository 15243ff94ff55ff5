"""GPU: the Winograd F(2x2,3x3) conv2 kernels (the production path behind slk_conv2_fwd_pool /
slk_conv2_dgrad / slk_conv2_wgrad) against the direct implicit-GEMM kernels kept in the library
(slk_conv2_*_direct) and against the numpy oracle, on identical inputs: ragged batches (1, 5, 64,
130), the padded 12th tile group of dgrad, determinism.

Tolerances: Winograd and direct are both f32 with different summation orders; measured and simulated
differences are ~3e-7 relative, asserted at 1e-5 (max |diff| / max |ref|). Max-pool routing may differ
only at numerical ties of the fp64 conv output (tie_discrepancies, 1e-5)."""
import numpy as np
import pytest
import torch

from conftest import rel_err

pytestmark = pytest.mark.gpu


def _inputs(gpu, B, seed):
    from splitcnn.data import SyntheticMNIST, init_models
    from splitcnn.engine import ClientStage
    a, b = init_models(seed=seed)
    x, y = SyntheticMNIST(seed + 1).batch(B)
    act = ClientStage(a, device=gpu).forward(x.to(gpu)).clone()
    p = {k: v.detach().to(gpu).contiguous() for k, v in
         {"W2": b.conv2.weight, "b2": b.conv2.bias, "W3": b.fc1.weight, "b3": b.fc1.bias}.items()}
    return act, p, y.to(gpu)


@pytest.mark.parametrize("B", [1, 5, 64, 130])
def test_winograd_matches_direct_and_oracle(gpu, B):
    from oracle.split_step import conv3x3, conv3x3_dgrad, conv3x3_wgrad, maxpool2_bwd, relu, tie_discrepancies
    from splitcnn import ops
    act, p, y = _inputs(gpu, B, seed=B)
    pw, cw = ops.conv2_fwd_pool(act, p["W2"], p["b2"])
    pd, cd = ops.conv2_fwd_pool(act, p["W2"], p["b2"], direct=True)
    a64 = act.double().cpu().numpy()
    r = relu(conv3x3(a64, p["W2"].double().cpu().numpy(), p["b2"].double().cpu().numpy()))
    codes_w, codes_d = cw.cpu().numpy().astype(np.int64), cd.cpu().numpy().astype(np.int64)
    n, ok = tie_discrepancies(r, codes_d, codes_w)
    assert ok, f"{n} routing differences that are not ties"
    same = torch.from_numpy(codes_w == codes_d).to(gpu)
    assert rel_err(pw[same].cpu().numpy(), pd[same].cpu().numpy()) <= 1e-5
    pr = r.reshape(B, 64, 12, 2, 12, 2).max(axis=(3, 5))
    assert rel_err(pw.cpu().numpy(), pr) <= 1e-5

    # backward on identical inputs (the Winograd forward's routing for both paths)
    _, _, _, dp = ops.fc_xent(pw, p["W3"], p["b3"], y, 1.0 / B)
    gw = ops.conv2_dgrad(dp, cw, p["W2"])
    gd = ops.conv2_dgrad(dp, cw, p["W2"], direct=True)
    assert rel_err(gw.cpu().numpy(), gd.cpu().numpy()) <= 1e-5
    # oracle: dc from the GPU routing, then the fp64 input / weight gradients
    dp64 = dp.double().cpu().numpy().reshape(B, 64, 12, 12)
    dc = maxpool2_bwd(np.where(codes_w < 4, dp64, 0.0), np.minimum(codes_w, 3), (B, 64, 24, 24))
    assert rel_err(gw.cpu().numpy(), conv3x3_dgrad(dc, p["W2"].double().cpu().numpy())) <= 1e-5
    sw = ops.reduce_slabs(ops.conv2_wgrad_slabs(act, dp, cw))
    sd = ops.reduce_slabs(ops.conv2_wgrad_slabs(act, dp, cw, direct=True))
    assert ops.conv2_wgrad_nslab(B) == min(3 * B, 256)
    assert rel_err(sw[:18432].cpu().numpy(), sd[:18432].cpu().numpy()) <= 1e-5
    assert rel_err(sw[18432:].cpu().numpy(), sd[18432:].cpu().numpy()) <= 1e-5
    dW, db = conv3x3_wgrad(a64, dc)
    assert rel_err(sw[:18432].cpu().numpy(), dW.reshape(-1)) <= 1e-5
    assert rel_err(sw[18432:].cpu().numpy(), db) <= 1e-5


def test_winograd_kernels_deterministic(gpu):
    from splitcnn import ops
    B = 300
    act, p, y = _inputs(gpu, B, seed=3)
    runs = []
    for _ in range(2):
        pw, cw = ops.conv2_fwd_pool(act, p["W2"], p["b2"])
        _, _, _, dp = ops.fc_xent(pw, p["W3"], p["b3"], y, 1.0 / B)
        runs.append((pw.clone(), cw.clone(), ops.conv2_dgrad(dp, cw, p["W2"]).clone(),
                     ops.reduce_slabs(ops.conv2_wgrad_slabs(act, dp, cw)).clone()))
    for a, b in zip(*runs):
        assert torch.equal(a, b)


@pytest.mark.parametrize("B", [257, 300, 777])
def test_winograd_multi_unit_per_workgroup(gpu, B):
    """Batches past one unit per workgroup: the forward's two band streams per workgroup (odd band
    count at B = 777), and dgrad's rolling 169-tile stream whose 32-tile iterations straddle
    samples held in different LDS buffers (B = 257: one workgroup with 2 samples). Winograd vs direct
    kernels on identical inputs."""
    from splitcnn import ops
    act, p, y = _inputs(gpu, B, seed=B)
    pw, cw = ops.conv2_fwd_pool(act, p["W2"], p["b2"])
    pd, cd = ops.conv2_fwd_pool(act, p["W2"], p["b2"], direct=True)
    same = cw == cd
    assert same.float().mean().item() > 0.9999
    assert rel_err(pw[same].cpu().numpy(), pd[same].cpu().numpy()) <= 1e-5
    _, _, _, dp = ops.fc_xent(pw, p["W3"], p["b3"], y, 1.0 / B)
    gw = ops.conv2_dgrad(dp, cw, p["W2"])
    gd = ops.conv2_dgrad(dp, cw, p["W2"], direct=True)
    assert torch.isfinite(gw).all()
    assert rel_err(gw.cpu().numpy(), gd.cpu().numpy()) <= 1e-5
    # every sample's cut gradient individually (a misrouted straddling group would hit one sample)
    num = (gw - gd).abs().flatten(1).max(dim=1).values
    den = gd.abs().flatten(1).max(dim=1).values.clamp_min(1e-30)
    assert (num / den).max().item() <= 1e-5
    sw = ops.reduce_slabs(ops.conv2_wgrad_slabs(act, dp, cw))
    sd = ops.reduce_slabs(ops.conv2_wgrad_slabs(act, dp, cw, direct=True))
    assert rel_err(sw[:18432].cpu().numpy(), sd[:18432].cpu().numpy()) <= 1e-5
    assert rel_err(sw[18432:].cpu().numpy(), sd[18432:].cpu().numpy()) <= 1e-5


def test_full_size_b4096_vs_direct_and_oracle(gpu):
    """K2 size (B = 4096, where every dgrad/wgrad workgroup runs 16 units of its persistent stream):
    Winograd fwd / dgrad / wgrad against the independent direct implicit-GEMM kernels on identical
    inputs — pooled outside tie-routed windows, the cut gradient per sample, dW2 / db2 — all at 1e-5;
    then dW3 / db3 (fc wgrad) and dW1 / db1 (client conv1 wgrad) against the fp64 oracle on the
    same GPU-produced operands at 1e-5 / 1e-4."""
    from oracle.split_step import client_backward, cross_entropy
    from splitcnn import ops
    from splitcnn.data import SyntheticMNIST, init_models
    from splitcnn.engine import ClientStage
    B = 4096
    a, b = init_models(seed=21)
    x, y = SyntheticMNIST(22).batch(B)
    x, y = x.to(gpu), y.to(gpu)
    client = ClientStage(a, device=gpu)
    act = client.forward(x).clone()
    p = {k: v.detach().to(gpu).contiguous() for k, v in
         {"W2": b.conv2.weight, "b2": b.conv2.bias, "W3": b.fc1.weight, "b3": b.fc1.bias}.items()}
    pw, cw = ops.conv2_fwd_pool(act, p["W2"], p["b2"])
    pd, cd = ops.conv2_fwd_pool(act, p["W2"], p["b2"], direct=True)
    same = cw == cd
    assert same.float().mean().item() > 0.9999
    assert rel_err(pw[same].cpu().numpy(), pd[same].cpu().numpy()) <= 1e-5
    logits, _, dlogits, dp = ops.fc_xent(pw, p["W3"], p["b3"], y, 1.0 / B)
    gw = ops.conv2_dgrad(dp, cw, p["W2"])
    gd = ops.conv2_dgrad(dp, cw, p["W2"], direct=True)
    num = (gw - gd).abs().flatten(1).max(dim=1).values
    den = gd.abs().flatten(1).max(dim=1).values.clamp_min(1e-30)
    assert (num / den).max().item() <= 1e-5
    sw = ops.reduce_slabs(ops.conv2_wgrad_slabs(act, dp, cw))
    sd = ops.reduce_slabs(ops.conv2_wgrad_slabs(act, dp, cw, direct=True))
    assert rel_err(sw[:18432].cpu().numpy(), sd[:18432].cpu().numpy()) <= 1e-5
    assert rel_err(sw[18432:].cpu().numpy(), sd[18432:].cpu().numpy()) <= 1e-5
    # fc1: loss / dlogits / dW3 / db3 in fp64 from the GPU's pooled features
    flat = pw.double().cpu().numpy().reshape(B, 9216)
    z = flat @ p["W3"].double().cpu().numpy().T + p["b3"].double().cpu().numpy()
    assert rel_err(logits.cpu().numpy(), z) <= 1e-4
    _, _, dz = cross_entropy(z, y.cpu().numpy())
    assert rel_err(dlogits.cpu().numpy(), dz) <= 1e-4
    s3 = ops.reduce_slabs(ops.fc_wgrad_slabs(dlogits, pw)).cpu().numpy()
    assert rel_err(s3[:92160], (dz.T @ flat).reshape(-1)) <= 1e-5
    assert rel_err(s3[92160:], dz.sum(axis=0)) <= 1e-5
    assert rel_err(dp.cpu().numpy().reshape(B, 9216), dz @ p["W3"].double().cpu().numpy()) <= 1e-5
    # client conv1 wgrad (ReLU mask recomputed from x) vs the oracle on the GPU cut gradient
    s1 = ops.reduce_slabs(ops.conv1_wgrad_remask_slabs(x, client.W1.detach(), client.b1.detach(), gw)).cpu().numpy()
    dW1, db1 = client_backward(x.double().cpu().numpy(), act.double().cpu().numpy(), gw.double().cpu().numpy())
    assert rel_err(s1[:288], dW1.reshape(-1)) <= 1e-5
    assert rel_err(s1[288:], db1) <= 1e-5
