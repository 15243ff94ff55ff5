"""The fused server head (slk_fc_xent / slk_fc_xent_amax: fc1 forward, cross-entropy forward + backward,
fc1 input gradient — src/model_def.py:28, src/server_part.py:49-51) against float64 and against the
separate launches (slk_fc_fwd -> slk_fc_dgrad), over ragged batch sizes (a workgroup holds 16 samples)."""
import numpy as np
import pytest
import torch

from conftest import rel_err

pytestmark = pytest.mark.gpu


def _ref64(pooled, W3, b3, y, scale):
    p, W, b = (t.double().cpu().numpy() for t in (pooled, W3, b3))
    z = p.reshape(p.shape[0], -1) @ W.T + b
    m = z.max(axis=1, keepdims=True)
    e = np.exp(z - m)
    sm = e / e.sum(axis=1, keepdims=True)
    yy = y.cpu().numpy()
    loss = (m[:, 0] + np.log(e.sum(axis=1))) - z[np.arange(len(yy)), yy]
    dz = (sm - np.eye(10)[yy]) * scale
    return z, loss, dz, (dz @ W).reshape(pooled.shape)


@pytest.mark.parametrize("B", [1, 7, 15, 16, 17, 33, 100, 4096])
def test_fc_xent_mfma_vs_float64_and_separate_kernels(gpu, B):
    from splitcnn import ops
    g = torch.Generator().manual_seed(B)
    pooled = torch.relu(torch.randn(B, 64, 12, 12, generator=g)).to(gpu)
    W3 = (torch.randn(10, 9216, generator=g) * 0.01).to(gpu)
    b3 = (torch.randn(10, generator=g) * 0.1).to(gpu)
    y = torch.randint(0, 10, (B,), generator=g).to(gpu)
    dpa = torch.empty(B, device=gpu)
    logits, loss_i, dlogits, dp = ops.fc_xent(pooled, W3, b3, y, 1.0 / B, dp_amax=dpa)
    z64, l64, dz64, dp64 = _ref64(pooled, W3, b3, y, 1.0 / B)
    assert rel_err(logits.cpu().numpy(), z64) <= 1e-5
    assert rel_err(loss_i.cpu().numpy(), l64) <= 1e-5
    assert rel_err(dlogits.cpu().numpy(), dz64) <= 1e-5
    assert rel_err(dp.cpu().numpy(), dp64) <= 1e-5
    assert torch.equal(dpa, dp.reshape(B, -1).abs().amax(dim=1))
    # the separate launches run the same per-phase code: bit-identical logits and input gradient
    lg2 = ops.fc_fwd(pooled, W3, b3)
    assert torch.equal(lg2, logits)
    dp2 = ops.fc_dgrad(dlogits, W3)
    assert torch.equal(dp2.reshape(dp.shape), dp)
    # without dp_amax: the same outputs bit for bit
    r2 = ops.fc_xent(pooled, W3, b3, y, 1.0 / B)
    assert all(torch.equal(u, v) for u, v in zip(r2, (logits, loss_i, dlogits, dp)))


def test_fc_xent_bad_label_sets_flag(gpu):
    from splitcnn import ops
    B = 20
    pooled = torch.rand(B, 64, 12, 12, device=gpu)
    W3 = torch.randn(10, 9216, device=gpu) * 0.01
    b3 = torch.zeros(10, device=gpu)
    y = torch.randint(0, 10, (B,), device=gpu)
    y[17] = 10
    flag = torch.zeros(1, dtype=torch.int32, device=gpu)
    _, loss_i, dlogits, _ = ops.fc_xent(pooled, W3, b3, y, 1.0 / B, err_flag=flag)
    assert int(flag.item()) == 1
    assert torch.isnan(loss_i[17]) and torch.isnan(dlogits[17]).all()
    assert torch.isfinite(loss_i[:17]).all() and torch.isfinite(loss_i[18:]).all()



@pytest.mark.parametrize("B", [1, 7, 15, 16, 17, 33, 100, 4096])
def test_split_head_bitwise_vs_fused_head_with_amax(gpu, B):
    """The server's default split head (engine.ServerStage.fc_split: slk_fc_fwd -> slk_xent_fwd_bwd ->
    slk_fc_dgrad_amax) against the fused slk_fc_xent_amax: every output bit-identical, dp_amax included."""
    from splitcnn import ops
    g = torch.Generator().manual_seed(1000 + B)
    pooled = torch.relu(torch.randn(B, 64, 12, 12, generator=g)).to(gpu)
    W3 = (torch.randn(10, 9216, generator=g) * 0.01).to(gpu)
    b3 = (torch.randn(10, generator=g) * 0.1).to(gpu)
    y = torch.randint(0, 10, (B,), generator=g).to(gpu)
    dpa = torch.empty(B, device=gpu)
    logits, loss_i, dlogits, dp = ops.fc_xent(pooled, W3, b3, y, 1.0 / B, dp_amax=dpa)
    lg2 = ops.fc_fwd(pooled, W3, b3)
    l2, dl2 = ops.xent_fwd_bwd(lg2, y, 1.0 / B)
    dpa2 = torch.full((B,), float("nan"), device=gpu)
    dp2 = ops.fc_dgrad(dl2, W3, dp_amax=dpa2)
    assert torch.equal(lg2, logits)
    assert torch.equal(l2, loss_i)
    assert torch.equal(dl2, dlogits)
    assert torch.equal(dp2.reshape(dp.shape), dp)
    assert torch.equal(dpa2, dpa)
    # the step's launch (round 6): logits + cross-entropy in one kernel, bitwise the two launches
    lg3, l3, dl3 = ops.fc_logits_xent(pooled, W3, b3, y, 1.0 / B)
    assert torch.equal(lg3, logits) and torch.equal(l3, loss_i) and torch.equal(dl3, dlogits)


def test_fc_logits_xent_bad_label_sets_flag(gpu):
    from splitcnn import ops
    B = 20
    pooled = torch.rand(B, 64, 12, 12, device=gpu)
    W3 = torch.randn(10, 9216, device=gpu) * 0.01
    b3 = torch.zeros(10, device=gpu)
    y = torch.randint(0, 10, (B,), device=gpu)
    y[7] = 10
    flag = torch.zeros(1, dtype=torch.int32, device=gpu)
    _, loss_i, dlogits = ops.fc_logits_xent(pooled, W3, b3, y, 1.0 / B, err_flag=flag)
    assert int(flag.item()) == 1
    assert torch.isnan(loss_i[7]) and torch.isnan(dlogits[7]).all()
    assert torch.isfinite(loss_i[:7]).all() and torch.isfinite(dlogits[8:]).all()


@pytest.mark.parametrize("B", [17, 4096])
def test_server_stage_split_head_bitwise_vs_fused_head(gpu, B):
    """ServerStage.forward_backward with fc_split True (default) and False: the same cut gradient,
    conv2 slabs (s2) and fc1 slabs (s3), bit for bit (src/server_part.py:48-51)."""
    from splitcnn.data import SyntheticMNIST, init_models
    from splitcnn.engine import ClientStage, ServerStage
    a, b = init_models(seed=0)
    cl = ClientStage(a, device=gpu)
    cl.emit_amax = True
    x, y = SyntheticMNIST(5).batch(B)
    x, y = x.to(gpu), y.to(gpu)
    act = cl.forward(x)
    outs = []
    for split in (True, False):
        s = ServerStage(init_models(seed=0)[1], device=gpu)
        s.fc_split = split
        cut, loss_i, s2, s3 = s.forward_backward(act, y, 1.0 / B, act_amax=cl._act_amax)
        outs.append([t.clone() for t in (cut, loss_i, s2, s3)])
    for u, v, name in zip(outs[0], outs[1], ("cut_grad", "loss_i", "s2", "s3")):
        assert torch.equal(u, v), name
