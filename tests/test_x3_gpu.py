"""GPU: the "x3" conv2 kernels (direct implicit GEMM on the f16 MFMA with hi/lo-split operands,
csrc/slk_x3.hip) against the fp64 oracle and against the f32-MFMA kernels on identical inputs.

Tolerances: the same bars as the Winograd path (tests/test_wino_gpu.py): 1e-5 of max |ref|, routing
differences only at numerical ties of the fp64 conv output. The x3 error is also compared with the
f32 Winograd path's own error against fp64 (it must not be worse by more than 2x: an fp32-grade path,
not a reduced-precision one)."""
import numpy as np
import pytest
import torch

from conftest import rel_err
from ref64 import assert_routing_ties, conv_relu64, dgrad64, route64, wgrad64

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


def test_row_amax(gpu):
    from splitcnn import ops
    x = torch.randn(37, 21632, device=gpu) * torch.logspace(-8, 8, 37, device=gpu)[:, None]
    x[3] = 0
    x[5, 7] = float("nan")
    got = ops.row_amax(x).cpu()
    want = torch.nan_to_num(x.cpu(), nan=0.0).abs().amax(dim=1)
    assert torch.equal(got, want)
    odd = torch.randn(5, 33, device=gpu)
    assert torch.equal(ops.row_amax(odd).cpu(), odd.cpu().abs().amax(dim=1))


@pytest.mark.parametrize("B", [1, 5, 64, 130, 777])
def test_x3_fwd_matches_oracle(gpu, B):
    from oracle.split_step import conv3x3, relu, tie_discrepancies
    from splitcnn import ops
    act, p, _ = _inputs(gpu, B, seed=B)
    px, cx = ops.conv2_fwd_pool(act, p["W2"], p["b2"], impl="x3")
    pw, cw = ops.conv2_fwd_pool(act, p["W2"], p["b2"])
    a64 = act.double().cpu().numpy()
    r = relu(conv3x3(a64, p["W2"].double().cpu().numpy(), p["b2"].double().cpu().numpy()))
    pr = r.reshape(B, 64, 12, 2, 12, 2).max(axis=(3, 5))
    n, ok = tie_discrepancies(r, cw.cpu().numpy().astype(np.int64), cx.cpu().numpy().astype(np.int64))
    assert ok, f"{n} routing differences that are not ties"
    ex = rel_err(px.cpu().numpy(), pr)
    ew = rel_err(pw.cpu().numpy(), pr)
    assert ex <= 1e-5
    assert ex <= max(2 * ew, 1e-6), (ex, ew)


def test_x3_fwd_scale_invariance(gpu):
    """Per-sample power-of-two scales: scaling one sample's act by 2^k (exact) scales its pooled output
    by 2^k bit for bit (bias 0), whatever the other samples hold — incl. magnitudes far outside f16."""
    from splitcnn import ops
    B = 6
    act, p, _ = _inputs(gpu, B, seed=9)
    b0 = torch.zeros_like(p["b2"])
    base, cb = ops.conv2_fwd_pool(act, p["W2"], b0, impl="x3")
    k = torch.tensor([0, -40, 30, 0, 60, -100], device=gpu, dtype=torch.float32)
    sc = torch.pow(2.0, k)
    out, co = ops.conv2_fwd_pool(act * sc[:, None, None, None], p["W2"], b0, impl="x3")
    assert torch.equal(co, cb)
    assert torch.equal(out, base * sc[:, None, None, None])
    # weights scaled by 2^k: the launch scale absorbs it
    out2, _ = ops.conv2_fwd_pool(act, p["W2"] * 2.0 ** -30, b0, impl="x3")
    assert torch.equal(out2, base * 2.0 ** -30)


def test_x3_fwd_deterministic_and_full_size(gpu):
    from splitcnn import ops
    B = 4096
    act, p, _ = _inputs(gpu, B, seed=21)
    r1 = ops.conv2_fwd_pool(act, p["W2"], p["b2"], impl="x3")
    r2 = ops.conv2_fwd_pool(act, p["W2"], p["b2"], impl="x3")
    assert torch.equal(r1[0], r2[0]) and torch.equal(r1[1], r2[1])
    pd, cd = ops.conv2_fwd_pool(act, p["W2"], p["b2"], impl="direct")
    # every window whose routing differs from float64's is a numerical tie (all 37.7 M windows checked)
    assert_routing_ties(act, p["W2"], p["b2"], r1[1])
    assert_routing_ties(act, p["W2"], p["b2"], cd)
    assert rel_err(r1[0].cpu().numpy(), pd.cpu().numpy()) <= 1e-5


@pytest.mark.parametrize("B", [1, 5, 64, 130, 777])
def test_x3_dgrad_matches_oracle(gpu, B):
    from oracle.split_step import conv3x3_dgrad, maxpool2_bwd
    from splitcnn import ops
    act, p, y = _inputs(gpu, B, seed=B + 100)
    pw, cw = ops.conv2_fwd_pool(act, p["W2"], p["b2"])
    _, _, _, dp = ops.fc_xent(pw, p["W3"], p["b3"], y, 1.0 / B)
    gx = ops.conv2_dgrad(dp, cw, p["W2"], impl="x3")
    gw = ops.conv2_dgrad(dp, cw, p["W2"])
    codes = cw.cpu().numpy().astype(np.int64)
    dp64 = dp.double().cpu().numpy().reshape(B, 64, 12, 12)
    dc = maxpool2_bwd(np.where(codes < 4, dp64, 0.0), np.minimum(codes, 3), (B, 64, 24, 24))
    ref = conv3x3_dgrad(dc, p["W2"].double().cpu().numpy())
    ex = rel_err(gx.cpu().numpy(), ref)
    ew = rel_err(gw.cpu().numpy(), ref)
    assert ex <= 1e-5
    assert ex <= max(2 * ew, 1e-6), (ex, ew)
    # every sample on its own (a misrouted unit would hit one sample)
    g64 = torch.from_numpy(ref)
    num = (gx.cpu().double() - g64).abs().flatten(1).max(dim=1).values
    den = g64.abs().flatten(1).max(dim=1).values.clamp_min(1e-30)
    assert (num / den).max().item() <= 1e-5


def test_x3_dgrad_scale_invariance(gpu):
    from splitcnn import ops
    B = 6
    act, p, y = _inputs(gpu, B, seed=19)
    pw, cw = ops.conv2_fwd_pool(act, p["W2"], p["b2"])
    _, _, _, dp = ops.fc_xent(pw, p["W3"], p["b3"], y, 1.0 / B)
    base = ops.conv2_dgrad(dp, cw, p["W2"], impl="x3")
    sc = torch.pow(2.0, torch.tensor([0, -40, 30, 0, 60, -90], device=gpu, dtype=torch.float32))
    out = ops.conv2_dgrad((dp.reshape(B, -1) * sc[:, None]).reshape(dp.shape).contiguous(), cw, p["W2"], impl="x3")
    assert torch.equal(out, base * sc[:, None, None, None])


@pytest.mark.parametrize("B", [1, 5, 64, 130, 777])
def test_x3_wgrad_matches_oracle(gpu, B):
    from oracle.split_step import conv3x3_wgrad, maxpool2_bwd
    from splitcnn import ops
    act, p, y = _inputs(gpu, B, seed=B + 200)
    pw, cw = ops.conv2_fwd_pool(act, p["W2"], p["b2"])
    _, _, _, dp = ops.fc_xent(pw, p["W3"], p["b3"], y, 1.0 / B)
    assert ops.conv2_wgrad_nslab(B, impl="x3") == min(6 * B, 256)
    sx = ops.reduce_slabs(ops.conv2_wgrad_slabs(act, dp, cw, impl="x3")).cpu().numpy()
    sw = ops.reduce_slabs(ops.conv2_wgrad_slabs(act, dp, cw)).cpu().numpy()
    codes = cw.cpu().numpy().astype(np.int64)
    dp64 = dp.double().cpu().numpy().reshape(B, 64, 12, 12)
    dc = maxpool2_bwd(np.where(codes < 4, dp64, 0.0), np.minimum(codes, 3), (B, 64, 24, 24))
    dW, db = conv3x3_wgrad(act.double().cpu().numpy(), dc)
    for got, w, ref in ((sx[:18432], sw[:18432], dW.reshape(-1)), (sx[18432:], sw[18432:], db)):
        ex, ew = rel_err(got, ref), rel_err(w, ref)
        assert ex <= 1e-5
        assert ex <= max(2 * ew, 1e-6), (ex, ew)


def test_x3_wgrad_deterministic(gpu):
    from splitcnn import ops
    B = 300
    act, p, y = _inputs(gpu, B, seed=3)
    pw, cw = ops.conv2_fwd_pool(act, p["W2"], p["b2"])
    _, _, _, dp = ops.fc_xent(pw, p["W3"], p["b3"], y, 1.0 / B)
    a = ops.conv2_wgrad_slabs(act, dp, cw, impl="x3").clone()
    b = ops.conv2_wgrad_slabs(act, dp, cw, impl="x3")
    assert torch.equal(a, b)


def test_fused_amax_outputs(gpu):
    """conv1_fwd's act_amax is the cut's x3 scale value, the bound max_c (sum_k |W1[c,k]| max|x| + b1[c]+)
    (round 5: conv1_cut_bound, the same as slk_conv1_fwd_x3 emits), never below the cut's max; fc_xent's
    dp_amax equals row_amax of dpooled (exact: a max)."""
    from splitcnn import ops
    from splitcnn.data import SyntheticMNIST, init_models
    B = 37
    a, b = init_models(seed=4)
    x, y = SyntheticMNIST(5).batch(B)
    x, y = x.to(gpu), y.to(gpu)
    W1, b1 = a.conv1.weight.detach().to(gpu), a.conv1.bias.detach().to(gpu)
    am = torch.empty(B, device=gpu)
    act = ops.conv1_fwd(x, W1, b1, act_amax=am)
    assert torch.equal(act, ops.conv1_fwd(x, W1, b1))
    true_max = ops.row_amax(act)
    assert bool((am >= true_max).all())
    xm = x.reshape(B, -1).abs().amax(dim=1).double().cpu().numpy()
    w = W1.reshape(32, 9).abs().double().sum(dim=1).cpu().numpy()
    bound = (w[None, :] * xm[:, None] + np.maximum(b1.double().cpu().numpy(), 0.0)[None, :]).max(axis=1)
    assert rel_err(am.cpu().numpy(), bound) <= 1e-6
    am_x3 = torch.empty(B, device=gpu)
    ops.conv1_fwd_x3(x, W1, b1, am_x3, torch.empty(ops.conv2_act16_bytes(B), dtype=torch.uint8, device=gpu))
    assert torch.equal(am_x3, am)   # the two client kernels emit the same value
    W2, b2 = b.conv2.weight.detach().to(gpu), b.conv2.bias.detach().to(gpu)
    W3, b3 = b.fc1.weight.detach().to(gpu), b.fc1.bias.detach().to(gpu)
    pooled, code = ops.conv2_fwd_pool(act, W2, b2)
    dpa = torch.empty(B, device=gpu)
    r1 = ops.fc_xent(pooled, W3, b3, y, 1.0 / B, dp_amax=dpa)
    r2 = ops.fc_xent(pooled, W3, b3, y, 1.0 / B)
    for u, v in zip(r1, r2):
        assert torch.equal(u, v)
    assert torch.equal(dpa, ops.row_amax(r1[3]))


@pytest.mark.parametrize("conv", ["f32", "x3"])
def test_trainer_conv_presets_match_fixture(gpu, conv):
    """One fused SplitTrainer step (conv1 emitting the cut's amax for x3) per conv preset against the
    reference fixture: post-step weights at the fixture bars (conftest.weight_ok)."""
    from conftest import PARAMS, load_fixture, weight_ok
    from splitcnn.engine import SplitTrainer
    from test_gpu_parity import make_models, param_of
    for name in ("split_step_b4.npz", "split_step_b13.npz"):
        fx = load_fixture(name)
        a, b = make_models(fx)
        tr = SplitTrainer(a, b, device=gpu, graph=False, conv=conv)
        assert tr.client.emit_amax == (conv == "x3")
        tr.step(torch.from_numpy(fx["x_1"]).to(gpu), torch.from_numpy(fx["y_1"]).to(gpu))
        for k in PARAMS:
            assert weight_ok(param_of(tr.client, tr.server, k), fx[f"post_{k}_1"], fx[f"init_{k}"]), (name, k)


@pytest.mark.parametrize("B", [1, 7, 300])
def test_x3_wgrad_from_forward_images_bitwise(gpu, B):
    """The forward's split input images (act16) fed to the wgrad by LDS-DMA give the weight gradient of
    the wgrad that loads and splits act itself (same per-sample scales, same f16 values; since round 5 the
    images kernel owns both co halves per workgroup over 4-row units, so the two differ only in summation
    order: 2e-6 of max |ref|); the forward in that mode is the plain x3 forward bit for bit and meets the
    oracle bar."""
    from oracle.split_step import conv3x3, relu, tie_discrepancies
    from splitcnn import ops
    act, p, y = _inputs(gpu, B, seed=B + 300)
    am = ops.row_amax(act)
    a16 = torch.empty(ops.conv2_act16_bytes(B), dtype=torch.uint8, device=gpu)
    ps, cs = ops.conv2_fwd_pool(act, p["W2"], p["b2"], impl="x3", act_amax=am, act16=a16)
    _, _, _, dp = ops.fc_xent(ps, p["W3"], p["b3"], y, 1.0 / B)
    s1 = ops.conv2_wgrad_slabs(act, dp, cs, impl="x3", act_amax=am)
    s2 = ops.conv2_wgrad_slabs(act, dp, cs, impl="x3", act_amax=am, act16=a16)
    assert s1.shape == s2.shape == (min(6 * B, 256), ops.CONV2_SLAB)
    g1, g2 = (ops.reduce_slabs(s).double().cpu().numpy() for s in (s1, s2))
    assert rel_err(g2, g1) <= 2e-6
    px, cx = ops.conv2_fwd_pool(act, p["W2"], p["b2"], impl="x3", act_amax=am)
    assert torch.equal(px, ps) and torch.equal(cx, cs)
    r = relu(conv3x3(act.double().cpu().numpy(), p["W2"].double().cpu().numpy(), p["b2"].double().cpu().numpy()))
    pw, cw = ops.conv2_fwd_pool(act, p["W2"], p["b2"])
    n, ok = tie_discrepancies(r, cw.cpu().numpy().astype(np.int64), cs.cpu().numpy().astype(np.int64))
    assert ok, n
    assert rel_err(ps.cpu().numpy(), r.reshape(B, 64, 12, 2, 12, 2).max(axis=(3, 5))) <= 1e-5


@pytest.mark.parametrize("B", [1, 2, 4, 300, 513, 4096])
def test_x3_fwd_with_in_kernel_amax_bitwise(gpu, B):
    """slk_conv2_fwd_pool_x3sa (the drop-in module forward: the per-sample max |act| computed inside the
    forward, whole samples per workgroup, chunks of the next sample read ahead) == row_amax + the x3
    forward writing act16: amax, pooled, code and every act16 byte. B = 1, 2, 4: one sample per
    workgroup (no read-ahead); 300, 513: ragged ranges (2-3 samples on some workgroups, none on others);
    4096: 16 samples per workgroup. One sample carries a NaN (ignored by both maxima) and one is zero."""
    from splitcnn import ops
    act, p, _ = _inputs(gpu, B, seed=B + 77)
    act[B // 2] *= 2.0 ** -20
    if B > 2:
        act[1] = 0.0
        act[2, 5, 3, 4] = float("nan")
    am = ops.row_amax(act)
    nb = ops.conv2_act16_bytes(B)
    i0 = torch.empty(nb, dtype=torch.uint8, device=gpu)
    p0, c0 = ops.conv2_fwd_pool(act, p["W2"], p["b2"], impl="x3", act_amax=am, act16=i0)
    am1 = torch.full((B,), -1.0, device=gpu)
    i1 = torch.full((nb,), 0x5A, dtype=torch.uint8, device=gpu)
    p1, c1 = ops.conv2_fwd_pool(act, p["W2"], p["b2"], impl="x3", act16=i1, act_amax_out=am1)
    torch.cuda.synchronize()
    assert torch.equal(am1, am)
    assert torch.equal(c1, c0)
    assert torch.equal(p1.view(torch.int32), p0.view(torch.int32))
    assert torch.equal(i1, i0)


@pytest.mark.parametrize("B", [1, 6, 257])
def test_conv1_x3_images_and_forward_from_images_bitwise(gpu, B):
    """slk_conv1_fwd_x3 writes the same f32 act and act_amax as conv1_fwd(act_amax=...), and the same
    act16 images as the x3 forward does from that act (bitwise, every byte); the forward reading those
    images (slk_conv2_fwd_pool_x3i) gives the x3 forward's pooled / code bit for bit, and the wgrad
    reading them the same slabs."""
    from splitcnn import ops
    from splitcnn.data import SyntheticMNIST, init_models
    a, b = init_models(seed=B + 11)
    x, y = SyntheticMNIST(B + 12).batch(B)
    x, y = x.to(gpu), y.to(gpu)
    W1, b1 = a.conv1.weight.detach().to(gpu), a.conv1.bias.detach().to(gpu)
    W2, b2 = b.conv2.weight.detach().to(gpu), b.conv2.bias.detach().to(gpu)
    W3, b3 = b.fc1.weight.detach().to(gpu), b.fc1.bias.detach().to(gpu)
    am0 = torch.empty(B, device=gpu)
    act0 = ops.conv1_fwd(x, W1, b1, act_amax=am0)
    nb = ops.conv2_act16_bytes(B)
    am1, i1 = torch.empty(B, device=gpu), torch.full((nb,), 7, dtype=torch.uint8, device=gpu)
    act1 = ops.conv1_fwd_x3(x, W1, b1, am1, i1, act=torch.empty_like(act0))
    am2, i2 = torch.empty(B, device=gpu), torch.full((nb,), 9, dtype=torch.uint8, device=gpu)
    bits = torch.full((B, ops.RELU_BITS_WORDS), -1, dtype=torch.int32, device=gpu)
    assert ops.conv1_fwd_x3(x, W1, b1, am2, i2, relu_bits=bits) is None
    assert torch.equal(act1, act0) and torch.equal(am1, am0) and torch.equal(am2, am0)
    # the ReLU bit map is exactly act > 0 (every bit; the padding bits past pixel 675 are zero)
    assert np.array_equal(_decode_bits(bits), (act0 > 0).reshape(B, 32, 676).cpu().numpy())
    i0 = torch.empty(nb, dtype=torch.uint8, device=gpu)
    p0, c0 = ops.conv2_fwd_pool(act0, W2, b2, impl="x3", act_amax=am0, act16=i0)
    assert torch.equal(i1, i0) and torch.equal(i2, i0)
    p1, c1 = ops.conv2_fwd_pool_x3i(i2, am2, W2, b2)
    assert torch.equal(p1, p0) and torch.equal(c1, c0)
    _, _, _, dp = ops.fc_xent(p0, W3, b3, y, 1.0 / B)
    s0 = ops.conv2_wgrad_slabs(act0, dp, c0, impl="x3", act_amax=am0)
    s1 = ops.conv2_wgrad_slabs(None, dp, c0, impl="x3", act_amax=am2, act16=i2)
    s1b = ops.conv2_wgrad_slabs(None, dp, c0, impl="x3", act_amax=am0, act16=i0)
    assert torch.equal(s1, s1b)   # the same images -> the same slabs, bit for bit
    # the f32-act kernel sums in another order (test_x3_wgrad_from_forward_images_bitwise)
    g0, g1 = (ops.reduce_slabs(s).double().cpu().numpy() for s in (s0, s1))
    assert rel_err(g1, g0) <= 2e-6


def test_trainer_client_images_bitwise(gpu):
    """SplitTrainer with the client writing the x3 images (no f32 cut) and with the f32 cut + the
    forward writing them: identical parameters and losses after three steps, bit for bit (both with the
    separate client backward: the fused one needs the client's images and bit map)."""
    from splitcnn.data import SyntheticMNIST, init_models
    from splitcnn.engine import SplitTrainer
    out = []
    for img in (True, False):
        a, b = init_models(seed=21)
        tr = SplitTrainer(a, b, device=gpu, graph=True, conv="x3", act16=img, fuse_client_backward=False)
        assert tr.client.emit_act16 == img
        data = SyntheticMNIST(22)
        for _ in range(3):
            x, y = data.batch(96)
            tr.step(x.to(gpu), y.to(gpu))
        torch.cuda.synchronize()
        out.append((tr.client.params.clone(), tr.server.params.clone(), tr.loss_log.flush()))
    assert torch.equal(out[0][0], out[1][0]) and torch.equal(out[0][1], out[1][1])
    assert out[0][2] == out[1][2] and len(out[0][2]) == 3


@pytest.mark.parametrize("B", [1, 5, 130])
def test_dgrad_with_fused_client_backward(gpu, B):
    """slk_conv2_dgrad_x3_c1w: the client's gradient from the fused dgrad equals the separate path
    (x3 dgrad -> cut gradient -> conv1_wgrad_remask) up to summation order (1e-5 of max |ref|), and the
    fp64 oracle at the same bar."""
    from splitcnn import ops
    from splitcnn.data import SyntheticMNIST, init_models
    a, b = init_models(seed=B + 40)
    x, y = SyntheticMNIST(B + 41).batch(B)
    x, y = x.to(gpu), y.to(gpu)
    W1, b1 = a.conv1.weight.detach().to(gpu), a.conv1.bias.detach().to(gpu)
    W2, b2 = b.conv2.weight.detach().to(gpu), b.conv2.bias.detach().to(gpu)
    W3, b3 = b.fc1.weight.detach().to(gpu), b.fc1.bias.detach().to(gpu)
    act = ops.conv1_fwd(x, W1, b1)
    pooled, code = ops.conv2_fwd_pool(act, W2, b2, impl="x3")
    dpa = torch.empty(B, device=gpu)
    _, _, _, dp = ops.fc_xent(pooled, W3, b3, y, 1.0 / B, dp_amax=dpa)
    slabs = ops.conv2_dgrad_client_slabs(dp, code, W2, x, _relu_bits(x, W1, b1), dp_amax=dpa)
    assert slabs.shape == (min(3 * B, 256), 320)
    fused = ops.reduce_slabs(slabs).cpu().numpy()
    g = ops.conv2_dgrad(dp, code, W2, impl="x3", dp_amax=dpa)
    sep = ops.reduce_slabs(ops.conv1_wgrad_remask_slabs(x, W1, b1, g)).cpu().numpy()
    ref = _c1_ref64(x, W1, b1, g)
    for sl in (slice(0, 288), slice(288, 320)):
        assert rel_err(fused[sl], sep[sl]) <= 1e-5
        assert rel_err(fused[sl], ref[sl]) <= 1e-5


def _relu_bits(x, W1, b1):
    """The cut's ReLU bit map as the fused step gets it (conv1_fwd_x3 writes it next to the images)."""
    from splitcnn import ops
    B = x.shape[0]
    bits = ops.relu_bits_buffer(B, x.device)
    ops.conv1_fwd_x3(x, W1, b1, torch.empty(B, device=x.device),
                     torch.empty(ops.conv2_act16_bytes(B), dtype=torch.uint8, device=x.device), relu_bits=bits)
    return bits


def _decode_bits(bits):
    """[B, 676] int32 -> bool [B, 32, 676]: bit 4 (c & 7) + u of word (c >> 3, t) = pixel 4 t + u of channel c."""
    w = bits.cpu().numpy().view(np.uint32).reshape(-1, 4, 169)
    c = np.arange(32)
    sh = (4 * (c & 7))[:, None, None] + np.arange(4)[None, None, :]          # c, 1, u
    b = (w[:, c >> 3, :, None] >> sh[None].astype(np.uint32)) & 1            # B, c, t, u
    return b.reshape(-1, 32, 676).astype(bool)


def _c1_ref64(x, W1, b1, g):
    """fp64 ReLU backward + conv1 weight/bias gradient (the oracle's conv1 restated at the test)."""
    x, W1, b1, g = (t.double().cpu().numpy() for t in (x, W1, b1, g))
    B = x.shape[0]
    win = np.stack([x[:, 0, ky:ky + 26, kx:kx + 26] for ky in range(3) for kx in range(3)], axis=1)  # B,9,26,26
    s = np.einsum("bkyx,ck->bcyx", win, W1.reshape(32, 9)) + b1[None, :, None, None]
    gm = np.where(s > 0, g, 0.0)
    dW = np.einsum("bcyx,bkyx->ck", gm, win)
    return np.concatenate([dW.reshape(-1), gm.sum(axis=(0, 2, 3))])


def test_trainer_fused_client_backward_matches_unfused(gpu):
    """SplitTrainer with the client's backward fused into the x3 dgrad vs the separate cut-gradient path:
    the parameter updates of three steps agree to summation-order differences (1e-3 of the largest
    update; a wrong gradient would be off by the update's own size)."""
    from splitcnn.data import SyntheticMNIST, init_models
    from splitcnn.engine import SplitTrainer
    out = []
    for fuse in (True, False):
        a, b = init_models(seed=31)
        tr = SplitTrainer(a, b, device=gpu, graph=True, conv="x3", fuse_client_backward=fuse)
        init = (tr.client.params.cpu().numpy().copy(), tr.server.params.cpu().numpy().copy())
        assert tr.fuse_client_backward == fuse
        data = SyntheticMNIST(32)
        for _ in range(3):
            x, y = data.batch(200)
            tr.step(x.to(gpu), y.to(gpu))
        torch.cuda.synchronize()
        out.append((tr.client.params.cpu().numpy() - init[0], tr.server.params.cpu().numpy() - init[1]))
    for u, v in zip(out[0], out[1]):
        assert np.abs(u - v).max() <= 1e-3 * np.abs(v).max(), (np.abs(u - v).max(), np.abs(v).max())


def test_x3_zero_samples(gpu):
    """A sample whose cut is all zeros (amax 0) and one whose pooled gradient is all zeros: every x3
    kernel stays finite and on the oracle bar (the wgrad's dY compensation must not scale by the zero
    sample's exponent)."""
    from oracle.split_step import conv3x3_wgrad, maxpool2_bwd
    from splitcnn import ops
    B = 6
    act, p, y = _inputs(gpu, B, seed=77)
    act[2] = 0
    am = ops.row_amax(act)
    assert float(am[2]) == 0.0
    a16 = torch.empty(ops.conv2_act16_bytes(B), dtype=torch.uint8, device=gpu)
    ps, cs = ops.conv2_fwd_pool(act, p["W2"], p["b2"], impl="x3", act_amax=am, act16=a16)
    _, _, _, dp = ops.fc_xent(ps, p["W3"], p["b3"], y, 1.0 / B)
    dp[4] = 0
    dpa = ops.row_amax(dp)
    for s in (ops.conv2_wgrad_slabs(act, dp, cs, impl="x3", act_amax=am, dp_amax=dpa),
              ops.conv2_wgrad_slabs(None, dp, cs, impl="x3", act_amax=am, dp_amax=dpa, act16=a16)):
        got = ops.reduce_slabs(s).cpu().numpy()
        assert np.isfinite(got).all()
        codes = cs.cpu().numpy().astype(np.int64)
        dp64 = dp.double().cpu().numpy().reshape(B, 64, 12, 12)
        dc = maxpool2_bwd(np.where(codes < 4, dp64, 0.0), np.minimum(codes, 3), (B, 64, 24, 24))
        dW, db = conv3x3_wgrad(act.double().cpu().numpy(), dc)
        assert rel_err(got[:18432], dW.reshape(-1)) <= 1e-5 and rel_err(got[18432:], db) <= 1e-5
    g = ops.conv2_dgrad(dp, cs, p["W2"], impl="x3", dp_amax=dpa)
    assert torch.isfinite(g).all() and float(g[4].abs().max()) == 0.0


def test_default_fused_path_full_size_vs_direct_f32(gpu):
    """K2 size (B = 4096: every persistent x3 workgroup runs its full unit stream): the default step's
    kernels — conv1 images, forward from images, fused dgrad + client backward, wgrad from images —
    against the independent direct f32-MFMA kernels on the same inputs (themselves checked vs fp64 in
    test_wino_gpu.py): 1e-5 of max |ref|, every window where either path's routing differs from the float64
    conv's a numerical tie (checked per window). Run twice: bit-identical (fixed summation orders)."""
    from splitcnn import ops
    from splitcnn.data import SyntheticMNIST, init_models
    B = 4096
    a, b = init_models(seed=51)
    x, y = SyntheticMNIST(52).batch(B)
    x, y = x.to(gpu), y.to(gpu)
    W1, b1 = a.conv1.weight.detach().to(gpu), a.conv1.bias.detach().to(gpu)
    W2, b2 = b.conv2.weight.detach().to(gpu), b.conv2.bias.detach().to(gpu)
    W3, b3 = b.fc1.weight.detach().to(gpu), b.fc1.bias.detach().to(gpu)

    def fused():
        am = torch.empty(B, device=gpu)
        img = torch.empty(ops.conv2_act16_bytes(B), dtype=torch.uint8, device=gpu)
        ops.conv1_fwd_x3(x, W1, b1, am, img)
        pooled, code = ops.conv2_fwd_pool_x3i(img, am, W2, b2)
        dpa = torch.empty(B, device=gpu)
        _, _, _, dp = ops.fc_xent(pooled, W3, b3, y, 1.0 / B, dp_amax=dpa)
        c1 = ops.reduce_slabs(ops.conv2_dgrad_client_slabs(dp, code, W2, x, _relu_bits(x, W1, b1), dp_amax=dpa))
        s2 = ops.reduce_slabs(ops.conv2_wgrad_slabs(None, dp, code, impl="x3", act_amax=am, dp_amax=dpa, act16=img))
        return pooled, code, dp, c1, s2

    r1, r2 = fused(), fused()
    for u, v in zip(r1, r2):
        assert torch.equal(u, v)
    pooled, code, dp, c1, s2 = r1
    act = ops.conv1_fwd(x, W1, b1)
    pd, cd = ops.conv2_fwd_pool(act, W2, b2, impl="direct")
    assert_routing_ties(act, W2, b2, code)
    assert_routing_ties(act, W2, b2, cd)
    assert rel_err(pooled.cpu().numpy(), pd.cpu().numpy()) <= 1e-5
    # backward references on the SAME routing (the x3 forward's code) through the f32 direct kernels
    g = ops.conv2_dgrad(dp, code, W2, impl="direct")
    c1ref = ops.reduce_slabs(ops.conv1_wgrad_remask_slabs(x, W1, b1, g)).cpu().numpy()
    s2ref = ops.reduce_slabs(ops.conv2_wgrad_slabs(act, dp, code, impl="direct")).cpu().numpy()
    c1, s2 = c1.cpu().numpy(), s2.cpu().numpy()
    for got, ref in ((c1[:288], c1ref[:288]), (c1[288:], c1ref[288:]), (s2[:18432], s2ref[:18432]), (s2[18432:], s2ref[18432:])):
        assert rel_err(got, ref) <= 1e-5, rel_err(got, ref)


def test_full_size_x3_error_within_2x_of_f32(gpu):
    """B = 4096 (the K2 batch, src/server_part.py:47-52 at that size): every x3 conv2 output's error
    against float64 is at most 2x the direct f32-MFMA kernel's own error on the same inputs — forward
    (pooled), cut gradient, dW2 / db2 and the fused client gradient (dW1 / db1, src/client_part.py:132)
    — and within 1e-5 of max |ref|. Backward references use the x3 forward's routing (its differences
    from float64 are ties: assert_routing_ties)."""
    from splitcnn import ops
    from splitcnn.data import SyntheticMNIST, init_models
    B = 4096
    a, b = init_models(seed=61)
    x, y = SyntheticMNIST(62).batch(B)
    x, y = x.to(gpu), y.to(gpu)
    W1, b1 = a.conv1.weight.detach().to(gpu), a.conv1.bias.detach().to(gpu)
    W2, b2 = b.conv2.weight.detach().to(gpu), b.conv2.bias.detach().to(gpu)
    W3, b3 = b.fc1.weight.detach().to(gpu), b.fc1.bias.detach().to(gpu)
    am = torch.empty(B, device=gpu)
    act = ops.conv1_fwd(x, W1, b1, act_amax=am)
    img = torch.empty(ops.conv2_act16_bytes(B), dtype=torch.uint8, device=gpu)
    ops.conv1_fwd_x3(x, W1, b1, torch.empty(B, device=gpu), img)
    px, cx = ops.conv2_fwd_pool_x3i(img, am, W2, b2)
    pd, cd = ops.conv2_fwd_pool(act, W2, b2, impl="direct")
    r64 = conv_relu64(act, W2, b2)
    p64 = r64.reshape(B, 64, 12, 2, 12, 2).amax(dim=(3, 5))
    assert_routing_ties(act, W2, b2, cx)

    def errs(got_x3, got_f32, ref):
        ref = ref.double()
        sc = ref.abs().max().item()
        ex = (got_x3.double() - ref).abs().max().item() / sc
        ew = (got_f32.double() - ref).abs().max().item() / sc
        return ex, ew
    checks = {"pooled": errs(px, pd, p64)}
    dpa = torch.empty(B, device=gpu)
    _, _, _, dp = ops.fc_xent(px, W3, b3, y, 1.0 / B, dp_amax=dpa)
    dc = route64(dp, cx)
    g64 = dgrad64(dc, W2)
    checks["cut_grad"] = errs(ops.conv2_dgrad(dp, cx, W2, impl="x3", dp_amax=dpa),
                              ops.conv2_dgrad(dp, cx, W2, impl="direct"), g64)
    sx = ops.reduce_slabs(ops.conv2_wgrad_slabs(None, dp, cx, impl="x3", act_amax=am, dp_amax=dpa, act16=img))
    sd = ops.reduce_slabs(ops.conv2_wgrad_slabs(act, dp, cx, impl="direct"))
    dW64, db64 = wgrad64(act, dc)
    checks["dW2"] = errs(sx[:18432], sd[:18432], dW64.reshape(-1))
    checks["db2"] = errs(sx[18432:], sd[18432:], db64)
    c1x = ops.reduce_slabs(ops.conv2_dgrad_client_slabs(dp, cx, W2, x, _relu_bits(x, W1, b1), dp_amax=dpa))
    c1d = ops.reduce_slabs(ops.conv1_wgrad_remask_slabs(x, W1, b1, ops.conv2_dgrad(dp, cx, W2, impl="direct")))
    c164 = torch.from_numpy(_c1_ref64(x, W1, b1, g64)).to(gpu)
    checks["dW1"] = errs(c1x[:288], c1d[:288], c164[:288])
    checks["db1"] = errs(c1x[288:], c1d[288:], c164[288:])
    for k, (ex, ew) in checks.items():
        assert ex <= 1e-5, (k, ex, ew)
        assert ex <= max(2 * ew, 1e-6), (k, ex, ew)


@pytest.mark.parametrize("tiny", [1e-38, 1e-44])
def test_x3_tiny_sample_maxima_stay_finite(gpu, tiny):
    """A sample whose cut max or pooled-gradient max is ~1e-38 or ~1e-44 (subnormal in f32; e.g. a
    confidently-correct sample's dpooled): the per-sample scale is clamped so that 2^s and 2^-s stay
    normal floats, so every x3 kernel stays finite and on the float64 bar (1e-5 of max |ref|)."""
    from splitcnn import ops
    B = 6
    act, p, y = _inputs(gpu, B, seed=78)
    act[2] *= tiny / act[2].abs().max()
    am = ops.row_amax(act)
    a16 = torch.empty(ops.conv2_act16_bytes(B), dtype=torch.uint8, device=gpu)
    ps, cs = ops.conv2_fwd_pool(act, p["W2"], p["b2"], impl="x3", act_amax=am, act16=a16)
    pi, ci = ops.conv2_fwd_pool_x3i(a16, am, p["W2"], p["b2"])
    assert torch.isfinite(ps).all() and torch.equal(ps, pi) and torch.equal(cs, ci)
    r64 = conv_relu64(act, p["W2"], p["b2"])
    assert rel_err(ps.cpu().numpy(), r64.reshape(B, 64, 12, 2, 12, 2).amax(dim=(3, 5)).cpu().numpy()) <= 1e-5
    _, _, _, dp = ops.fc_xent(ps, p["W3"], p["b3"], y, 1.0 / B)
    dp[4] *= tiny / dp[4].abs().max()
    dpa = ops.row_amax(dp)
    dc = route64(dp, cs)
    g = ops.conv2_dgrad(dp, cs, p["W2"], impl="x3", dp_amax=dpa)
    assert torch.isfinite(g).all()
    assert rel_err(g.cpu().numpy(), dgrad64(dc, p["W2"]).cpu().numpy()) <= 1e-5
    dW64, db64 = wgrad64(act, dc)
    for s in (ops.conv2_wgrad_slabs(act, dp, cs, impl="x3", act_amax=am, dp_amax=dpa),
              ops.conv2_wgrad_slabs(None, dp, cs, impl="x3", act_amax=am, dp_amax=dpa, act16=a16)):
        got = ops.reduce_slabs(s).cpu().numpy()
        assert np.isfinite(got).all()
        assert rel_err(got[:18432], dW64.reshape(-1).cpu().numpy()) <= 1e-5
        assert rel_err(got[18432:], db64.cpu().numpy()) <= 1e-5
    # the fused client backward on the same tiny-dpooled sample (x chosen freely, with its own ReLU bits)
    from splitcnn.data import SyntheticMNIST, init_models
    a, _ = init_models(seed=79)
    x = SyntheticMNIST(80).batch(B)[0].to(gpu)
    W1, b1 = a.conv1.weight.detach().to(gpu), a.conv1.bias.detach().to(gpu)
    c1 = ops.reduce_slabs(ops.conv2_dgrad_client_slabs(dp, cs, p["W2"], x, _relu_bits(x, W1, b1), dp_amax=dpa)).cpu().numpy()
    assert np.isfinite(c1).all()
    ref = _c1_ref64(x, W1, b1, dgrad64(dc, p["W2"]))
    assert rel_err(c1[:288], ref[:288]) <= 1e-5 and rel_err(c1[288:], ref[288:]) <= 1e-5


def test_trajectory_100_steps_b4096_default_vs_f32_preset(gpu):
    """The north star's fp32 parity run at the K2 batch (BASELINE config 2, B = 4096): 100 steps of the
    default SplitTrainer (x3 conv2, client-written split images, client backward fused into the dgrad)
    against the independent all-f32 preset (Winograd F(2x2,3x3) on the f32 MFMA, separate client
    backward) on the same batches (src/server_part.py:47-52 + src/client_part.py:132-133 per step).
    Bars: every step's loss within 1e-4 relative; after 100 steps each parameter tensor's update
    (w_100 - w_0) agrees to 1e-3 of its largest element (the two paths round differently, and 100
    steps of SGD carry that forward)."""
    from splitcnn.data import SyntheticMNIST, init_models
    from splitcnn.engine import SplitTrainer
    B, steps = 4096, 100
    data = SyntheticMNIST(71)
    xs, ys = zip(*(data.batch(B) for _ in range(8)))
    X, Y = torch.stack(xs).to(gpu), torch.stack(ys).to(gpu)
    runs = []
    for conv in ("x3", "f32"):
        tr = SplitTrainer(*init_models(seed=72), device=gpu, graph=True, conv=conv)
        if conv == "x3":
            assert tr.client.emit_act16 and tr.fuse_client_backward
        init = (tr.client.params.clone(), tr.server.params.clone())
        losses = []
        for i in range(steps):
            # a fresh batch every step: 8 base batches, each sample's noise re-drawn (seeded, same for both)
            g = torch.Generator(device=gpu).manual_seed(1000 + i)
            x = X[i % 8] + 0.05 * torch.randn(X[i % 8].shape, generator=g, device=gpu)
            tr.step(x, Y[i % 8])
            if (i + 1) % 25 == 0:
                losses += [l for _, l in tr.loss_log.flush()]
        torch.cuda.synchronize()
        runs.append((np.array(losses), (tr.client.params - init[0]).double().cpu().numpy(),
                     (tr.server.params - init[1]).double().cpu().numpy()))
    (lx, cx, sx), (lf, cf, sf) = runs
    assert len(lx) == len(lf) == steps
    rel = np.abs(lx - lf) / np.abs(lf)
    assert rel.max() <= 1e-4, (rel.max(), int(rel.argmax()), lx[-1], lf[-1])
    assert lx[-1] < 0.5 * lx[0]  # it trains
    segs = {"W1": (cx, slice(0, 288)), "b1": (cx, slice(288, 320)), "W2": (sx, slice(0, 18432)),
            "b2": (sx, slice(18432, 18496)), "W3": (sx, slice(18496, 110656)), "b3": (sx, slice(110656, 110666))}
    ref = {"W1": cf, "b1": cf, "W2": sf, "b2": sf, "W3": sf, "b3": sf}
    for k, (arr, sl) in segs.items():
        d, r = arr[sl], ref[k][sl]
        err = np.abs(d - r).max() / np.abs(r).max()
        assert err <= 1e-3, (k, err)


@pytest.mark.parametrize("k", [4, 6])
def test_x3_loose_scale_bound_error_within_2x_of_f32(gpu, k):
    """act_amax from the client's conv1 is conv1_cut_bound (>= max act), not the max; with mixed-sign
    W1 or cancelling inputs it can sit several times above the cut's max, which moves the hi/lo split lower and
    drops the low parts of small elements into f16's subnormal range. Bounds 2^k x the true per-sample max
    (k = 4, 6; the dgrad's dp_amax likewise): forward, wgrad and dgrad stay within the f32 path's bars against
    fp64 (1e-5 of max |ref|, <= 2x the f32 Winograd kernel's own error)."""
    from oracle.split_step import conv3x3, conv3x3_dgrad, conv3x3_wgrad, maxpool2_bwd, relu, tie_discrepancies
    from splitcnn import ops
    B = 64
    act, p, y = _inputs(gpu, B, seed=31 + k)
    loose = ops.row_amax(act) * 2.0 ** k
    px, cx = ops.conv2_fwd_pool(act, p["W2"], p["b2"], impl="x3", act_amax=loose)
    pw, cw = ops.conv2_fwd_pool(act, p["W2"], p["b2"])
    a64 = act.double().cpu().numpy()
    r = relu(conv3x3(a64, p["W2"].double().cpu().numpy(), p["b2"].double().cpu().numpy()))
    pr = r.reshape(B, 64, 12, 2, 12, 2).max(axis=(3, 5))
    n, ok = tie_discrepancies(r, cw.cpu().numpy().astype(np.int64), cx.cpu().numpy().astype(np.int64))
    assert ok, f"{n} routing differences that are not ties"
    ex, ew = rel_err(px.cpu().numpy(), pr), rel_err(pw.cpu().numpy(), pr)
    assert ex <= 1e-5 and ex <= max(2 * ew, 1e-6), (ex, ew)

    _, _, _, dp = ops.fc_xent(pw, p["W3"], p["b3"], y, 1.0 / B)
    codes = cw.cpu().numpy().astype(np.int64)
    dp64 = dp.double().cpu().numpy().reshape(B, 64, 12, 12)
    dc = maxpool2_bwd(np.where(codes < 4, dp64, 0.0), np.minimum(codes, 3), (B, 64, 24, 24))
    dloose = ops.row_amax(dp.reshape(B, -1)) * 2.0 ** k
    sx = ops.reduce_slabs(ops.conv2_wgrad_slabs(act, dp, cw, impl="x3", act_amax=loose, dp_amax=dloose)).cpu().numpy()
    sw = ops.reduce_slabs(ops.conv2_wgrad_slabs(act, dp, cw)).cpu().numpy()
    dW, db = conv3x3_wgrad(a64, dc)
    for got, w, ref in ((sx[:18432], sw[:18432], dW.reshape(-1)), (sx[18432:], sw[18432:], db)):
        ex, ew = rel_err(got, ref), rel_err(w, ref)
        assert ex <= 1e-5 and ex <= max(2 * ew, 1e-6), (ex, ew)

    gx = ops.conv2_dgrad(dp, cw, p["W2"], impl="x3", dp_amax=dloose)
    gw = ops.conv2_dgrad(dp, cw, p["W2"])
    ref = conv3x3_dgrad(dc, p["W2"].double().cpu().numpy())
    ex, ew = rel_err(gx.cpu().numpy(), ref), rel_err(gw.cpu().numpy(), ref)
    assert ex <= 1e-5 and ex <= max(2 * ew, 1e-6), (ex, ew)
