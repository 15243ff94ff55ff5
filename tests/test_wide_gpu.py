"""GPU parity of the widened split CNN (BASELINE config 5) against oracle/wide_step.py.

Tolerances (the north star's "stated looser bound for bf16"):
  * bf16 tensors (activations, pooled maps, cut gradient, unpooled/masked gradients): every element
    equal to the oracle's bf16 rounding of the same math, except rare elements where the f32
    accumulation order of the GPU and the oracle's float64 land on opposite sides of a bf16 rounding
    boundary: those may differ by one bf16 ulp (<= 2^-7 relative) plus the f32 accumulation floor
    (4e-6 x the tensor's max), and must be < 0.1 % of elements;
  * max-pool routing codes: equal except numerical ties (the two candidates within 1e-5 of the
    window's scale), as in the fp32 path (oracle.split_step.tie_discrepancies);
  * weight gradients (f32 sums of exact bf16 x bf16 products): 1e-5 of the gradient's max;
  * Adam (f32 tensor math, torch formula): 1e-6 of the update's max + 2 f32 ulp;
  * loss curve over 30 steps: 2e-2 relative per step (SURVEY.md §8c's bf16 bound).
Each kernel is checked on the GPU's own inputs of that layer (layer-isolated), so a rounding flip
upstream cannot cascade into a false failure downstream.
"""
import numpy as np
import pytest
import torch

from oracle import wide_step as W

pytestmark = pytest.mark.gpu


def _np(t):
    return t.detach().float().cpu().numpy().astype(np.float64)


def _nchw(t):
    from splitcnn.wide import c8_to_nchw
    return _np(c8_to_nchw(t))


def bf16_close(got, want, frac=1e-3, acc_floor=4e-6):
    """One bf16 ulp where the rounding flipped, on top of the f32 accumulation noise floor
    (acc_floor x the tensor's max: f32 sums of O(1) terms carry absolute, not relative, error)."""
    got, want = np.asarray(got), np.asarray(want)
    assert got.shape == want.shape, (got.shape, want.shape)
    bad = got != want
    if not bad.any():
        return
    d = np.abs(got - want)[bad]
    lim = 2.0 ** -7 * np.abs(want)[bad] + acc_floor * np.abs(want).max() + 1e-30
    assert (d <= lim * 1.0001).all(), f"max rel diff {np.max(d / np.maximum(np.abs(want[bad]), 1e-30)):.3g}"
    assert bad.mean() <= frac, f"{bad.mean():.2e} of elements differ by one bf16 ulp"


def codes_close(c_pre, code_got, code_want, rtol=1e-5):
    """Routing differences must be numerical ties of the f32/f64 pre-pool values c_pre."""
    diff = code_got != code_want
    if not diff.any():
        return
    B, C, H, Wd = c_pre.shape
    win = c_pre.reshape(B, C, H // 2, 2, Wd // 2, 2).transpose(0, 1, 2, 4, 3, 5).reshape(B, C, H // 2, Wd // 2, 4)
    win = np.maximum(win, 0.0)[diff]
    scale = max(np.abs(c_pre).max(), 1e-30)

    def val(code):
        return np.where(code < 4, np.take_along_axis(win, np.minimum(code, 3)[:, None], axis=1)[:, 0], 0.0)
    va, vb = val(code_got[diff]), val(code_want[diff])
    assert (np.abs(va - vb) <= rtol * scale).all(), f"{diff.sum()} non-tie routing differences"
    assert diff.mean() < 1e-3


def grad_close(got, want, rtol=1e-5):
    got, want = np.asarray(got, np.float64), np.asarray(want, np.float64)
    err = np.abs(got - want).max() / max(np.abs(want).max(), 1e-30)
    assert err <= rtol, err


def _params(client, server):
    P = {}
    for k, v in client.model.state_dict().items():
        P[k] = _np(v)
    for k, v in server.model.state_dict().items():
        P[k] = _np(v)
    return P


def test_wide_step_layer_by_layer_vs_oracle(gpu):
    from splitcnn.wide import SyntheticCIFAR, WideTrainer, init_wide_models
    A, Bm = init_wide_models(seed=0)
    tr = WideTrainer(A, Bm, device=gpu, graph=False)
    B = 5  # ragged: not a multiple of any tile
    x, y = SyntheticCIFAR(42).batch(B)
    c, s = tr.client, tr.server
    P0 = _params(c, s)
    cut = c.forward(x.to(gpu))
    dcut, loss_i = s.step_request(cut, y.to(gpu))
    grads_s = s.grads.clone()
    c.backward_step(dcut)
    torch.cuda.synchronize()
    xs = x.double().numpy()
    bf = lambda a: W.bf16(a).astype(np.float64)  # noqa: E731

    # conv1 (f32 VALU) -> a1 bf16
    a1 = _nchw(c._a1)
    xb = bf(xs)
    bf16_close(a1, bf(np.maximum(W.conv3x3p1(xb, bf(P0["conv1.weight"]), P0["conv1.bias"]), 0)))
    # conv2 + pool on the GPU's a1
    W2b, W3b = bf(P0["conv2.weight"]), bf(P0["conv3.weight"])
    c2 = W.conv3x3p1(a1, W2b, P0["conv2.bias"])
    p2f, code2 = W.relu_pool_code(c2)
    code2_gpu = _nchw(c._code2).astype(np.int64)
    codes_close(c2, code2_gpu, code2)
    p2 = _nchw(c._p2)
    p2f_g = np.take_along_axis(np.maximum(c2, 0).reshape(B, 128, 16, 2, 16, 2).transpose(0, 1, 2, 4, 3, 5)
                               .reshape(B, 128, 16, 16, 4), np.minimum(code2_gpu, 3)[..., None], -1)[..., 0]
    bf16_close(p2, bf(np.where(code2_gpu < 4, p2f_g, 0.0)))
    # conv3 + pool on the GPU's p2 -> the cut
    c3 = W.conv3x3p1(p2, W3b, P0["conv3.bias"])
    _, code3 = W.relu_pool_code(c3)
    code3_gpu = _nchw(c._code3).astype(np.int64)
    codes_close(c3, code3_gpu, code3)
    cut_g = _nchw(cut)
    p3_g = np.take_along_axis(np.maximum(c3, 0).reshape(B, 256, 8, 2, 8, 2).transpose(0, 1, 2, 4, 3, 5)
                              .reshape(B, 256, 8, 8, 4), np.minimum(code3_gpu, 3)[..., None], -1)[..., 0]
    bf16_close(cut_g, bf(np.where(code3_gpu < 4, p3_g, 0.0)))
    # server on the GPU's cut: dropout mask of step 0, seed 0
    keep = W.dropout_keep(0, 0, B)
    sv = W.server_step(P0, cut_g, y.numpy(), keep)
    np.testing.assert_allclose(_np(loss_i), sv["loss_i"], rtol=2e-6, atol=1e-6)
    np.testing.assert_allclose(_np(s._dlogits), sv["dlogits"], rtol=0, atol=2e-7)
    bf16_close(_nchw(dcut), sv["dcut"])
    grad_close(_np(grads_s[:163840]).reshape(10, -1), sv["grads"]["fc.weight"])
    grad_close(_np(grads_s[163840:]), sv["grads"]["fc.bias"])
    # client backward on the GPU's tensors
    dcut_g = _nchw(dcut)
    dc3 = W.unpool(dcut_g, code3_gpu)     # conv3's kernels route dcut by code3 while staging it
    # conv3's dgrad stores dp2, the gradient of p2 (16 x 16); conv2's kernels route it by code2
    bf16_close(_nchw(c._dp2), bf(W.conv3x3p1_dgrad(dc3, W3b)))
    dc2_g = W.unpool(_nchw(c._dp2), code2_gpu)
    da1 = W.conv3x3p1_dgrad(dc2_g, W2b)
    bf16_close(_nchw(c._da1m), bf(np.where(a1 > 0, da1, 0.0)))
    g = _np(c.grads)
    dW3, db3 = W.conv3x3p1_wgrad(p2, dc3)
    grad_close(g[75648:370560].reshape(256, 128, 3, 3), dW3)
    grad_close(g[370560:], db3)
    dW2, db2 = W.conv3x3p1_wgrad(a1, dc2_g)
    grad_close(g[1792:75520].reshape(128, 64, 3, 3), dW2)
    grad_close(g[75520:75648], db2)
    dW1, db1 = W.conv3x3p1_wgrad(xb, _nchw(c._da1m))
    grad_close(g[:1728].reshape(64, 3, 3, 3), dW1)
    grad_close(g[1728:1792], db1)
    # Adam (t = 1) on the GPU's own gradients
    flat0 = np.concatenate([P0[k].ravel() for k in W.CLIENT_KEYS])
    want, _, _ = W.adam(flat0, g, np.zeros_like(g), np.zeros_like(g), 1)
    got = _np(c.params)
    tol = 1e-6 * np.abs(want - flat0).max() + 2 * np.finfo(np.float32).eps * np.abs(want)
    assert (np.abs(got - want) <= tol).all()
    assert int(c.step_ctr.item()) == 1 and int(s.step_ctr.item()) == 1


def test_wide_large_batch_per_sample_rows_and_linearity(gpu):
    """B = 520 exercises the persistent multi-tile pipelines of every kernel (each workgroup walks
    several tiles). Size-independent properties: per-sample forward and input-gradient rows are
    bit-identical to small-batch runs (per-element K order does not depend on the tile mapping);
    weight gradients are linear in the batch (1e-5)."""
    from splitcnn.wide import SyntheticCIFAR, WideClientStage, init_wide_models
    A, _ = init_wide_models(seed=0)
    c = WideClientStage(A, device=gpu)
    B = 520
    x, _ = SyntheticCIFAR(7).batch(B)
    x = x.to(gpu)
    gen = torch.Generator().manual_seed(3)
    dcut = (torch.randn(B, 32, 8, 8, 8, generator=gen) * 1e-3).to(torch.bfloat16).to(gpu)
    cut = c.forward(x).clone()
    s1, s2, s3 = (t.sum(0) for t in c.backward_slabs(dcut))
    dp2, da1m = c._dp2.clone(), c._da1m.clone()
    parts = []
    for lo, hi in ((0, 4), (4, 260), (260, 516), (516, 520)):
        cut_p = c.forward(x[lo:hi].contiguous()).clone()
        assert torch.equal(cut_p, cut[lo:hi]), (lo, hi)
        t1, t2, t3 = (t.sum(0) for t in c.backward_slabs(dcut[lo:hi].contiguous()))
        assert torch.equal(c._dp2, dp2[lo:hi]) and torch.equal(c._da1m, da1m[lo:hi]), (lo, hi)
        parts.append((t1, t2, t3))
    for k, tot in enumerate((s1, s2, s3)):
        acc = sum(p[k].double() for p in parts)
        grad_close(_np(tot), _np(acc))
    torch.cuda.synchronize()


def test_wide_graph_replay_equals_eager_and_is_deterministic(gpu):
    from splitcnn.wide import SyntheticCIFAR, WideTrainer, init_wide_models
    runs = []
    for graph in (True, False, True):
        A, Bm = init_wide_models(seed=0)
        tr = WideTrainer(A, Bm, device=gpu, graph=graph)
        data = SyntheticCIFAR(42)
        for _ in range(3):
            x, y = data.batch(64)
            tr.step(x.to(gpu), y.to(gpu))
        torch.cuda.synchronize()
        runs.append((tr.client.params.clone(), tr.server.params.clone(), [l for _, l in tr.loss_log.flush()]))
    for r in runs[1:]:
        assert torch.equal(r[0], runs[0][0]) and torch.equal(r[1], runs[0][1])
        assert r[2] == runs[0][2]


def test_wide_loss_curve_vs_oracle(gpu):
    """30 Adam steps at B = 8 through the HIP graph vs the bf16 oracle chained on its own state."""
    from splitcnn.wide import SyntheticCIFAR, WideTrainer, init_wide_models
    A, Bm = init_wide_models(seed=0)
    P = {k: v.detach().double().numpy() for k, v in list(A.state_dict().items()) + list(Bm.state_dict().items())}
    tr = WideTrainer(A, Bm, device=gpu, graph=True)
    data = SyntheticCIFAR(11)
    opt, want = {}, []
    for t in range(1, 31):
        x, y = data.batch(8)
        tr.step(x.to(gpu), y.to(gpu))
        P, opt, rec = W.wide_step(P, opt, t, x.numpy(), y.numpy(), seed=0)
        want.append(rec["loss"])
    got = [l for _, l in tr.loss_log.flush()]
    rel = np.abs(np.array(got) - np.array(want)) / np.abs(np.array(want))
    assert rel.max() <= 2e-2, rel
    assert np.mean(got[-5:]) < np.mean(got[:5])   # it learns


def test_wide_hub_stage_interface_loopback(gpu):
    """The stage methods dist.WideHub drives — clients: forward(x, tag) / backward_grads(dcut, tag,
    accumulate) / step_from_grads; server: accumulate(part) / finish_step — run in one process for 2
    simulated clients x 2 micro-batches (server order: micro-batch outer, client inner; all-reduce by
    hand) equal the fused single-GPU step at the concatenated batch: loss, server and client gradients
    to 1e-6 (summation order), Adam on those gradients to the torch formula."""
    from splitcnn.wide import SyntheticCIFAR, WideClientStage, WideServerStage, WideTrainer, init_wide_models
    B, m = 24, 2
    b = B // m
    x, y = SyntheticCIFAR(3).batch(2 * B)
    x, y = x.to(gpu), y.to(gpu)
    ref = WideTrainer(*init_wide_models(seed=0), device=gpu, graph=False)
    ref.step(x, y)
    clients = [WideClientStage(init_wide_models(seed=0)[0], device=gpu) for _ in range(2)]
    server = WideServerStage(init_wide_models(seed=0)[1], device=gpu)
    cuts = {}
    for c in range(2):
        for k in range(m):
            cuts[c, k] = clients[c].forward(x[c * B + k * b:c * B + (k + 1) * b].contiguous(), tag=k).clone()
    dcuts, part = {}, 0
    for k in range(m):
        for c in range(2):
            sl = slice(c * B + k * b, c * B + (k + 1) * b)
            dcuts[c, k] = server.accumulate(cuts[c, k], y[sl].contiguous(), 1.0 / (2 * B), c * B + k * b, part,
                                            2 * m).clone()
            part += 1
    server_grads = server.grads.clone()
    server.finish_step(2 * m, step=0)
    for c in range(2):
        for k in range(m):
            clients[c].backward_grads(dcuts[c, k], tag=k, accumulate=k > 0)
    total = clients[0].grads + clients[1].grads
    for c in clients:
        c.grads.copy_(total)
        c.step_from_grads()
    torch.cuda.synchronize()
    assert abs(server.loss_log.flush()[0][1] - ref.loss_log.flush()[0][1]) <= 1e-6
    grad_close(_np(server_grads), _np(ref.server.grads), rtol=1e-6)
    grad_close(_np(clients[0].grads), _np(ref.client.grads), rtol=1e-6)
    assert torch.equal(clients[0].params, clients[1].params)
    # Adam from the all-reduced gradient (nslab = 1 path) = the torch formula on that gradient. (Not
    # compared with ref's params: Adam's first step is ~lr*sign(g), so a 1e-7 summation-order
    # difference on a gradient that cancels to ~0 legitimately flips that weight's update.)
    for stage, model, g in ((clients[0], init_wide_models(seed=0)[0], _np(clients[0].grads)),
                            (server, init_wide_models(seed=0)[1], _np(server_grads))):
        flat0 = np.concatenate([v.detach().double().numpy().ravel() for v in model.state_dict().values()])
        want, _, _ = W.adam(flat0, g, np.zeros_like(g), np.zeros_like(g), 1)
        got = _np(stage.params)
        tol = 1e-6 * np.abs(want - flat0).max() + 2 * np.finfo(np.float32).eps * np.abs(want)
        assert (np.abs(got - want) <= tol).all()


def test_adam_multi_bit_identical_to_separate_launches():
    """WideClientStage.step_from_slabs' single slk_adam_multi_from_slabs launch == one
    slk_adam_from_slabs per slab set, bit for bit (params, grads, m, v)."""
    from splitcnn.wide import WideClientStage, init_wide_models
    dev = torch.device("cuda:0")
    g = torch.Generator(device=dev).manual_seed(11)
    stages = []
    for fuse in (True, False):
        a, _ = init_wide_models(seed=0)
        st = WideClientStage(a, device=dev)
        st.fuse_adam = fuse
        stages.append(st)
    # slab counts on both sides of the 64-slab order switch (the production conv1 set has 512 slabs)
    slabs = [torch.randn(n_s, n, device=dev, generator=g) * 1e-3 for n_s, n in ((512, 1792), (17, 73856), (65, 295168))]
    for _ in range(2):  # two steps: the second reads m, v and the step counter the first wrote
        for st in stages:
            st.step_from_slabs(*slabs)
    torch.cuda.synchronize()
    for x, y in zip((stages[0].params, stages[0].grads, stages[0].m, stages[0].v),
                    (stages[1].params, stages[1].grads, stages[1].m, stages[1].v)):
        assert torch.equal(x, y)


def test_wide_graph_alternating_batch_sizes_equal_eager(gpu):
    """WideTrainer: one HIP graph per batch size with its own scratch; 16 / 8 / 16 / 8 graph replays
    equal the eager steps bit for bit (the dropout mask follows the device step counter in both)."""
    from splitcnn.wide import SyntheticCIFAR, WideTrainer, init_wide_models
    data = SyntheticCIFAR(9)
    batches = [data.batch(B) for B in (16, 8, 16, 8)]
    results = []
    for graph in (False, True):
        tr = WideTrainer(*init_wide_models(seed=1), device=gpu, graph=graph)
        for x, y in batches:
            tr.step(x.to(gpu), y.to(gpu))
        torch.cuda.synchronize()
        results.append((tr.client.params.cpu(), tr.server.params.cpu(), [l for _, l in tr.loss_log.flush()]))
    assert torch.equal(results[0][0], results[1][0])
    assert torch.equal(results[0][1], results[1][1])
    assert results[0][2] == results[1][2]


def test_wide_modules_run_the_reference_step_code(gpu):
    """Module contract for the widened model: the reference's own step code (client_part.py:112-133,
    server_part.py:45-57) run verbatim on WideModelPartA / WideModelPartB with torch.optim.Adam and the
    drop-in CrossEntropyLoss. Same kernels as the stages, so the cut, the loss, the cut gradient and
    every weight gradient equal the fused WideTrainer step's; Adam (torch's own here) matches the
    torch formula on those gradients; WideFullModel's forward/backward equals the split modules'."""
    from splitcnn.model_def import CrossEntropyLoss
    from splitcnn.wide import SyntheticCIFAR, WideFullModel, WideTrainer, c8_to_nchw, init_wide_models
    B = 8
    x, y = SyntheticCIFAR(4).batch(B)
    x, y = x.to(gpu), y.to(gpu)
    ref = WideTrainer(*init_wide_models(seed=0), device=gpu, graph=False)
    cut_r = ref.client.forward(x)           # the stage path (dcut returned to the client)
    dcut_r, _ = ref.server.step_request(cut_r, y)
    ref.client.backward_step(dcut_r)
    torch.cuda.synchronize()
    ref_cut, ref_dcut = c8_to_nchw(cut_r), c8_to_nchw(dcut_r)
    (_, ref_loss), = ref.loss_log.flush()

    client_m, server_m = init_wide_models(seed=0)
    client_m, server_m = client_m.to(gpu), server_m.to(gpu)
    P0 = {k: _np(v) for k, v in list(client_m.state_dict().items()) + list(server_m.state_dict().items())}
    optimizer_c = torch.optim.Adam(client_m.parameters(), lr=1e-3)
    optimizer_s = torch.optim.Adam(server_m.parameters(), lr=1e-3)
    criterion = CrossEntropyLoss()
    # --- client_part.py:112-122
    optimizer_c.zero_grad()
    activations = client_m(x)
    client_activations = activations.clone().detach()
    # --- server_part.py:45-57
    client_activations.requires_grad_(True)
    optimizer_s.zero_grad()
    outputs = server_m(client_activations)
    loss = criterion(outputs, y)
    loss.backward()
    optimizer_s.step()
    server_grads = client_activations.grad.clone().detach()
    # --- client_part.py:131-133
    activations.backward(server_grads)
    optimizer_c.step()
    torch.cuda.synchronize()

    assert activations.dtype == torch.bfloat16 and tuple(activations.shape) == (B, 256, 8, 8)
    assert torch.equal(activations, ref_cut)
    assert abs(loss.item() - ref_loss) <= 1e-6 * abs(ref_loss)
    assert torch.equal(server_grads, ref_dcut)
    cg, sg = _np(ref.client.grads), _np(ref.server.grads)
    offs = {"conv1.weight": (0, 1728), "conv1.bias": (1728, 1792), "conv2.weight": (1792, 75520),
            "conv2.bias": (75520, 75648), "conv3.weight": (75648, 370560), "conv3.bias": (370560, 370816)}
    for name, p in client_m.named_parameters():
        lo, hi = offs[name]
        grad_close(_np(p.grad).ravel(), cg[lo:hi], rtol=1e-6)
    grad_close(_np(server_m.fc.weight.grad).ravel(), sg[:163840], rtol=1e-6)
    grad_close(_np(server_m.fc.bias.grad), sg[163840:], rtol=1e-6)
    # torch's Adam on these gradients = the torch formula (oracle/wide_step.adam) to f32 rounding
    for m in (client_m, server_m):
        for name, p in m.named_parameters():
            g = _np(p.grad).ravel()
            want, _, _ = W.adam(P0[name].ravel(), g, np.zeros_like(g), np.zeros_like(g), 1)
            tol = 1e-6 * np.abs(want - P0[name].ravel()).max() + 2 * np.finfo(np.float32).eps * np.abs(want)
            assert (np.abs(_np(p).ravel() - want) <= tol).all(), name

    # WideFullModel (seeded like the halves): same logits and gradients as the split modules
    torch.manual_seed(0)
    full = WideFullModel().to(gpu)
    out_full = full(x)
    assert torch.equal(out_full, outputs)
    criterion(out_full, y).backward()
    for name in ("conv1.weight", "conv3.weight", "fc.weight"):
        mod, attr = name.split(".")
        a = getattr(getattr(full, mod), attr).grad
        b = getattr(getattr(client_m if mod != "fc" else server_m, mod), attr).grad
        assert torch.equal(a, b), name
    # eval mode: no dropout, no counter advance
    server_m.eval()
    with torch.no_grad():
        e1 = server_m(client_activations)
        e2 = server_m(client_activations)
    assert torch.equal(e1, e2)


def test_pooled_gradient_routing_random_codes(gpu):
    """The client backward never stores an unpooled gradient: conv3's dgrad/wgrad route the pooled
    dcut by code3 while staging it, and conv2's route dp2 by code2. Drive client_backward_kernels
    with arbitrary codes (every window position and the ReLU-blocked code 4, uniformly) and random
    operands at a ragged batch (9: one image past the 8-XCD grouping), against the oracle applied to
    the explicitly unpooled gradients."""
    from splitcnn import wide
    B = 9
    g = torch.Generator().manual_seed(5)
    rnd = lambda *shape, scale=1.0: torch.randn(*shape, generator=g) * scale  # noqa: E731
    code = lambda *shape: torch.randint(0, 5, shape, generator=g, dtype=torch.uint8)  # noqa: E731
    W1, W2, W3 = rnd(64, 3, 3, 3, scale=0.2), rnd(128, 64, 3, 3, scale=0.05), rnd(256, 128, 3, 3, scale=0.03)
    x = rnd(B, 3, 32, 32)
    a1 = rnd(B, 64, 32, 32).bfloat16()                  # signed: the a1 > 0 mask matters
    p2 = rnd(B, 128, 16, 16).abs().bfloat16()
    code2, code3 = code(B, 128, 16, 16), code(B, 256, 8, 8)
    dcut = rnd(B, 256, 8, 8, scale=1e-2).bfloat16()
    dev = torch.device(gpu)
    sh = wide.new_shadows(dev)
    W1d, W2d, W3d = (w.to(dev) for w in (W1, W2, W3))
    wide.build_shadows(W1d, W2d, W3d, sh, wide._stream(W1d))
    c8 = lambda t: wide.nchw_to_c8(t.to(dev))  # noqa: E731
    saved = (x.to(dev), c8(a1), c8(p2), c8(code2), c8(code3))
    scratch = wide.client_backward_scratch(B, lambda n, shp, dt: torch.empty(shp, dtype=dt, device=dev))
    slabs = [torch.empty(shp, dtype=torch.float32, device=dev) for shp in wide.client_backward_slab_shapes(B)]
    wide.client_backward_kernels(c8(dcut), saved, sh["w2d"], sh["w3d"], scratch, *slabs)
    g1, g2, g3 = (_np(wide._reduce(sl)) for sl in slabs)
    dp2, da1m = (_nchw(t) for t in scratch)

    f = lambda t: t.double().numpy()  # noqa: E731
    bf = lambda a: W.bf16(a).astype(np.float64)  # noqa: E731
    dc3 = W.unpool(f(dcut), f(code3).astype(np.int64))
    bf16_close(dp2, bf(W.conv3x3p1_dgrad(dc3, bf(f(W3)))))
    dW3, db3 = W.conv3x3p1_wgrad(f(p2), dc3)
    grad_close(g3[:294912].reshape(256, 128, 3, 3), dW3)
    grad_close(g3[294912:], db3)
    dc2 = W.unpool(dp2, f(code2).astype(np.int64))      # on the GPU's dp2 (layer-isolated)
    bf16_close(da1m, bf(np.where(f(a1) > 0, W.conv3x3p1_dgrad(dc2, bf(f(W2))), 0.0)))
    dW2, db2 = W.conv3x3p1_wgrad(f(a1), dc2)
    grad_close(g2[:73728].reshape(128, 64, 3, 3), dW2)
    grad_close(g2[73728:], db2)
    dW1, db1 = W.conv3x3p1_wgrad(bf(f(x)), da1m)
    grad_close(g1[:1728].reshape(64, 3, 3, 3), dW1)
    grad_close(g1[1728:], db1)


def test_wide_head_ragged_batch_vs_oracle(gpu):
    """The step's head (wide_head16_kernel<true> + wide_head_back_kernel<false>) at a ragged B = 1000
    (62.5 sixteen-sample workgroups, 15.6 weight-gradient groups) as micro-batch b0 = 3 of step 2, seed 5:
    logits / loss / dlogits vs the fp64 oracle, the cut gradient within one bf16 ulp, the fc slabs' sum
    vs the oracle's weight gradient, and the dropout bits the head hands the weight-gradient pass in
    `work` equal to the oracle's mask (bit k of byte [b][chunk] = feature (plane * 8 + k) * 64 + pixel)."""
    from splitcnn.wide import WideServerStage, _q, init_wide_models, nchw_to_c8
    _, Bm = init_wide_models(seed=0)
    s = WideServerStage(Bm, device=gpu, seed=5)
    B, b0, step = 1000, 3, 2
    gen = torch.Generator().manual_seed(9)
    cut_nchw = torch.randn(B, 256, 8, 8, generator=gen).clamp_min(0).to(torch.bfloat16)
    y = torch.randint(0, 10, (B,), generator=gen)
    s.step_ctr.fill_(step)
    dcut, loss_i, sf = s.forward_backward(nchw_to_c8(cut_nchw).to(gpu), y.to(gpu), 1.0 / B, b0=b0)
    work = s._b("work", (_q("slk_wide_head_work", B),), torch.float32)
    torch.cuda.synchronize()
    P = {k: _np(v) for k, v in s.model.state_dict().items()}
    keep = W.dropout_keep(5, step, B, b0=b0)
    sv = W.server_step(P, _np(cut_nchw), y.numpy(), keep)
    grad_close(_np(s._logits), sv["logits"], rtol=1e-5)
    np.testing.assert_allclose(_np(loss_i), sv["loss_i"], rtol=2e-6, atol=1e-6)
    np.testing.assert_allclose(_np(s._dlogits), sv["dlogits"], rtol=0, atol=2e-7)
    bf16_close(_nchw(dcut), sv["dcut"])
    g = _np(sf.sum(0))
    grad_close(g[:163840].reshape(10, -1), sv["grads"]["fc.weight"])
    grad_close(g[163840:], sv["grads"]["fc.bias"])
    bits = work.view(torch.uint8)[:B * 2048].cpu().numpy().reshape(B, 2048)
    want = np.packbits(keep.reshape(B, 32, 8, 64).transpose(0, 1, 3, 2), axis=-1, bitorder="little")
    assert np.array_equal(bits, want.reshape(B, 2048))
