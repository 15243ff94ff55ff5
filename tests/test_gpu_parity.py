"""GPU parity: the HIP split step (libslk.so via the C-ABI) against the reference's golden fixtures
(tests/golden/, generated from the reference src/model_def.py) and the numpy oracle.

Tolerances (SURVEY §8c noise floor: fp32 thread-count drift 9e-6 loss / 7e-5 weights):
  per-step tensors from identical state  rel_err <= 1e-4  (max|diff| / max|ref|)
  conv1 activations                      rel_err <= 1e-5
  loss                                   relative <= 1e-5
  1k-step loss curve                     relative <= 1e-3 per step
"""
import numpy as np
import pytest
import torch

from conftest import FIXTURES, PARAMS, load_fixture, rel_err, weight_ok

pytestmark = pytest.mark.gpu

KEYS = {"W1": ("conv1", "weight"), "b1": ("conv1", "bias"), "W2": ("conv2", "weight"),
        "b2": ("conv2", "bias"), "W3": ("fc1", "weight"), "b3": ("fc1", "bias")}


def make_models(fx, prefix="init_"):
    from splitcnn.model_def import ModelPartA, ModelPartB
    a, b = ModelPartA(), ModelPartB()
    sd_a = {"conv1.weight": torch.from_numpy(fx[prefix + "W1"]), "conv1.bias": torch.from_numpy(fx[prefix + "b1"])}
    sd_b = {"conv2.weight": torch.from_numpy(fx[prefix + "W2"]), "conv2.bias": torch.from_numpy(fx[prefix + "b2"]),
            "fc1.weight": torch.from_numpy(fx[prefix + "W3"]), "fc1.bias": torch.from_numpy(fx[prefix + "b3"])}
    a.load_state_dict(sd_a)
    b.load_state_dict(sd_b)
    return a, b


def param_of(client, server, k):
    mod, attr = KEYS[k]
    m = client.model if k in ("W1", "b1") else server.model
    return getattr(getattr(m, mod), attr).detach().cpu().numpy()


def grad_of(client, server, k):
    off = {"W1": (0, 288), "b1": (288, 320), "W2": (0, 18432), "b2": (18432, 18496),
           "W3": (18496, 110656), "b3": (110656, 110666)}[k]
    g = client.grads if k in ("W1", "b1") else server.grads
    return g[off[0]:off[1]].cpu().numpy()


@pytest.mark.parametrize("name", FIXTURES)
def test_engine_matches_reference_fixture(gpu, name):
    from splitcnn.engine import ClientStage, ServerStage
    fx = load_fixture(name)
    a, b = make_models(fx)
    client, server = ClientStage(a, device=gpu), ServerStage(b, device=gpu)
    prev = {k: fx[f"init_{k}"] for k in PARAMS}
    for s in range(1, int(fx["nsteps"]) + 1):
        x = torch.from_numpy(fx[f"x_{s}"]).to(gpu)
        y = torch.from_numpy(fx[f"y_{s}"]).to(gpu)
        act = client.forward(x)
        assert rel_err(act.cpu().numpy(), fx[f"act_{s}"]) <= 1e-5
        cut_grad, loss_i = server.step_request(act, y, step=s)
        logits = server._buf.get("logits", (x.shape[0], 10), torch.float32, gpu)
        assert rel_err(logits.cpu().numpy(), fx[f"logits_{s}"]) <= 1e-4
        assert rel_err(cut_grad.cpu().numpy(), fx[f"cut_grad_{s}"]) <= 1e-4
        client.backward_step(cut_grad)
        torch.cuda.synchronize()
        (step, loss), = server.loss_log.flush()
        assert step == s
        assert abs(loss - float(fx[f"loss_{s}"])) <= 1e-5 * abs(float(fx[f"loss_{s}"]))
        if s == 1:
            for k in PARAMS:
                assert rel_err(grad_of(client, server, k), fx[f"grad_{k}_1"]) <= 1e-4, k
        if f"post_W1_{s}" in fx:
            for k in PARAMS:
                assert weight_ok(param_of(client, server, k), fx[f"post_{k}_{s}"], prev[k]), (k, s)
        prev = {k: param_of(client, server, k) for k in PARAMS}


@pytest.mark.parametrize("name", ["split_step_b4.npz", "split_step_b13.npz"])
def test_dropin_modules_reference_code(gpu, name):
    """The reference's own step code (client_part.py:112-133, server_part.py:45-57) run verbatim on
    the drop-in modules: autograd, .grad on the received leaf, activations.backward(grad)."""
    from splitcnn.model_def import CrossEntropyLoss
    fx = load_fixture(name)
    client_m, server_m = make_models(fx)
    client_m, server_m = client_m.to(gpu), server_m.to(gpu)
    copt = torch.optim.SGD(client_m.parameters(), lr=0.01)
    sopt = torch.optim.SGD(server_m.parameters(), lr=0.01)
    criterion = CrossEntropyLoss()
    x = torch.from_numpy(fx["x_1"]).to(gpu)
    y = torch.from_numpy(fx["y_1"]).to(gpu)
    copt.zero_grad()
    activations = client_m(x)
    client_activations = activations.clone().detach()
    client_activations.requires_grad_(True)
    sopt.zero_grad()
    outputs = server_m(client_activations)
    loss = criterion(outputs, y)
    loss.backward()
    sopt.step()
    cut = client_activations.grad.clone().detach()
    activations.backward(cut)
    copt.step()
    assert rel_err(activations.detach().cpu().numpy(), fx["act_1"]) <= 1e-5
    assert rel_err(outputs.detach().cpu().numpy(), fx["logits_1"]) <= 1e-4
    assert abs(loss.item() - float(fx["loss_1"])) <= 1e-5 * abs(float(fx["loss_1"]))
    assert rel_err(cut.cpu().numpy(), fx["cut_grad_1"]) <= 1e-4
    sd = {**client_m.state_dict(), **server_m.state_dict()}
    for k, (mod, attr) in KEYS.items():
        assert weight_ok(sd[f"{mod}.{attr}"].cpu().numpy(), fx[f"post_{k}_1"], fx[f"init_{k}"]), k


@pytest.mark.parametrize("B", [4, 300])
def test_dropin_eager_fast_path_bitwise_vs_custom_ops(gpu, B):
    """Eager calls of the drop-in modules take autograd.Functions over the same op bodies (library.eager: less
    Python dispatch per call); with the fast path off every call goes through the torch.library custom ops.
    Three steps of the reference's step code (client_part.py:112-133, server_part.py:45-57) each way: every
    activation, loss, cut gradient and parameter bit for bit the same, and the fast path really was taken."""
    from splitcnn import library
    from splitcnn.data import SyntheticMNIST, init_models
    from splitcnn.model_def import CrossEntropyLoss
    data = SyntheticMNIST(12)
    batches = [tuple(t.to(gpu) for t in data.batch(B)) for _ in range(3)]
    runs = []
    for fast in (True, False):
        old = library._EAGER
        library._EAGER = fast
        try:
            client_m, server_m = (m.to(gpu) for m in init_models(seed=4))
            copt = torch.optim.SGD(client_m.parameters(), lr=0.01)
            sopt = torch.optim.SGD(server_m.parameters(), lr=0.01)
            crit = CrossEntropyLoss()
            rec = []
            for x, y in batches:
                copt.zero_grad()
                activations = client_m(x)
                assert (type(activations.grad_fn).__name__.startswith("Conv1ReluFn")) == fast
                ca = activations.clone().detach()
                ca.requires_grad_(True)
                sopt.zero_grad()
                loss = crit(server_m(ca), y)
                loss.backward()
                sopt.step()
                cut = ca.grad.clone().detach()
                activations.backward(cut)
                copt.step()
                rec += [activations.detach().clone(), loss.detach().clone(), cut]
            rec += [p.detach().clone() for p in list(client_m.parameters()) + list(server_m.parameters())]
            runs.append(rec)
        finally:
            library._EAGER = old
    assert all(torch.equal(a, b) for a, b in zip(*runs))


def test_fullmodel_matches_split(gpu):
    from splitcnn.data import init_models
    from splitcnn.model_def import CrossEntropyLoss
    fx = load_fixture("split_step_b4.npz")
    full = init_models(seed=0, full=True).to(gpu)
    x = torch.from_numpy(fx["x_1"]).to(gpu)
    y = torch.from_numpy(fx["y_1"]).to(gpu)
    loss = CrossEntropyLoss()(full(x), y)
    loss.backward()
    assert abs(loss.item() - float(fx["loss_1"])) <= 1e-5 * float(fx["loss_1"])
    assert rel_err(full.conv1.weight.grad.cpu().numpy(), fx["grad_W1_1"]) <= 1e-4
    assert rel_err(full.fc1.weight.grad.cpu().numpy(), fx["grad_W3_1"]) <= 1e-4


def test_loss_curve_1k_steps_graph(gpu):
    """1000 steps at B=64 (HIP-graph replay) follow the reference's curve within 1e-3 per step."""
    from splitcnn.data import SyntheticMNIST, init_models
    from splitcnn.engine import SplitTrainer
    fx = load_fixture("loss_curve_b64.npz")
    a, b = init_models(seed=0)
    tr = SplitTrainer(a, b, device=gpu, graph=True)
    data = SyntheticMNIST(42)
    n = int(fx["nsteps"])
    xs, ys = zip(*(data.batch(64) for _ in range(n)))
    X = torch.stack(xs).to(gpu)
    Y = torch.stack(ys).to(gpu)
    losses = []
    for s in range(n):
        tr.step(X[s], Y[s])
        if (s + 1) % 250 == 0:
            losses += [l for _, l in tr.loss_log.flush()]
    losses = np.array(losses)
    want = fx["losses"].astype(np.float64)
    rel = np.abs(losses - want) / np.abs(want)
    assert rel.max() <= 1e-3, (rel.argmax(), rel.max())
    for k in PARAMS:
        got = param_of(tr.client, tr.server, k)
        assert rel_err(got, fx[f"final_{k}"]) <= 1e-3, k


def test_graph_equals_eager_and_deterministic(gpu):
    from splitcnn.data import SyntheticMNIST, init_models
    from splitcnn.engine import SplitTrainer
    data = SyntheticMNIST(1)
    batches = [data.batch(96) for _ in range(4)]
    results = []
    for graph in (False, True, True):
        a, b = init_models(seed=2)
        tr = SplitTrainer(a, b, device=gpu, graph=graph)
        for x, y in batches:
            tr.step(x.to(gpu), y.to(gpu))
        torch.cuda.synchronize()
        results.append((tr.client.params.cpu(), tr.server.params.cpu(),
                        [l for _, l in tr.loss_log.flush()]))
    for r in results[1:]:
        assert torch.equal(r[0], results[0][0])
        assert torch.equal(r[1], results[0][1])
        assert r[2] == results[0][2]


def tie_aware_oracle(run, relu_out, code_ref, code_gpu):
    """Re-run the oracle with the GPU's max-pool/ReLU routing after checking that every routing
    difference is a numerical tie (top-2 window values within 1e-5 relative: fp32 rounding can
    legitimately flip a first-max decision there; the reference's own fp32 run could too)."""
    from oracle.split_step import tie_discrepancies
    n, ok = tie_discrepancies(relu_out, code_ref, code_gpu)
    assert ok, f"{n} routing differences that are not numerical ties"
    return run(code_gpu) if n else None, n


@pytest.mark.parametrize("B", [1, 3, 5, 17, 63, 64, 65, 127])
def test_ragged_batches_vs_oracle(gpu, B):
    from oracle.split_step import split_step
    from splitcnn.data import SyntheticMNIST, init_models
    from splitcnn.engine import ClientStage, ServerStage
    a, b = init_models(seed=B)
    P = {"W1": a.conv1.weight, "b1": a.conv1.bias, "W2": b.conv2.weight, "b2": b.conv2.bias,
         "W3": b.fc1.weight, "b3": b.fc1.bias}
    P = {k: v.detach().double().numpy() for k, v in P.items()}
    x, y = SyntheticMNIST(100 + B).batch(B)
    xd, yn = x.double().numpy(), y.numpy()
    new, rec = split_step(P, xd, yn)
    client, server = ClientStage(a, device=gpu), ServerStage(b, device=gpu)
    act = client.forward(x.to(gpu))
    cut, _ = server.step_request(act, y.to(gpu), step=0)
    client.backward_step(cut)
    torch.cuda.synchronize()
    code = server._buf.get("code", (B, 64, 12, 12), torch.uint8, gpu).cpu().numpy().astype(np.int64)
    r2, _ = tie_aware_oracle(lambda c: split_step(P, xd, yn, code_override=c)[1],
                             rec["relu_out"], rec["code"], code)
    rec = r2 or rec
    (_, loss), = server.loss_log.flush()
    assert rel_err(act.cpu().numpy(), rec["act"]) <= 1e-5
    assert rel_err(server._buf.get("pooled", (B, 64, 12, 12), torch.float32, gpu).cpu().numpy(),
                   rec["pooled"]) <= 1e-5
    assert rel_err(cut.cpu().numpy(), rec["cut_grad"]) <= 1e-4
    assert abs(loss - rec["loss"]) <= 1e-5 * abs(rec["loss"])
    for k in PARAMS:
        assert rel_err(grad_of(client, server, k), rec["grads"][k]) <= 1e-4, k


def test_b4096_per_sample_independence(gpu):
    """K2 size (B=4096): rows of a full-batch server pass are bit-identical to the same rows run as
    a small batch (per-sample work is independent), weight grads are linear over batch chunks, and
    8 sampled rows match the oracle."""
    from oracle.split_step import server_step
    from splitcnn.data import SyntheticMNIST, init_models
    from splitcnn.engine import ClientStage, ServerStage
    B = 4096
    a, b = init_models(seed=11)
    W = {"W2": b.conv2.weight, "b2": b.conv2.bias, "W3": b.fc1.weight, "b3": b.fc1.bias}
    W = {k: v.detach().double().numpy() for k, v in W.items()}
    client, server = ClientStage(a, device=gpu), ServerStage(b, device=gpu)
    x, y = SyntheticMNIST(5).batch(B)
    x, y = x.to(gpu), y.to(gpu)
    act = client.forward(x).clone()
    cut, loss_i, s2, s3 = server.forward_backward(act, y, 1.0 / B)
    cut = cut.clone()
    loss_i = loss_i.clone()
    server.reduce_grads(s2, s3)
    g_full = server.grads.clone()
    rows = torch.tensor([0, 1, 777, 2048, 3001, 4090, 4094, 4095], device=gpu)
    cut_s, loss_s, _, _ = server.forward_backward(act[rows].contiguous(), y[rows].contiguous(), 1.0 / B)
    code_s = server._buf.get("code", (8, 64, 12, 12), torch.uint8, gpu).cpu().numpy().astype(np.int64)
    assert torch.equal(cut_s, cut[rows])
    assert torch.equal(loss_s, loss_i[rows])
    # linearity of the weight gradient over batch chunks
    acc = torch.zeros_like(g_full)
    for c in range(8):
        sl = slice(c * 512, (c + 1) * 512)
        _, _, s2c, s3c = server.forward_backward(act[sl].contiguous(), y[sl].contiguous(), 1.0 / B)
        server.reduce_grads(s2c, s3c)
        acc += server.grads
    assert rel_err(acc.cpu().numpy(), g_full.cpu().numpy()) <= 1e-5
    # oracle on the sampled rows (scaled by the full batch size)
    a_np, y_np = act[rows].double().cpu().numpy(), y[rows].cpu().numpy()
    run = lambda c=None: server_step(a_np, y_np, W["W2"], W["b2"], W["W3"], W["b3"],  # noqa: E731
                                     grad_scale_batch=B, code_override=c)
    r = run()
    r2, _ = tie_aware_oracle(run, r["relu_out"], r["code"], code_s)
    r = r2 or r
    assert rel_err(cut_s.cpu().numpy(), r["cut_grad"]) <= 1e-4
    assert rel_err(loss_s.cpu().numpy(), r["loss_i"]) <= 1e-5


def test_bad_label_sets_flag(gpu):
    from splitcnn.data import init_models
    from splitcnn.engine import ServerStage
    _, b = init_models(seed=0)
    server = ServerStage(b, device=gpu)
    act = torch.rand(4, 32, 26, 26, device=gpu)
    y = torch.tensor([0, 1, 10, 2], device=gpu)
    server.step_request(act, y)
    with pytest.raises(IndexError):
        server.check_labels()


def test_cpu_tensors_raise(gpu):
    from splitcnn.model_def import ModelPartA
    m = ModelPartA()
    with pytest.raises(RuntimeError, match="HIP kernels"):
        m(torch.zeros(2, 1, 28, 28))


@pytest.mark.gpu
def test_conv1_wgrad_remask_bit_identical_to_act_mask(gpu):
    """slk_conv1_wgrad_remask recomputes the ReLU mask from x, W1, b1 in conv1_fwd's FMA order: its
    slabs must equal slk_conv1_wgrad's (mask read from act) bit for bit, incl. a ragged batch."""
    from splitcnn import ops
    from splitcnn.data import SyntheticMNIST, init_models
    a, _ = init_models(seed=0)
    W1, b1 = a.conv1.weight.detach().to(gpu), a.conv1.bias.detach().to(gpu)
    for B in (5, 4096):
        x, _y = SyntheticMNIST(3).batch(B)
        x = x.to(gpu)
        act = ops.conv1_fwd(x, W1, b1)
        g = torch.randn(B, 32, 26, 26, generator=torch.Generator().manual_seed(1)).to(gpu)
        s_act = ops.conv1_wgrad_slabs(x, act, g)
        s_rm = ops.conv1_wgrad_remask_slabs(x, W1, b1, g)
        assert torch.equal(s_act, s_rm), B


def test_sgd_multi_bit_identical_to_separate_launches():
    """slk_sgd_multi_from_slabs (every optimizer step + the loss log of a server step in one launch,
    as ServerStage.step_request uses it) == slk_sgd_from_slabs per segment + slk_loss_log, bit for bit."""
    from splitcnn import ops
    dev = torch.device("cuda:0")
    g = torch.Generator(device=dev).manual_seed(5)
    shapes = [(128, 320), (256, 18496), (64, 92170)]
    slabs = [torch.randn(s, device=dev, generator=g) for s in shapes]
    params = [torch.randn(s[1], device=dev, generator=g) for s in shapes]
    loss_i = torch.rand(4093, device=dev, generator=g)
    ref_p = [p.clone() for p in params]
    ref_g = [torch.empty_like(p) for p in params]
    ring_a, ring_b = torch.zeros(8, device=dev), torch.zeros(8, device=dev)
    ctr_a, ctr_b = torch.full((1,), 3, dtype=torch.int32, device=dev), torch.full((1,), 3, dtype=torch.int32, device=dev)
    for p, gr, s in zip(ref_p, ref_g, slabs):
        ops.sgd_from_slabs(p, gr, s, 0.01)
    ops.loss_log(loss_i, 1.0 / 4093, ring_a, ctr_a)
    new_p = [p.clone() for p in params]
    new_g = [torch.empty_like(p) for p in params]
    ops.sgd_multi_from_slabs(list(zip(new_p, new_g, slabs)), 0.01, loss=(loss_i, 1.0 / 4093, ring_b, ctr_b))
    torch.cuda.synchronize()
    for a, b in zip(ref_p + ref_g, new_p + new_g):
        assert torch.equal(a, b)
    assert torch.equal(ring_a, ring_b) and int(ctr_b.item()) == 4


def test_graph_alternating_batch_sizes_equal_eager(gpu):
    """A ragged loader alternates batch sizes (60000 % 64 = 32): one HIP graph per size, each with
    its own scratch buffers (a graph must never replay into buffers another size replaced). Graph
    replays of 64 / 32 / 64 / 32 / 64 must equal the eager steps bit for bit."""
    from splitcnn.data import SyntheticMNIST, init_models
    from splitcnn.engine import SplitTrainer
    data = SyntheticMNIST(7)
    batches = [data.batch(B) for B in (64, 32, 64, 32, 64)]
    results = []
    for graph in (False, True):
        tr = SplitTrainer(*init_models(seed=3), device=gpu, graph=graph)
        for x, y in batches:
            tr.step(x.to(gpu), y.to(gpu))
        torch.cuda.synchronize()
        results.append((tr.client.params.cpu(), tr.server.params.cpu(), [l for _, l in tr.loss_log.flush()]))
    assert torch.equal(results[0][0], results[1][0])
    assert torch.equal(results[0][1], results[1][1])
    assert results[0][2] == results[1][2]


@pytest.mark.parametrize("nslab", [16, 17, 33, 64, 65, 256])
def test_slab_reduction_both_orders_vs_float64(gpu, nslab):
    """slk_reduce_slabs / slk_sgd_from_slabs pick their summation order by slab count (<= 16: thread per
    column, ascending; 17-64: 4 waves per 64 columns over slabs w, w+4, ...; > 64: 16 waves over slabs w,
    w+16, ..., partials combined in wave order — include/slk.h). All are fixed orders (run-to-run
    identical) and all match a float64 sum (n = 5000: partial column blocks at every form)."""
    from splitcnn import ops
    g = torch.Generator(device=gpu).manual_seed(nslab)
    n = 5000
    slabs = torch.randn(nslab, n, device=gpu, generator=g)
    got = ops.reduce_slabs(slabs)
    again = ops.reduce_slabs(slabs)
    want = slabs.double().sum(0)
    assert torch.equal(got, again)
    err = (got.double() - want).abs().max().item() / want.abs().max().item()
    assert err <= 1e-6, err
    param = torch.zeros(n, device=gpu)
    grad = torch.empty(n, device=gpu)
    ops.sgd_from_slabs(param, grad, slabs, 0.5)
    assert torch.equal(grad, got) and torch.equal(param, -0.5 * got)


def test_traced_step_runs_the_custom_ops(gpu):
    """make_fx of a full split step (forward, CE, autograd backward) over the drop-in modules: the
    traced graph's forward AND backward are splitcnn:: ops (library.py), and running the traced graph
    gives the eager step's loss and gradients bit for bit."""
    from torch.fx.experimental.proxy_tensor import make_fx
    from splitcnn.data import SyntheticMNIST, init_models
    from splitcnn.model_def import CrossEntropyLoss
    full = init_models(seed=4, full=True).to(gpu)
    names = [n for n, _ in full.named_parameters()]
    ce = CrossEntropyLoss()

    def step(x, y, *params):
        out = torch.func.functional_call(full, dict(zip(names, params)), (x,))
        loss = ce(out, y)
        return (loss, *torch.autograd.grad(loss, params))

    x, y = SyntheticMNIST(3).batch(6)
    x, y = x.to(gpu), y.to(gpu)
    params = [p.detach().clone().requires_grad_(True) for p in full.parameters()]
    gm = make_fx(step, tracing_mode="fake")(x, y, *params)
    targets = {str(n.target) for n in gm.graph.nodes if n.op == "call_function"}
    for op in ("conv1_relu", "conv2_relu_pool", "linear", "cross_entropy", "cross_entropy_grad", "linear_dgrad",
               "linear_wgrad", "row_amax", "conv2_dgrad_x3", "conv2_wgrad_x3", "conv1_wgrad"):
        assert f"splitcnn.{op}.default" in targets, op
    assert not any("convolution" in t or "addmm" in t or "nll_loss" in t for t in targets)
    got = gm(x, y, *params)
    want = step(x, y, *params)
    for a, b in zip(got, want):
        assert torch.equal(a, b)


def test_graphs_on_caller_buffers_bitwise_vs_static_inputs(gpu):
    """SplitTrainer replays graphs captured on the caller's own input buffers (a loader's ring; no copy
    into the static inputs) for up to `graph_inputs` buffer pairs per batch size, and falls back to the
    static inputs for others (here: a fresh tensor every step past the ring): all bit-identical to a
    trainer that always copies into the static inputs."""
    from splitcnn.data import SyntheticMNIST, init_models
    from splitcnn.engine import SplitTrainer
    data = SyntheticMNIST(12)
    B = 96
    xs, ys = zip(*(data.batch(B) for _ in range(3)))
    X, Y = torch.stack(xs).to(gpu), torch.stack(ys).to(gpu)
    own = SplitTrainer(*init_models(seed=5), device=gpu, graph=True, graph_inputs=2)
    cpy = SplitTrainer(*init_models(seed=5), device=gpu, graph=True, graph_inputs=0)
    for i in range(9):
        x, y = X[i % 3], Y[i % 3]          # buffers 0, 1 captured; buffer 2 goes through the copy
        if i >= 6:
            x, y = x.clone(), y.clone()    # fresh tensors
        own.step(x, y)
        cpy.step(x, y)
    torch.cuda.synchronize()
    assert sum(1 for k in own._graphs if isinstance(k, tuple)) == 2
    assert not any(isinstance(k, tuple) for k in cpy._graphs)
    assert torch.equal(own.client.params, cpy.client.params)
    assert torch.equal(own.server.params, cpy.server.params)
    assert [l for _, l in own.loss_log.flush()] == [l for _, l in cpy.loss_log.flush()]


def test_graph_inputs_static_buffers_and_register(gpu):
    """The static inputs handed back (static_inputs(B)) replay their own graph (no second capture on
    the same memory); register_inputs() captures on a declared buffer pair at once; an undeclared pair
    is captured only the second time it is seen. All bit-identical to the always-copy trainer."""
    from splitcnn.data import SyntheticMNIST, init_models
    from splitcnn.engine import SplitTrainer
    data = SyntheticMNIST(13)
    B = 64
    xs, ys = zip(*(data.batch(B) for _ in range(3)))
    X, Y = torch.stack(xs).to(gpu), torch.stack(ys).to(gpu)
    own = SplitTrainer(*init_models(seed=6), device=gpu, graph=True, graph_inputs=4)
    cpy = SplitTrainer(*init_models(seed=6), device=gpu, graph=True, graph_inputs=0)
    sx, sy = own.static_inputs(B)
    assert own.register_inputs(X[0], Y[0])
    n_caller = lambda: sum(1 for k in own._graphs if isinstance(k, tuple))  # noqa: E731
    assert n_caller() == 1
    sx.copy_(X[2])
    sy.copy_(Y[2])
    own.step(sx, sy)
    cpy.step(X[2], Y[2])
    assert n_caller() == 1                       # no graph captured on the static buffers
    own.step(X[1], Y[1])
    cpy.step(X[1], Y[1])
    assert n_caller() == 1                       # first sight of X[1]: static-input copy
    for i in range(4):
        own.step(X[i % 2], Y[i % 2])
        cpy.step(X[i % 2], Y[i % 2])
    assert n_caller() == 2                       # X[1] captured on its second sight
    torch.cuda.synchronize()
    assert torch.equal(own.client.params, cpy.client.params)
    assert torch.equal(own.server.params, cpy.server.params)
    assert [l for _, l in own.loss_log.flush()] == [l for _, l in cpy.loss_log.flush()]


@pytest.mark.parametrize("B", [13, 4096])
def test_dropin_fused_byproducts_bitwise_vs_recomputed(gpu, monkeypatch, B):
    """The drop-in modules' backward takes linear_dgrad's fused per-sample max |dpooled| and the cross
    entropy's forward dlogits (library._MEMO) instead of re-running row_amax / the CE kernel: every gradient
    of the reference's step is bit-identical to the path that recomputes them, and the memo is hit."""
    from splitcnn import library
    from splitcnn.data import SyntheticMNIST, init_models
    from splitcnn.model_def import CrossEntropyLoss
    x, y = SyntheticMNIST(21).batch(B)
    x, y = x.to(gpu), y.to(gpu)
    hits = []
    take = library._Memo.take

    def counting_take(self, kind, t):
        v = take(self, kind, t)
        hits.append((kind, v is not None))
        return v

    def run(use_memo):
        client, server = (m.to(gpu) for m in init_models(seed=2))
        with monkeypatch.context() as mp:
            mp.setattr(library._Memo, "take", counting_take if use_memo else (lambda self, kind, t: None))
            act = client(x)
            ca = act.clone().detach().requires_grad_(True)
            loss = CrossEntropyLoss()(server(ca), y)
            loss.backward()
            act.backward(ca.grad.clone())
        return [loss.detach(), ca.grad] + [p.grad for p in (*client.parameters(), *server.parameters())]

    got = run(True)
    assert sorted(hits) == [("dlogits", True), ("dp_amax", True)], hits
    want = run(False)
    for a, b in zip(got, want):
        assert torch.equal(a, b)


@pytest.mark.parametrize("B", [3, 300])
def test_dropin_server_unaligned_cut_bitwise(gpu, B):
    """ModelPartB on a cut whose storage is not 16-byte aligned takes the row_amax + x3 forward path
    instead of the forward that computes its scales in-kernel (slk_conv2_fwd_pool_x3sa needs 16-B rows):
    the same logits, loss and every gradient bit for bit."""
    from splitcnn.data import SyntheticMNIST, init_models
    from splitcnn.model_def import CrossEntropyLoss
    x, y = SyntheticMNIST(33).batch(B)
    x, y = x.to(gpu), y.to(gpu)
    client, _ = (m.to(gpu) for m in init_models(seed=3))
    act = client(x).detach()
    buf = torch.empty(act.numel() + 1, device=gpu)

    def run(cut):
        _, server = (m.to(gpu) for m in init_models(seed=3))
        ca = cut.requires_grad_(True)
        logits = server(ca)
        loss = CrossEntropyLoss()(logits, y)
        loss.backward()
        return [logits.detach(), loss.detach(), ca.grad] + [p.grad for p in server.parameters()]

    want = run(act.clone())
    un = buf[1:].view(act.shape)
    un.copy_(act)
    assert un.data_ptr() % 16 != 0
    got = run(un)
    for a, b in zip(got, want):
        assert torch.equal(a, b)
