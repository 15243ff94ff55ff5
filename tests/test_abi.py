"""CPU-side checks of the drop-in boundary: the C-ABI library loads and exports exactly what
include/slk.h declares, argument validation works without a GPU, and the Python module contract
(src/model_def.py:1-71) is preserved: names, state_dict keys/shapes, seeded init, get_model."""
import os
import re

import numpy as np
import pytest
import torch

from conftest import ROOT, load_fixture


def header_symbols():
    src = open(os.path.join(ROOT, "include", "slk.h")).read()
    return sorted(set(re.findall(r"^\s*(?:const\s+char\*|int64_t|int)\s+(slk_\w+)\s*\(", src, re.M)))


def test_library_exports_every_header_symbol():
    from splitcnn import _lib
    lib = _lib.load()
    syms = header_symbols()
    assert len(syms) >= 20
    for s in syms:
        assert hasattr(lib, s), s
    assert sorted(_lib.SYMBOLS) == syms, "ctypes bindings and include/slk.h disagree"
    assert lib.slk_abi_version() == 1


def test_argument_validation_without_gpu():
    from splitcnn import _lib
    lib = _lib.load()
    assert lib.slk_conv1_fwd(None, None, None, None, -1, None) == 1      # hipErrorInvalidValue
    assert lib.slk_conv1_fwd(None, None, None, None, 0, None) == 0       # empty batch: no launch
    assert lib.slk_conv2_fwd_pool(None, None, None, None, None, 5, None) == 1  # null buffers
    assert lib.slk_loss_log(None, 0, 1.0, None, 1, None, None) == 1
    assert lib.slk_error_string(1) == b"invalid argument"
    with pytest.raises(_lib.SLKError, match="invalid argument"):
        _lib.call("slk_conv2_dgrad", None, None, None, None, 3, None)


def test_slab_counts_are_functions_of_batch_only():
    from splitcnn import ops
    assert ops.conv2_wgrad_nslab(4096) == 256 and ops.conv2_wgrad_nslab(3) == 9
    assert ops.conv1_wgrad_nslab(4096) == 128 and ops.conv1_wgrad_nslab(50) == 50 and ops.conv1_wgrad_nslab(1) == 1
    assert ops.fc_wgrad_nslab(4096) == 64 and ops.fc_wgrad_nslab(13) == 1
    assert ops.conv2_wgrad_nslab(0) == 0


def test_shipped_kernel_forms():
    """The default build's weight gradients run on the 2:4-sparse MFMA (K2 x3 images wgrad: form 2; K5: 1)."""
    from splitcnn import _lib
    assert _lib.query("slk_conv2_wgrad_x3_form") == 2
    assert _lib.query("slk_wide_wgrad_form") == 1


def test_ops_refuse_cpu_tensors():
    from splitcnn import ops
    with pytest.raises(RuntimeError, match="no CPU fallback"):
        ops.conv1_fwd(torch.zeros(2, 1, 28, 28), torch.zeros(32, 1, 3, 3), torch.zeros(32))


def test_module_contract_matches_reference():
    from splitcnn import FullModel, ModelPartA, ModelPartB
    a, b, f = ModelPartA(), ModelPartB(), FullModel()
    assert {k: tuple(v.shape) for k, v in a.state_dict().items()} == {
        "conv1.weight": (32, 1, 3, 3), "conv1.bias": (32,)}
    assert {k: tuple(v.shape) for k, v in b.state_dict().items()} == {
        "conv2.weight": (64, 32, 3, 3), "conv2.bias": (64,), "fc1.weight": (10, 9216), "fc1.bias": (10,)}
    assert set(f.state_dict()) == set(a.state_dict()) | set(b.state_dict())
    for m in (a, b, f):
        with pytest.raises(RuntimeError, match="HIP kernels"):
            m(torch.zeros(1, 1, 28, 28) if m is not b else torch.zeros(1, 32, 26, 26))


def test_seeded_init_is_bit_identical_to_reference():
    """torch.manual_seed(0); ModelPartA(); ModelPartB() consumes the RNG exactly like the reference
    (SURVEY §3.3), so weights equal the fixture's init weights (made by the reference modules)."""
    from splitcnn.data import init_models
    fx = load_fixture("split_step_b4.npz")
    a, b = init_models(seed=0)
    got = {"W1": a.conv1.weight, "b1": a.conv1.bias, "W2": b.conv2.weight, "b2": b.conv2.bias,
           "W3": b.fc1.weight, "b3": b.fc1.bias}
    for k, v in got.items():
        assert np.array_equal(v.detach().numpy(), fx["init_" + k]), k
    full = init_models(seed=0, full=True)
    assert np.array_equal(full.fc1.weight.detach().numpy(), fx["init_W3"])


def test_get_model_dispatch(monkeypatch):
    from splitcnn import FullModel, ModelPartA, ModelPartB, get_model
    monkeypatch.delenv("LEARNING_MODE", raising=False)
    assert isinstance(get_model("client"), ModelPartA)
    assert isinstance(get_model("server"), ModelPartB)
    assert isinstance(get_model(), ModelPartA)
    monkeypatch.setenv("LEARNING_MODE", "Split")
    assert isinstance(get_model("anything"), ModelPartB)
    monkeypatch.setenv("LEARNING_MODE", "FEDERATED")
    assert isinstance(get_model("client"), FullModel)
    monkeypatch.setenv("LEARNING_MODE", "vertical")
    with pytest.raises(ValueError, match="Unknown LEARNING_MODE: vertical"):
        get_model("client")


def test_model_def_shim_importable_like_reference():
    import importlib
    md = importlib.import_module("model_def")  # split-learning-k8s_amd/model_def.py
    assert md.get_model.__module__ == "splitcnn.model_def"


def test_forward_never_calls_torch_conv(monkeypatch):
    """The nn.Conv2d/nn.Linear submodules are parameter containers only."""
    import torch.nn as nn
    from splitcnn import ModelPartA
    called = []
    monkeypatch.setattr(nn.Conv2d, "forward", lambda self, x: called.append(1))
    m = ModelPartA()
    with pytest.raises(RuntimeError):
        m(torch.zeros(1, 1, 28, 28))
    assert not called


def test_library_build_id_matches_tree():
    """Binary provenance: libslk.so carries the sha256 of the sources it was compiled from; the
    loader refuses a library built from other sources, and needs_build() compares hashes."""
    from splitcnn import _lib, build
    lib = _lib.load()
    assert lib.slk_build_id().decode() == build.source_hash() == build.library_build_id()
    assert not build.needs_build()


def test_modules_export_as_splitcnn_custom_ops():
    """torch.library registration (splitcnn/library.py): the drop-in modules trace under
    torch.export with fake CUDA inputs (no GPU needed, fake kernels give the shapes); the exported
    graph holds only splitcnn:: ops plus views — no aten conv / linear / loss."""
    from torch._subclasses.fake_tensor import FakeTensorMode
    from splitcnn.model_def import CrossEntropyLoss, FullModel

    class Step(torch.nn.Module):
        def __init__(self):
            super().__init__()
            self.m, self.ce = FullModel(), CrossEntropyLoss()

        def forward(self, x, y):
            return self.ce(self.m(x), y)

    with FakeTensorMode():
        x = torch.empty(4, 1, 28, 28, device="cuda")
        y = torch.zeros(4, dtype=torch.int64, device="cuda")
    ep = torch.export.export(Step().to("meta"), (x, y), strict=False)
    targets = [str(n.target) for n in ep.graph.nodes if n.op == "call_function"]
    assert [t for t in targets if t.startswith("splitcnn.")] == [
        "splitcnn.conv1_relu.default", "splitcnn.conv2_relu_pool.default", "splitcnn.linear.default",
        "splitcnn.cross_entropy.default"]
    assert all(t.startswith("splitcnn.") or t in ("aten.view.default", "<built-in function getitem>") for t in targets)
    loss = [n for n in ep.graph.nodes if n.op == "output"][0].args[0][0]
    assert tuple(loss.meta["val"].shape) == ()


def test_custom_op_fake_kernels_shapes():
    """Every splitcnn op's fake kernel returns the shapes/dtypes the real kernel writes."""
    from torch._subclasses.fake_tensor import FakeTensorMode
    from splitcnn import library  # noqa: F401
    O = torch.ops.splitcnn
    with FakeTensorMode():
        x = torch.empty(3, 1, 28, 28, device="cuda")
        act = O.conv1_relu(x, torch.empty(32, 1, 3, 3, device="cuda"), torch.empty(32, device="cuda"))
        pooled, code, amax, a16 = O.conv2_relu_pool(act, torch.empty(64, 32, 3, 3, device="cuda"),
                                                     torch.empty(64, device="cuda"))
        flat = pooled.view(3, 9216)
        logits = O.linear(flat, torch.empty(10, 9216, device="cuda"), torch.empty(10, device="cuda"))
        y = torch.zeros(3, dtype=torch.int64, device="cuda")
        got = {"act": act, "pooled": pooled, "code": code, "logits": logits,
               "loss": O.cross_entropy(logits, y), "dlogits": O.cross_entropy_grad(logits, y, logits.new_ones(())),
               "dflat": O.linear_dgrad(logits, torch.empty(10, 9216, device="cuda")),
               "g3": O.linear_wgrad(logits, flat), "cut": O.conv2_dgrad(pooled, code, torch.empty(64, 32, 3, 3, device="cuda")),
               "g2": O.conv2_wgrad(act, pooled, code), "g1": O.conv1_wgrad(x, torch.empty(32, 1, 3, 3, device="cuda"), torch.empty(32, device="cuda"), act),
               "amax": amax, "a16": a16, "dpa": O.row_amax(pooled),
               "cut_x3": O.conv2_dgrad_x3(pooled, code, torch.empty(64, 32, 3, 3, device="cuda"), amax),
               "g2_x3": O.conv2_wgrad_x3(a16, amax, pooled, amax, code)}
    want = {"act": (3, 32, 26, 26), "pooled": (3, 64, 12, 12), "code": (3, 64, 12, 12), "logits": (3, 10),
            "loss": (), "dlogits": (3, 10), "dflat": (3, 9216), "g3": (92170,), "cut": (3, 32, 26, 26),
            "g2": (18496,), "g1": (320,), "amax": (3,), "a16": (3 * 86528,), "dpa": (3,), "cut_x3": (3, 32, 26, 26),
            "g2_x3": (18496,)}
    for k, shp in want.items():
        assert tuple(got[k].shape) == shp, k
        assert got[k].dtype == (torch.uint8 if k in ("code", "a16") else torch.float32), k


def test_fused_step_preconditions_without_gpu():
    """The split-image and fused-client-backward paths refuse configurations they cannot serve before
    touching a kernel: client images need the x3 forward AND wgrad plus act_amax; the wrappers need
    act16 / act_amax when act is None; conv presets name their kernels."""
    from splitcnn import ops
    from splitcnn.engine import CONV_PRESETS, ServerStage
    assert CONV_PRESETS["x3"] == ("x3", "x3", "x3") and CONV_PRESETS["f32"] == ("wino", "wino", "wino")
    y = torch.zeros(3, dtype=torch.int64)
    img = torch.empty(1, dtype=torch.uint8)
    for conv, amax in (("f32", torch.zeros(3)), ("x3w", torch.zeros(3)), ("x3", None)):
        with pytest.raises(ValueError, match="act16 input needs"):
            ServerStage(device="cpu", conv=conv).forward_backward(None, y, 1.0, act_amax=amax, act16=img)
    with pytest.raises(ValueError, match="act=None needs"):
        ops.conv2_wgrad_slabs(None, torch.zeros(3, 9216), torch.zeros(3, 64, 12, 12, dtype=torch.uint8), impl="x3")
