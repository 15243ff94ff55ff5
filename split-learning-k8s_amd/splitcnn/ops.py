"""Tensor-level wrappers over the libslk.so C-ABI (include/slk.h).

Every function takes device tensors, checks device / dtype / shape / contiguity on the host (the
kernels assume the exact shapes of src/model_def.py), allocates outputs and workspaces with torch's
caching allocator when the caller does not pass them, and launches on torch's current HIP stream.
Nothing here synchronises, so a sequence of these calls can be captured in a HIP graph.
"""
from __future__ import annotations

import ctypes

import torch

from . import _lib

CLIENT_NPARAM = 320
SERVER_NPARAM = 110666
OFF_W2, OFF_B2, OFF_W3, OFF_B3 = 0, 18432, 18496, 110656
CONV2_SLAB = 18496   # [dW2 | db2]
FC_SLAB = 92170      # [dW3 | db3]

_F32 = torch.float32


def _stream(t: torch.Tensor) -> int:
    return torch.cuda.current_stream(t.device).cuda_stream


def _dev(t: torch.Tensor, name: str, shape=None, dtype=_F32) -> int:
    if not isinstance(t, torch.Tensor):
        raise TypeError(f"{name}: expected a torch.Tensor")
    if t.device.type != "cuda":
        raise RuntimeError(
            f"splitcnn: {name} is on {t.device}; the split-CNN ops run only on the MI355X HIP kernels "
            "(move the module and its inputs to a ROCm device). There is no CPU fallback.")
    if t.dtype != dtype:
        raise TypeError(f"{name}: expected {dtype}, got {t.dtype}")
    if shape is not None and tuple(t.shape) != tuple(shape):
        raise ValueError(f"{name}: expected shape {tuple(shape)}, got {tuple(t.shape)}")
    if not t.is_contiguous():
        raise ValueError(f"{name}: must be contiguous")
    return t.data_ptr()


def _out(out, shape, like, dtype=_F32, name="out"):
    if out is None:
        return torch.empty(shape, dtype=dtype, device=like.device)
    _dev(out, name, shape, dtype)
    return out


def batch_of(x: torch.Tensor, tail: tuple, name: str) -> int:
    if x.dim() != 1 + len(tail) or tuple(x.shape[1:]) != tail:
        raise ValueError(f"{name}: expected shape [B,{','.join(map(str, tail))}], got {tuple(x.shape)}")
    return int(x.shape[0])


# ------------------------------------------------------------------------------------ client stage
def conv1_fwd(x, W1, b1, out=None, act_amax=None):
    """act = relu(conv1(x)); with act_amax (a [B] f32 tensor) also its per-sample x3 SCALE BOUND, fused:
    conv1_cut_bound (csrc/slk_common.h) = max_c (sum |W1[c]| * max |x| + max(b1[c], 0)) >= max act, not the
    max itself (only its power of two is used)."""
    B = batch_of(x, (1, 28, 28), "x")
    act = _out(out, (B, 32, 26, 26), x)
    if act_amax is not None:
        _lib.call("slk_conv1_fwd_amax", _dev(x, "x"), _dev(W1, "conv1.weight", (32, 1, 3, 3)),
                  _dev(b1, "conv1.bias", (32,)), _dev(act, "act"), _dev(act_amax, "act_amax", (B,)), B, _stream(x))
        return act
    _lib.call("slk_conv1_fwd", _dev(x, "x"), _dev(W1, "conv1.weight", (32, 1, 3, 3)),
              _dev(b1, "conv1.bias", (32,)), _dev(act, "act"), B, _stream(x))
    return act


RELU_BITS_WORDS = 676  # int32 words of the cut's ReLU bit map per sample (slk_relu_bits_bytes / 4)


def relu_bits_buffer(B: int, device) -> torch.Tensor:
    return torch.empty((B, RELU_BITS_WORDS), dtype=torch.int32, device=device)


def conv1_fwd_x3(x, W1, b1, act_amax, act16, act=None, relu_bits=None):
    """conv1 + ReLU writing the x3 server operand: act_amax [B] (the per-sample scale bound
    conv1_cut_bound, >= max act; see conv1_fwd) and the act16 images
    (conv2_act16_bytes(B) uint8), plus the f32 act when `act` is given and the cut's ReLU bit map
    (int32 [B, RELU_BITS_WORDS], the fused client backward's mask) when `relu_bits` is. Returns act (or None)."""
    B = batch_of(x, (1, 28, 28), "x")
    ap = _dev(act, "act", (B, 32, 26, 26)) if act is not None else None
    bp = _dev(relu_bits, "relu_bits", (B, RELU_BITS_WORDS), torch.int32) if relu_bits is not None else None
    _lib.call("slk_conv1_fwd_x3", _dev(x, "x"), _dev(W1, "conv1.weight", (32, 1, 3, 3)), _dev(b1, "conv1.bias", (32,)),
              ap, _dev(act_amax, "act_amax", (B,)), _act16(act16, B), bp, B, _stream(x))
    return act


def conv2_fwd_pool_x3i(act16, act_amax, W2, b2, pooled=None, code=None):
    """The x3 forward + pool reading the act16 images (conv1_fwd_x3 / conv2_fwd_pool(act16=...)) instead
    of the f32 act: the same pooled / code bitwise."""
    B = batch_of(act_amax, (), "act_amax")
    pooled = _out(pooled, (B, 64, 12, 12), act_amax, name="pooled")
    code = _out(code, (B, 64, 12, 12), act_amax, torch.uint8, "code")
    _lib.call("slk_conv2_fwd_pool_x3i", _act16(act16, B), _dev(act_amax, "act_amax", (B,)),
              _dev(W2, "conv2.weight", (64, 32, 3, 3)), _dev(b2, "conv2.bias", (64,)), _dev(pooled, "pooled"),
              _dev(code, "code", dtype=torch.uint8), B, _stream(act_amax))
    return pooled, code


def conv2_dgrad_c1w_nslab(B: int) -> int:
    return _lib.query("slk_conv2_dgrad_x3_c1w_nslab", B)


def conv2_dgrad_client_slabs(dpooled, code, W2, x, relu_bits, dp_amax=None, slabs=None):
    """x3 dgrad fused with the client's ReLU backward + conv1 wgrad: returns the client's gradient
    slabs [conv2_dgrad_c1w_nslab(B), 320] (conv1_wgrad_slabs' layout); the cut gradient is not
    materialised. relu_bits: the ReLU bit map conv1_fwd_x3 wrote for this cut."""
    B = _pooled_batch(dpooled)
    batch_of(x, (1, 28, 28), "x")
    if x.shape[0] != B:
        raise ValueError("x / dpooled batch mismatch")
    dp_amax = row_amax(dpooled) if dp_amax is None else dp_amax
    slabs = _out(slabs, (conv2_dgrad_c1w_nslab(B), CLIENT_NPARAM), x, name="slabs")
    _lib.call("slk_conv2_dgrad_x3_c1w", _dev(dpooled, "dpooled"), _dev(dp_amax, "dp_amax", (B,)),
              _dev(code, "code", (B, 64, 12, 12), torch.uint8), _dev(W2, "conv2.weight", (64, 32, 3, 3)),
              _dev(x, "x"), _dev(relu_bits, "relu_bits", (B, RELU_BITS_WORDS), torch.int32),
              _dev(slabs, "slabs"), B, _stream(x))
    return slabs


def conv1_wgrad_nslab(B: int) -> int:
    return _lib.query("slk_conv1_wgrad_nslab", B)


def conv1_wgrad_slabs(x, act, cut_grad, slabs=None):
    B = batch_of(x, (1, 28, 28), "x")
    nslab = conv1_wgrad_nslab(B)
    slabs = _out(slabs, (nslab, CLIENT_NPARAM), x, name="slabs")
    _lib.call("slk_conv1_wgrad", _dev(x, "x"), _dev(act, "act", (B, 32, 26, 26)),
              _dev(cut_grad, "cut_grad", (B, 32, 26, 26)), _dev(slabs, "slabs"), B, _stream(x))
    return slabs


def conv1_wgrad_remask_slabs(x, W1, b1, cut_grad, slabs=None):
    """conv1_wgrad_slabs with the ReLU mask recomputed from x, W1, b1 (bit-identical to act > 0 for
    the forward's weights): half the HBM traffic, act is not read."""
    B = batch_of(x, (1, 28, 28), "x")
    nslab = conv1_wgrad_nslab(B)
    slabs = _out(slabs, (nslab, CLIENT_NPARAM), x, name="slabs")
    _lib.call("slk_conv1_wgrad_remask", _dev(x, "x"), _dev(W1, "conv1.weight", (32, 1, 3, 3)),
              _dev(b1, "conv1.bias", (32,)), _dev(cut_grad, "cut_grad", (B, 32, 26, 26)), _dev(slabs, "slabs"),
              B, _stream(x))
    return slabs


# ------------------------------------------------------------------------------------ server stage
def row_amax(x, out=None):
    """out[r] = max |x[r]| over each row of a [rows, ...] tensor (the x3 kernels' per-sample scales)."""
    rows = int(x.shape[0])
    n = x.numel() // max(rows, 1)
    out = _out(out, (rows,), x, name="amax")
    _lib.call("slk_row_amax", _dev(x, "x"), rows, n, _dev(out, "amax"), _stream(x))
    return out


def _impl(direct, impl):
    if impl is None:
        return "direct" if direct else "wino"
    if impl not in ("wino", "direct", "x3"):
        raise ValueError(f"conv2 impl must be 'wino', 'direct' or 'x3', got {impl!r}")
    return impl


def conv2_act16_bytes(B: int) -> int:
    """Bytes of the f16 input images conv2_fwd_pool(impl='x3', act16=...) writes for the x3 wgrad."""
    return _lib.query("slk_conv2_act16_bytes", B)


def _act16(t, B):
    _dev(t, "act16", (conv2_act16_bytes(B),), torch.uint8)
    return t.data_ptr()


def conv2_fwd_pool(act, W2, b2, pooled=None, code=None, direct=False, impl=None, act_amax=None, act16=None,
                   act_amax_out=None):
    """impl: 'wino' (Winograd F(2x2,3x3) on the f32 MFMA, default), 'direct' (direct f32 MFMA kernel,
    cross-check; also direct=True) or 'x3' (direct on the f16 MFMA with split operands; act_amax = a
    per-sample scale bound >= max |act| — the client's conv1_cut_bound, or the exact max (row_amax), computed
    here when not given; only its power of two matters). act16 (x3 only, a uint8 tensor of
    conv2_act16_bytes(B)): also write the split input images for conv2_wgrad_slabs(act16=...).
    act_amax_out (x3 with act16, act_amax not given; a float tensor [B]): the forward kernel computes the
    per-sample max itself and writes it there (slk_conv2_fwd_pool_x3sa: no separate pass over act; the
    same values as row_amax, so the same outputs bitwise)."""
    impl = _impl(direct, impl)
    B = batch_of(act, (32, 26, 26), "act")
    if act_amax_out is not None and impl != "x3":
        raise ValueError("act_amax_out is an output of the x3 forward only")
    pooled = _out(pooled, (B, 64, 12, 12), act, name="pooled")
    code = _out(code, (B, 64, 12, 12), act, torch.uint8, "code")
    if impl == "x3":
        if act_amax_out is not None:
            if act_amax is not None or act16 is None:
                raise ValueError("act_amax_out needs act16 and no act_amax")
            _lib.call("slk_conv2_fwd_pool_x3sa", _dev(act, "act"), _dev(act_amax_out, "act_amax_out", (B,)),
                      _dev(W2, "conv2.weight", (64, 32, 3, 3)), _dev(b2, "conv2.bias", (64,)), _dev(pooled, "pooled"),
                      _dev(code, "code", dtype=torch.uint8), _act16(act16, B), B, _stream(act))
            return pooled, code
        if act_amax is None:
            act_amax = row_amax(act)
        if act16 is not None:
            _lib.call("slk_conv2_fwd_pool_x3s", _dev(act, "act"), _dev(act_amax, "act_amax", (B,)),
                      _dev(W2, "conv2.weight", (64, 32, 3, 3)), _dev(b2, "conv2.bias", (64,)), _dev(pooled, "pooled"),
                      _dev(code, "code", dtype=torch.uint8), _act16(act16, B), B, _stream(act))
            return pooled, code
        _lib.call("slk_conv2_fwd_pool_x3", _dev(act, "act"), _dev(act_amax, "act_amax", (B,)),
                  _dev(W2, "conv2.weight", (64, 32, 3, 3)), _dev(b2, "conv2.bias", (64,)), _dev(pooled, "pooled"),
                  _dev(code, "code", dtype=torch.uint8), B, _stream(act))
        return pooled, code
    _lib.call("slk_conv2_fwd_pool_direct" if impl == "direct" else "slk_conv2_fwd_pool", _dev(act, "act"),
              _dev(W2, "conv2.weight", (64, 32, 3, 3)), _dev(b2, "conv2.bias", (64,)), _dev(pooled, "pooled"),
              _dev(code, "code", dtype=torch.uint8), B, _stream(act))
    return pooled, code


def _pooled_batch(pooled):
    if pooled.dim() == 2:
        return batch_of(pooled, (9216,), "pooled")
    return batch_of(pooled, (64, 12, 12), "pooled")


def fc_fwd(pooled, W3, b3, out=None):
    B = _pooled_batch(pooled)
    logits = _out(out, (B, 10), pooled)
    _lib.call("slk_fc_fwd", _dev(pooled, "pooled"), _dev(W3, "fc1.weight", (10, 9216)),
              _dev(b3, "fc1.bias", (10,)), _dev(logits, "logits"), B, _stream(pooled))
    return logits


def fc_logits_xent(pooled, W3, b3, labels, grad_scale, logits=None, loss_i=None, dlogits=None, err_flag=None):
    """fc_fwd + xent_fwd_bwd in one launch (slk_fc_logits_xent), bitwise their outputs."""
    B = _pooled_batch(pooled)
    logits = _out(logits, (B, 10), pooled, name="logits")
    loss_i = _out(loss_i, (B,), pooled, name="loss_i")
    dlogits = _out(dlogits, (B, 10), pooled, name="dlogits")
    eptr = _dev(err_flag, "err_flag", (1,), torch.int32) if err_flag is not None else None
    _lib.call("slk_fc_logits_xent", _dev(pooled, "pooled"), _dev(W3, "fc1.weight", (10, 9216)),
              _dev(b3, "fc1.bias", (10,)), _labels(labels, B), _dev(logits, "logits"), _dev(loss_i, "loss_i"),
              _dev(dlogits, "dlogits"), float(grad_scale), eptr, B, _stream(pooled))
    return logits, loss_i, dlogits


def _labels(labels, B):
    _dev(labels, "labels", (B,), torch.int64)
    return labels.data_ptr()


def xent_fwd_bwd(logits, labels, grad_scale, loss_i=None, dlogits=None, err_flag=None):
    B = batch_of(logits, (10,), "logits")
    loss_i = _out(loss_i, (B,), logits, name="loss_i")
    dlogits = _out(dlogits, (B, 10), logits, name="dlogits")
    eptr = _dev(err_flag, "err_flag", (1,), torch.int32) if err_flag is not None else None
    _lib.call("slk_xent_fwd_bwd", _dev(logits, "logits"), _labels(labels, B), _dev(loss_i, "loss_i"),
              _dev(dlogits, "dlogits"), float(grad_scale), eptr, B, _stream(logits))
    return loss_i, dlogits


def fc_dgrad(dlogits, W3, out=None, dp_amax=None):
    """dp_amax (a [B] f32 tensor): also write the per-sample max |dpooled|, fused."""
    B = batch_of(dlogits, (10,), "dlogits")
    dpooled = _out(out, (B, 9216), dlogits, name="dpooled")
    if dp_amax is None:
        _lib.call("slk_fc_dgrad", _dev(dlogits, "dlogits"), _dev(W3, "fc1.weight", (10, 9216)),
                  _dev(dpooled, "dpooled"), B, _stream(dlogits))
    else:
        _lib.call("slk_fc_dgrad_amax", _dev(dlogits, "dlogits"), _dev(W3, "fc1.weight", (10, 9216)),
                  _dev(dpooled, "dpooled"), _dev(dp_amax, "dp_amax", (B,)), B, _stream(dlogits))
    return dpooled


def fc_xent(pooled, W3, b3, labels, grad_scale, logits=None, loss_i=None, dlogits=None,
            dpooled=None, err_flag=None, dp_amax=None):
    """dp_amax (a [B] f32 tensor): also write the per-sample max |dpooled|, fused."""
    B = _pooled_batch(pooled)
    logits = _out(logits, (B, 10), pooled, name="logits")
    loss_i = _out(loss_i, (B,), pooled, name="loss_i")
    dlogits = _out(dlogits, (B, 10), pooled, name="dlogits")
    dpooled = _out(dpooled, tuple(pooled.shape), pooled, name="dpooled")
    eptr = _dev(err_flag, "err_flag", (1,), torch.int32) if err_flag is not None else None
    if dp_amax is not None:
        _lib.call("slk_fc_xent_amax", _dev(pooled, "pooled"), _dev(W3, "fc1.weight", (10, 9216)),
                  _dev(b3, "fc1.bias", (10,)), _labels(labels, B), _dev(logits, "logits"),
                  _dev(loss_i, "loss_i"), _dev(dlogits, "dlogits"), _dev(dpooled, "dpooled"),
                  _dev(dp_amax, "dp_amax", (B,)), float(grad_scale), eptr, B, _stream(pooled))
        return logits, loss_i, dlogits, dpooled
    _lib.call("slk_fc_xent", _dev(pooled, "pooled"), _dev(W3, "fc1.weight", (10, 9216)),
              _dev(b3, "fc1.bias", (10,)), _labels(labels, B), _dev(logits, "logits"),
              _dev(loss_i, "loss_i"), _dev(dlogits, "dlogits"), _dev(dpooled, "dpooled"),
              float(grad_scale), eptr, B, _stream(pooled))
    return logits, loss_i, dlogits, dpooled


def fc_wgrad_nslab(B: int) -> int:
    return _lib.query("slk_fc_wgrad_nslab", B)


def fc_wgrad_slabs(dlogits, pooled, slabs=None):
    B = batch_of(dlogits, (10,), "dlogits")
    if _pooled_batch(pooled) != B:
        raise ValueError("pooled / dlogits batch mismatch")
    slabs = _out(slabs, (fc_wgrad_nslab(B), FC_SLAB), dlogits, name="slabs")
    _lib.call("slk_fc_wgrad", _dev(dlogits, "dlogits"), _dev(pooled, "pooled"), _dev(slabs, "slabs"),
              B, _stream(dlogits))
    return slabs


def _dpooled_batch(dpooled):
    return _pooled_batch(dpooled)


def conv2_dgrad(dpooled, code, W2, out=None, direct=False, impl=None, dp_amax=None):
    impl = _impl(direct, impl)
    B = _dpooled_batch(dpooled)
    cut_grad = _out(out, (B, 32, 26, 26), dpooled, name="cut_grad")
    if impl == "x3":
        if dp_amax is None:
            dp_amax = row_amax(dpooled)
        _lib.call("slk_conv2_dgrad_x3", _dev(dpooled, "dpooled"), _dev(dp_amax, "dp_amax", (B,)),
                  _dev(code, "code", (B, 64, 12, 12), torch.uint8), _dev(W2, "conv2.weight", (64, 32, 3, 3)),
                  _dev(cut_grad, "cut_grad"), B, _stream(dpooled))
        return cut_grad
    direct = impl == "direct"
    _lib.call("slk_conv2_dgrad_direct" if direct else "slk_conv2_dgrad", _dev(dpooled, "dpooled"),
              _dev(code, "code", (B, 64, 12, 12), torch.uint8), _dev(W2, "conv2.weight", (64, 32, 3, 3)),
              _dev(cut_grad, "cut_grad"), B, _stream(dpooled))
    return cut_grad


def conv2_dgrad_x3_pack(dpooled, code, W2, dp_amax, mask, ranks, vals):
    """The x3 cut gradient in the codec's packed form (slk_conv2_dgrad_x3_pack): the values of the elements
    set in `mask` (the received cut's: int32 words, ceil(B*21632/32)) at their word ranks (cut_ranks), into
    `vals` — what CutCodec.pack extracts from conv2_dgrad(..., impl="x3") without the dense gradient."""
    B = _dpooled_batch(dpooled)
    nw = (B * 21632 + 31) // 32
    _lib.call("slk_conv2_dgrad_x3_pack", _dev(dpooled, "dpooled"), _dev(dp_amax, "dp_amax", (B,)),
              _dev(code, "code", (B, 64, 12, 12), torch.uint8), _dev(W2, "conv2.weight", (64, 32, 3, 3)),
              _dev(mask, "mask", (nw,), torch.int32), _dev(ranks, "ranks", (nw,), torch.int32),
              _dev(vals, "vals"), B, _stream(dpooled))
    return vals


def conv2_dgrad_x3_pack_parts(dpooled, code, W2, dp_amax, parts, part_b):
    """conv2_dgrad_x3_pack over the B / part_b parts of a server chunk in one launch: parts = int64 device
    table [B / part_b, 3] of (mask, ranks, vals) pointers (slk_conv2_dgrad_x3_pack_parts)."""
    B = _dpooled_batch(dpooled)
    if part_b <= 0 or B % part_b:
        raise ValueError(f"part_b {part_b} must divide the chunk's {B} samples")
    _lib.call("slk_conv2_dgrad_x3_pack_parts", _dev(dpooled, "dpooled"), _dev(dp_amax, "dp_amax", (B,)),
              _dev(code, "code", (B, 64, 12, 12), torch.uint8), _dev(W2, "conv2.weight", (64, 32, 3, 3)),
              _dev(parts, "parts", (B // part_b, 3), torch.int64), part_b, B, _stream(dpooled))


def cut_unpack_x3_parts(parts, part_b, act_amax, act16):
    """cut_unpack_x3 over the B / part_b parts of a server chunk in one launch: parts = int64 device table
    [B / part_b, 3] of (vals, mask, ranks) pointers (slk_cut_unpack_x3_parts)."""
    B = batch_of(act_amax, (), "act_amax")
    if part_b <= 0 or B % part_b:
        raise ValueError(f"part_b {part_b} must divide the chunk's {B} samples")
    _lib.call("slk_cut_unpack_x3_parts", _dev(parts, "parts", (B // part_b, 3), torch.int64), part_b,
              _dev(act_amax, "act_amax", (B,)), B, _act16(act16, B), _stream(act_amax))
    return act16


def cut_offsets_ranks_parts(parts, n):
    """Counts, offsets, totals and word ranks of every part of a chunk from its received mask, three launches
    for all parts: parts = int64 device table [np, 5] of (mask, counts, offsets, total, ranks) pointers."""
    _lib.call("slk_cut_offsets_ranks_parts", _dev(parts, "parts", (parts.shape[0], 5), torch.int64), parts.shape[0], n,
              _stream(parts))


def mfma_probe_tflops(device=None, iters: int = 40000, reps: int = 3) -> float:
    """Measurement only: this device's sustained dense f16 MFMA rate in TFLOP/s (slk_mfma_probe: 6 independent
    v_mfma_f32_16x16x32_f16 chains per wave on varied operands, 2 waves per SIMD on every CU), median of
    `reps` launches timed with HIP events on the current stream."""
    dev = torch.device(device) if device is not None else torch.device("cuda", torch.cuda.current_device())
    nb = _lib.query("slk_mfma_probe_blocks")
    out = torch.empty(nb * 256, device=dev)
    st = torch.cuda.current_stream(dev)
    _lib.call("slk_mfma_probe", out.data_ptr(), iters, st.cuda_stream)   # warm-up (clocks ramp)
    ts = []
    for _ in range(reps):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(st)
        _lib.call("slk_mfma_probe", out.data_ptr(), iters, st.cuda_stream)
        e1.record(st)
        e1.synchronize()
        ts.append(e0.elapsed_time(e1))
    ms = sorted(ts)[len(ts) // 2]
    return nb * 4 * iters * 6 * 16384 / (ms * 1e-3) / 1e12


def cut_unpack_x3(vals, mask, ranks, act_amax, act16):
    """A received codec micro-batch (mask + values + word ranks, B samples) -> the x3 input images act16
    (conv2_act16_bytes(B) uint8) at the scales act_amax: conv1_fwd_x3's images of the same cut, bit for bit."""
    B = batch_of(act_amax, (), "act_amax")
    nw = (B * 21632 + 31) // 32
    _lib.call("slk_cut_unpack_x3", _dev(vals, "vals"), _dev(mask, "mask", (nw,), torch.int32),
              _dev(ranks, "ranks", (nw,), torch.int32), _dev(act_amax, "act_amax", (B,)), B, _act16(act16, B),
              _stream(act_amax))
    return act16


def conv2_wgrad_nslab(B: int, direct: bool = False, impl=None) -> int:
    impl = _impl(direct, impl)
    return _lib.query({"wino": "slk_conv2_wgrad_nslab", "direct": "slk_conv2_wgrad_direct_nslab",
                       "x3": "slk_conv2_wgrad_x3_nslab"}[impl], B)


def conv2_wgrad_slabs(act, dpooled, code, slabs=None, direct=False, impl=None, act_amax=None, dp_amax=None,
                      act16=None):
    """act16 (x3 only): the forward's split input images (conv2_fwd_pool(..., act16=...), same act and
    act_amax, or conv1_fwd_x3) — the kernel then moves them by LDS-DMA instead of loading and splitting
    act, and act may be None (act_amax is then required)."""
    impl = _impl(direct, impl)
    if act is None:
        if impl != "x3" or act16 is None or act_amax is None:
            raise ValueError("conv2_wgrad_slabs: act=None needs impl='x3', act16 and act_amax")
        B = _dpooled_batch(dpooled)
    else:
        B = batch_of(act, (32, 26, 26), "act")
        if _dpooled_batch(dpooled) != B:
            raise ValueError("act / dpooled batch mismatch")
    slabs = _out(slabs, (conv2_wgrad_nslab(B, impl=impl), CONV2_SLAB), dpooled, name="slabs")
    if impl == "x3":
        act_amax = row_amax(act) if act_amax is None else act_amax
        dp_amax = row_amax(dpooled) if dp_amax is None else dp_amax
        if act16 is not None:
            _lib.call("slk_conv2_wgrad_x3s", _act16(act16, B), _dev(act_amax, "act_amax", (B,)),
                      _dev(dpooled, "dpooled"), _dev(dp_amax, "dp_amax", (B,)),
                      _dev(code, "code", (B, 64, 12, 12), torch.uint8), _dev(slabs, "slabs"), B, _stream(dpooled))
            return slabs
        _lib.call("slk_conv2_wgrad_x3", _dev(act, "act"), _dev(act_amax, "act_amax", (B,)), _dev(dpooled, "dpooled"),
                  _dev(dp_amax, "dp_amax", (B,)), _dev(code, "code", (B, 64, 12, 12), torch.uint8),
                  _dev(slabs, "slabs"), B, _stream(act))
        return slabs
    direct = impl == "direct"
    _lib.call("slk_conv2_wgrad_direct" if direct else "slk_conv2_wgrad", _dev(act, "act"), _dev(dpooled, "dpooled"),
              _dev(code, "code", (B, 64, 12, 12), torch.uint8), _dev(slabs, "slabs"), B, _stream(act))
    return slabs


# ------------------------------------------------------------------------------------ reductions
def reduce_slabs(slabs, out=None, accumulate=False):
    """out (+)= sum over slabs (fixed order)."""
    nslab, n = slabs.shape
    out = _out(out, (n,), slabs, name="out")
    _lib.call("slk_reduce_slabs", _dev(slabs, "slabs"), nslab, n, _dev(out, "out"), int(bool(accumulate)),
              _stream(slabs))
    return out


def sgd_from_slabs(param, grad, slabs, lr):
    """param -= lr * sum(slabs); grad = sum(slabs) (grad may be None). 1-D flat views."""
    nslab, n = slabs.shape
    _dev(param, "param", (n,))
    gptr = _dev(grad, "grad", (n,)) if grad is not None else None
    _lib.call("slk_sgd_from_slabs", param.data_ptr(), gptr, _dev(slabs, "slabs"), nslab, n, float(lr),
              _stream(param))


def sgd_multi_from_slabs(segments, lr, loss=None):
    """ONE launch for every optimizer step of a split step: for each (param, grad, slabs) in
    `segments` (<= 4) sgd_from_slabs(param, grad, slabs, lr), plus loss_log(*loss) when
    loss = (values, scale, ring, counter) — bit-identical to the separate launches. A segment whose
    param is None only reduces its slabs into grad (reduce_slabs of several buffers in one launch)."""
    k = len(segments)
    if not 0 <= k <= 4:
        raise ValueError("sgd_multi_from_slabs: at most 4 segments")
    P = ctypes.c_void_p
    params, grads, slabs = (P * 4)(), (P * 4)(), (P * 4)()
    nslab, ns = (ctypes.c_int * 4)(), (ctypes.c_int * 4)()
    stream_of = None
    for i, (param, grad, sl) in enumerate(segments):
        nsl, n = sl.shape
        if param is None and grad is None:
            raise ValueError("sgd_multi_from_slabs: a segment needs a param or a grad")
        params[i] = _dev(param, "param", (n,)) if param is not None else None
        grads[i] = _dev(grad, "grad", (n,)) if grad is not None else None
        slabs[i] = _dev(sl, "slabs")
        nslab[i], ns[i] = nsl, n
        stream_of = (param if param is not None else grad) if stream_of is None else stream_of
    lv, ln, lsc, ring, cap, ctr = None, 0, 0.0, None, 0, None
    if loss is not None:
        values, lsc, ring_t, counter = loss
        lv, ln = _dev(values, "values"), values.numel()
        ring, cap = _dev(ring_t, "ring"), ring_t.numel()
        ctr = _dev(counter, "counter", (1,), torch.int32)
        stream_of = values if stream_of is None else stream_of
    if stream_of is None:
        return
    cast = lambda a: ctypes.cast(a, P)  # noqa: E731
    _lib.call("slk_sgd_multi_from_slabs", cast(params), cast(grads), cast(slabs), cast(nslab), cast(ns), k,
              float(lr), lv, ln, float(lsc), ring, cap, ctr, _stream(stream_of))


def sgd(param, grad, lr):
    n = param.numel()
    _lib.call("slk_sgd", _dev(param, "param"), _dev(grad, "grad", tuple(param.shape)), n, float(lr),
              _stream(param))


def loss_sum(values, scale, out=None):
    """out[0] = scale * sum(values) (fixed order); out may be a 1-element view of a bigger buffer."""
    n = values.numel()
    if out is None:
        out = torch.empty(1, dtype=_F32, device=values.device)
    _dev(out, "out")
    _lib.call("slk_loss_sum", _dev(values, "values"), n, float(scale), out.data_ptr(), _stream(values))
    return out


def loss_mean(loss_i, out=None):
    return loss_sum(loss_i, 1.0 / loss_i.numel(), out)


def loss_log(values, scale, ring, counter):
    n = values.numel()
    _lib.call("slk_loss_log", _dev(values, "values"), n, float(scale), _dev(ring, "ring"), ring.numel(),
              _dev(counter, "counter", (1,), torch.int32), _stream(values))


# ------------------------------------------------------------------------------------ data
MNIST_MEAN, MNIST_STD = 0.1307, 0.3081   # client_part.py:63


def mnist_batch(images, labels, idx, x=None, y=None, err_flag=None, mean=MNIST_MEAN, std=MNIST_STD):
    """Gather + ToTensor + Normalize one batch from the HBM-resident u8 dataset (slk_mnist_batch)."""
    n = batch_of(images, (28, 28), "images")
    if labels.shape != (n,):
        raise ValueError(f"labels: expected shape ({n},), got {tuple(labels.shape)}")
    B = int(idx.shape[0])
    x = _out(x, (B, 1, 28, 28), images, name="x")
    y = _out(y, (B,), images, dtype=torch.int64, name="y")
    _lib.call("slk_mnist_batch", _dev(images, "images", dtype=torch.uint8),
              _dev(labels, "labels", dtype=torch.uint8), n, _dev(idx, "idx", (B,), torch.int64), B,
              float(mean), float(std), x.data_ptr(), y.data_ptr(),
              None if err_flag is None else _dev(err_flag, "err_flag", (1,), torch.int32), _stream(x))
    return x, y
