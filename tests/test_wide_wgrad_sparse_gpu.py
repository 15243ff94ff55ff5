"""The K5 weight gradients on the 2:4-sparse bf16 MFMA (round 6, csrc/slk_wide.hip wide_wgrad_kernel<C, true>)
at sizes where every K share runs many tiles, against a float64 torch reference on the same operands.

The kernels take the POOLED output gradient + its routing code (codes 0-3 = window position 2 dy + dx, 4 = blocked)
and never see the unpooled gradient; the reference unpools it explicitly and forms dW = sum_p dC[co][p] x
In[ci][p + tap - 1] (padding 1) as a float64 GEMM over an unfolded input, db = sum dC. Both sides multiply bf16
values exactly and sum in f32 (kernel) / f64 (reference), so the bar is the f32 accumulation floor: 1e-5 of the
gradient's max (as tests/test_wide_gpu.py). Random operands: every routing position and blocked windows occur,
including windows of one channel routed differently from their neighbours, which is what the compressed records
and their index words encode. Ragged B leaves most of the 256 K shares with zero or one tile.
"""
import pytest
import torch

pytestmark = pytest.mark.gpu


def _unpool(pooled_nchw, code_nchw):
    """max-pool backward: the pooled value at window position code (0-3), nothing where code == 4."""
    B, C, H, W = pooled_nchw.shape
    out = torch.zeros(B, C, 2 * H, 2 * W, dtype=pooled_nchw.dtype, device=pooled_nchw.device)
    for pos in range(4):
        dy, dx = pos >> 1, pos & 1
        out[:, :, dy::2, dx::2] = torch.where(code_nchw == pos, pooled_nchw, torch.zeros_like(pooled_nchw))
    return out


def _ref_wgrad(inp_nchw, dC):
    """[dW (co, ci, 3, 3) | db (co)] in float64: dW = dC @ unfold(inp)^T summed over the batch."""
    B, CI, H, W = inp_nchw.shape
    CO = dC.shape[1]
    dW = torch.zeros(CO, CI * 9, dtype=torch.float64, device=dC.device)
    for b0 in range(0, B, 64):  # bounded memory
        u = torch.nn.functional.unfold(inp_nchw[b0:b0 + 64].double(), 3, padding=1)  # [b, CI*9, H*W]
        d = dC[b0:b0 + 64].double().reshape(-1, CO, H * W)
        dW += torch.einsum("bcp,bkp->ck", d, u)
    return torch.cat([dW.reshape(-1), dC.double().sum((0, 2, 3))])


def _case(B, layer, seed):
    from splitcnn import _lib
    from splitcnn.wide import c8_to_nchw
    dev = torch.device("cuda:0")
    g = torch.Generator(device=dev).manual_seed(seed)
    if layer == 2:   # conv2: in = a1 [B, 64, 32, 32], dC pooled = dp2 [B, 128, 16, 16]
        CI, CO, HW = 64, 128, 32
    else:            # conv3: in = p2 [B, 128, 16, 16], dC pooled = dcut [B, 256, 8, 8]
        CI, CO, HW = 128, 256, 16
    inp = (torch.randn(B, CI // 8, HW, HW, 8, device=dev, generator=g)).abs().to(torch.bfloat16)
    dp = (torch.randn(B, CO // 8, HW // 2, HW // 2, 8, device=dev, generator=g) * 1e-2).to(torch.bfloat16)
    code = torch.randint(0, 5, (B, CO // 8, HW // 2, HW // 2, 8), device=dev, generator=g).to(torch.uint8)
    nslab = _lib.query(f"slk_wide_conv{layer}_wgrad_nslab", B)
    slabs = torch.full((nslab, CO * CI * 9 + CO), float("nan"), device=dev)
    s = torch.cuda.current_stream().cuda_stream
    _lib.call(f"slk_wide_conv{layer}_wgrad", dp.data_ptr(), code.data_ptr(), inp.data_ptr(), slabs.data_ptr(), B, s)
    got = slabs.double().sum(0)
    dC = _unpool(c8_to_nchw(dp).float(), c8_to_nchw(code))
    want = _ref_wgrad(c8_to_nchw(inp).float(), dC)
    return got, want


@pytest.mark.parametrize("layer", [2, 3])
@pytest.mark.parametrize("B", [37, 512])
def test_sparse_wgrad_vs_float64(gpu, layer, B):
    from splitcnn import _lib
    assert _lib.query("slk_wide_wgrad_form") == 1
    got, want = _case(B, layer, seed=11 + B + layer)
    assert torch.isfinite(got).all(), "a slab was left unwritten"
    err = (got - want).abs().max().item()
    scale = want.abs().max().item()
    assert err <= 1e-5 * scale, (err, scale)
