"""GPU parity of the lossless sparse cut codec (csrc/slk_codec.hip via splitcnn/codec.py).

The codec has no counterpart in the reference (which pickles the dense cut over HTTP,
src/client_part.py:117-125); its contract is plain bit arithmetic, so the checker is numpy:
  mask bit i  = (bit pattern of x[i] != 0)      little-endian within uint32 words
  counts[b]   = set bits of elements [2048 b, 2048 b + 2048)
  offsets     = exclusive scan of counts,  total = sum
  vals        = x[mask] in element order
  unpack      = x where the bit is set, +0.0 elsewhere;  pack(g) = g[mask]
All bit-exact. Sizes cover ragged tails (n not a multiple of 32 / 64 / 2048), one element, more
blocks than the scan's 1024 threads, -0.0 (nonzero bit pattern, kept), NaN/inf/denormals, all-zero
and all-set inputs, and a full B = 1024 micro-batch of the K3 cut (22,151,168 elements)."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

CB = 2048


def _expect(x):
    bits = x.view(np.uint32)
    set_ = bits != 0
    n = x.size
    pad = np.zeros(((n + 31) // 32) * 32, dtype=bool)
    pad[:n] = set_
    words = np.packbits(pad.reshape(-1, 32)[:, ::-1], axis=1).view(">u4").ravel().astype(np.uint32)
    nb = (n + CB - 1) // CB
    cpad = np.zeros(nb * CB, dtype=np.int64)
    cpad[:n] = set_
    counts = cpad.reshape(nb, CB).sum(1)
    offsets = np.concatenate([[0], np.cumsum(counts)[:-1]]) if nb else counts
    return set_, words, counts, offsets, int(set_.sum())


def _input(n, kind, seed):
    rng = np.random.default_rng(seed)
    x = rng.standard_normal(n).astype(np.float32)
    if kind == "relu":
        x = np.maximum(x, 0).astype(np.float32)
    elif kind == "zeros":
        x[:] = 0
    elif kind == "dense":
        x = np.abs(x) + 1
    elif kind == "special":
        x = np.maximum(x, 0).astype(np.float32)
        pick = rng.integers(0, n, size=max(1, n // 16))
        x[pick] = rng.choice(np.array([-0.0, np.nan, np.inf, -np.inf, 1e-45, -1e-45], dtype=np.float32), size=pick.size)
    return x.astype(np.float32)


CASES = [(1, "dense"), (31, "relu"), (33, "relu"), (64, "special"), (2047, "relu"), (2048, "zeros"), (2049, "special"),
         (65_541, "relu"), (2048 * 1100 + 7, "special"), (3_000_017, "dense"), (1024 * 32 * 26 * 26, "relu")]


@pytest.mark.parametrize("n,kind", CASES)
def test_codec_roundtrip_vs_numpy(gpu, n, kind):
    from splitcnn.codec import CutCodec
    codec = CutCodec()
    x = _input(n, kind, n)
    g = np.random.default_rng(n + 1).standard_normal(n).astype(np.float32)
    set_, words, counts, offsets, total = _expect(x)
    xd, gd = torch.from_numpy(x).to(gpu), torch.from_numpy(g).to(gpu)
    bufs = codec.buffers("tx", n, gpu)
    codec.encode(xd, bufs)
    mask, cnt, off, tot, vals = bufs
    torch.cuda.synchronize()
    assert np.array_equal(mask.cpu().numpy().view(np.uint32), words)
    assert np.array_equal(cnt.cpu().numpy(), counts) and np.array_equal(off.cpu().numpy(), offsets)
    assert int(tot.item()) == total
    assert np.array_equal(vals[:total].cpu().numpy().view(np.uint32), x.view(np.uint32)[set_])

    # receiving side: offsets from the mask alone, then unpack
    rx = codec.buffers("rx", n, gpu)
    rx[0].copy_(mask)
    rx[4][:total].copy_(vals[:total])
    codec.offsets(n, rx)
    out = torch.full((n,), 7.0, device=gpu)
    codec.unpack(out, rx)
    torch.cuda.synchronize()
    assert np.array_equal(rx[2].cpu().numpy(), offsets) and int(rx[3].item()) == total
    want = np.where(set_, x, np.float32(0)).astype(np.float32)
    assert np.array_equal(out.cpu().numpy().view(np.uint32), want.view(np.uint32))

    # gradient direction: pack g at the mask positions, unpack on the other side
    gv = torch.empty(n, device=gpu)
    codec.pack(gd, rx, vals=gv)
    gout = torch.full((n,), 7.0, device=gpu)
    codec.unpack(gout, bufs, vals=gv)
    torch.cuda.synchronize()
    assert np.array_equal(gv[:total].cpu().numpy().view(np.uint32), g.view(np.uint32)[set_])
    assert np.array_equal(gout.cpu().numpy().view(np.uint32), np.where(set_, g, np.float32(0)).view(np.uint32))


def test_codec_empty_is_a_noop(gpu):
    from splitcnn import _lib
    assert _lib.query("slk_cut_blocks", 0) == 0
    from splitcnn.codec import CutCodec
    codec = CutCodec()
    x = torch.empty(0, device=gpu)
    bufs = codec.buffers("e", 0, gpu)
    codec.encode(x, bufs)
    codec.unpack(x, bufs)
    torch.cuda.synchronize()


def test_codec_of_a_real_cut(gpu):
    """The cut of the reference model (conv1 + ReLU of MNIST-shaped input): about half the
    elements are zero, so each direction moves ~(density + 1/32) of the dense bytes."""
    from splitcnn.engine import ClientStage
    from splitcnn.model_def import ModelPartA
    from splitcnn.codec import CutCodec
    torch.manual_seed(0)
    c = ClientStage(ModelPartA(), device=gpu)
    x = torch.rand(64, 1, 28, 28, device=gpu)
    act = c.forward(x)
    n = act.numel()
    codec = CutCodec()
    bufs = codec.buffers("a", n, gpu)
    codec.encode(act, bufs)
    torch.cuda.synchronize()
    total = int(bufs[3].item())
    assert total == int((act.view(torch.int32) != 0).sum().item())
    assert 0.2 * n < total < 0.8 * n
