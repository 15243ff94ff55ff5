"""Lossless sparse codec for the multi-GPU cut exchange (csrc/slk_codec.hip).

The reference ships the dense fp32 cut and the dense fp32 cut gradient (src/client_part.py:117-125,
src/server_part.py:57-58). The cut is a ReLU output, so on the RCCL path a micro-batch travels as a
bit mask of its nonzero elements plus those elements in order, and the gradient as its values at the
same positions only: the client applies its own ReLU mask before using the gradient (ReLU's backward
in activations.backward, src/client_part.py:132), so the positions left out never reach a result.
Every weight, loss and gradient downstream is bit-identical to the dense exchange.
"""
from __future__ import annotations

import torch

from . import _lib
from .ops import _stream


class CutCodec:
    """Per micro-batch encode / offsets / pack / unpack over caller-visible buffers (one set per key)."""

    def __init__(self):
        self._bufs = {}

    def _buf(self, key, shape, dtype, device):
        # keyed by shape too: a buffer is never replaced, so a HIP graph captured around these kernels at
        # one micro-batch size keeps valid pointers after another size has run (dist.Hub's chunk graphs)
        k = (key, tuple(shape), dtype, str(torch.device(device)))
        t = self._bufs.get(k)
        if t is None:
            t = torch.empty(shape, dtype=dtype, device=device)
            self._bufs[k] = t
        return t

    def buffers(self, key, n: int, device):
        """(mask words, counts, offsets, total[1], vals[n]) for a micro-batch of n elements."""
        nb = _lib.query("slk_cut_blocks", n)
        return (self._buf((key, "mask"), ((n + 31) // 32,), torch.int32, device),
                self._buf((key, "counts"), (nb,), torch.int32, device),
                self._buf((key, "offsets"), (nb,), torch.int32, device),
                self._buf((key, "total"), (1,), torch.int32, device),
                self._buf((key, "vals"), (n,), torch.float32, device))

    def ranks_buffer(self, key, n: int, device):
        """The word-ranks buffer of key's micro-batch (int32, ceil(n/32)), not computed."""
        return self._buf((key, "ranks"), ((n + 31) // 32,), torch.int32, device)

    def ranks(self, key, n: int, bufs):
        """Word ranks of a micro-batch whose offsets are computed (offsets() / encode()): ranks[w] = the vals
        index of mask word w's first set element, for the fused consumers (ops.cut_unpack_x3,
        ops.conv2_dgrad_x3_pack). Buffer keyed like buffers()."""
        mask, _, offsets, _, _ = bufs
        r = self.ranks_buffer(key, n, mask.device)
        _lib.call("slk_cut_ranks", mask.data_ptr(), n, offsets.data_ptr(), r.data_ptr(), _stream(mask))
        return r

    @staticmethod
    def encode(x, bufs):
        mask, counts, offsets, total, vals = bufs
        _lib.call("slk_cut_encode", x.data_ptr(), x.numel(), mask.data_ptr(), counts.data_ptr(), offsets.data_ptr(),
                  total.data_ptr(), vals.data_ptr(), _stream(x))

    @staticmethod
    def offsets(n: int, bufs):
        mask, counts, offsets, total, _ = bufs
        _lib.call("slk_cut_offsets", mask.data_ptr(), n, counts.data_ptr(), offsets.data_ptr(), total.data_ptr(),
                  _stream(mask))

    @staticmethod
    def pack(x, bufs, vals=None):
        mask, _, offsets, _, v = bufs
        v = v if vals is None else vals
        _lib.call("slk_cut_pack", x.data_ptr(), x.numel(), mask.data_ptr(), offsets.data_ptr(), v.data_ptr(), _stream(x))

    @staticmethod
    def unpack(out, bufs, vals=None):
        mask, _, offsets, _, v = bufs
        v = v if vals is None else vals
        _lib.call("slk_cut_unpack", v.data_ptr(), out.numel(), mask.data_ptr(), offsets.data_ptr(), out.data_ptr(),
                  _stream(out))
