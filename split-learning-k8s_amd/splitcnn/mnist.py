"""Real-MNIST input path, offline: IDX files from a local path instead of the
reference's S3 cache / torchvision download (src/client_part.py:20-95), with its transform
ToTensor + Normalize((0.1307,), (0.3081,)) (client_part.py:61-64) and its
DataLoader(batch_size=64, shuffle=True) (client_part.py:98).

The u8 dataset is copied to HBM once (47 MB for the 60k training images); each batch is a single
`slk_mnist_batch` launch that gathers the shuffled rows and normalises them (bit-identical to the
torchvision transform), so the training loop never touches host memory per step.
"""
import gzip
import os
import struct
from typing import Iterator, Optional, Tuple

import numpy as np
import torch

from . import ops

_FILES = {True: ("train-images-idx3-ubyte", "train-labels-idx1-ubyte"),
          False: ("t10k-images-idx3-ubyte", "t10k-labels-idx1-ubyte")}
_DTYPES = {0x08: np.uint8, 0x09: np.int8, 0x0B: np.dtype(">i2"), 0x0C: np.dtype(">i4"),
           0x0D: np.dtype(">f4"), 0x0E: np.dtype(">f8")}


def read_idx(path: str) -> np.ndarray:
    """Parse an IDX file (optionally .gz): magic 00 00 <type> <ndim>, ndim big-endian u32 dims, data."""
    opener = gzip.open if path.endswith(".gz") else open
    with opener(path, "rb") as f:
        raw = f.read()
    if len(raw) < 4 or raw[0] != 0 or raw[1] != 0 or raw[2] not in _DTYPES:
        raise ValueError(f"{path}: not an IDX file")
    ndim = raw[3]
    dims = struct.unpack(f">{ndim}I", raw[4:4 + 4 * ndim])
    dt = np.dtype(_DTYPES[raw[2]])
    n = int(np.prod(dims)) if dims else 1
    off = 4 + 4 * ndim
    if len(raw) - off != n * dt.itemsize:
        raise ValueError(f"{path}: {len(raw) - off} data bytes for dims {dims} of {dt}")
    return np.frombuffer(raw, dtype=dt, count=n, offset=off).reshape(dims).copy()


def write_idx(path: str, arr: np.ndarray) -> None:
    """Write a u8 array as IDX (gzip if the name ends in .gz) — for fixtures and tests."""
    arr = np.ascontiguousarray(arr, dtype=np.uint8)
    head = bytes([0, 0, 0x08, arr.ndim]) + struct.pack(f">{arr.ndim}I", *arr.shape)
    opener = gzip.open if path.endswith(".gz") else open
    with opener(path, "wb") as f:
        f.write(head + arr.tobytes())


def _find(root: str, name: str) -> str:
    for d in (root, os.path.join(root, "MNIST", "raw"), os.path.join(root, "raw")):
        for cand in (os.path.join(d, name), os.path.join(d, name + ".gz")):
            if os.path.exists(cand):
                return cand
    raise FileNotFoundError(f"{name}[.gz] not found under {root} (or its MNIST/raw)")


class MnistIDX:
    """The MNIST split at `root` (torchvision's layout or a flat directory of IDX files)."""

    def __init__(self, root: str, train: bool = True):
        img_name, lbl_name = _FILES[train]
        self.images = read_idx(_find(root, img_name))
        self.labels = read_idx(_find(root, lbl_name))
        if self.images.ndim != 3 or self.images.shape[1:] != (28, 28) or self.images.dtype != np.uint8:
            raise ValueError(f"images: expected u8 [N,28,28], got {self.images.dtype} {self.images.shape}")
        if self.labels.shape != (self.images.shape[0],):
            raise ValueError(f"labels: expected [{self.images.shape[0]}], got {self.labels.shape}")
        if self.labels.size and int(self.labels.max()) > 9:
            raise ValueError("labels must be in [0, 10)")

    def __len__(self):
        return int(self.images.shape[0])


class DeviceLoader:
    """DataLoader(dataset, batch_size, shuffle) with the dataset resident in HBM.

    Each epoch draws one permutation (torch.randperm with this loader's generator), copies it to the
    device once, and yields (x f32 [B,1,28,28], y i64 [B]) per batch; the last batch is ragged like
    the reference's (drop_last=False). Batches are written into two alternating device buffers, so
    a consumer must finish with a batch before asking for the one after next."""

    def __init__(self, dataset: MnistIDX, batch_size: int = 64, shuffle: bool = True,
                 seed: Optional[int] = None, device="cuda", drop_last: bool = False):
        self.device = torch.device(device)
        self.batch_size = int(batch_size)
        self.shuffle = shuffle
        self.drop_last = drop_last
        self.gen = torch.Generator()
        if seed is not None:
            self.gen.manual_seed(seed)
        self.images = torch.from_numpy(np.ascontiguousarray(dataset.images)).to(self.device)
        self.labels = torch.from_numpy(np.ascontiguousarray(dataset.labels)).to(self.device)
        self.err = torch.zeros(1, dtype=torch.int32, device=self.device)
        self.n = len(dataset)
        self._bufs = [None, None]

    def __len__(self):
        full, rem = divmod(self.n, self.batch_size)
        return full + (1 if rem and not self.drop_last else 0)

    def order(self) -> torch.Tensor:
        if self.shuffle:
            return torch.randperm(self.n, generator=self.gen)
        return torch.arange(self.n)

    def _buf(self, k: int, B: int):
        b = self._bufs[k]
        if b is None or b[0].shape[0] != B:
            b = (torch.empty((B, 1, 28, 28), dtype=torch.float32, device=self.device),
                 torch.empty((B,), dtype=torch.int64, device=self.device))
            self._bufs[k] = b
        return b

    def __iter__(self) -> Iterator[Tuple[torch.Tensor, torch.Tensor]]:
        perm = self.order().to(self.device, non_blocking=False)
        for k, start in enumerate(range(0, self.n, self.batch_size)):
            idx = perm[start:start + self.batch_size]
            if idx.numel() < self.batch_size and self.drop_last:
                break
            x, y = self._buf(k & 1, idx.numel())
            yield ops.mnist_batch(self.images, self.labels, idx, x=x, y=y, err_flag=self.err)
