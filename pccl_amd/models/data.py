"""Datasets for the examples and end-to-end tests — no network access is assumed.

* MNIST from local IDX files (``*-idx3-ubyte[.gz]``), e.g. the fixtures the reference ships under
  python/tests/end_to_end/data/MNIST/raw; falls back to a deterministic synthetic digit-like set of the same shape.
* Token streams: a ``uint16`` memmap (nanoGPT's ``train.bin`` format, reference prepare_owt_dataset.py) or synthetic
  uniformly random tokens of GPT-2 vocabulary size.
"""
from __future__ import annotations

import gzip
import os
from typing import Iterator, Optional, Tuple

import numpy as np
import torch


def _read_idx(path: str) -> np.ndarray:
    opener = gzip.open if path.endswith(".gz") else open
    with opener(path, "rb") as f:
        data = f.read()
    magic = int.from_bytes(data[0:4], "big")
    ndim = magic & 0xFF
    dims = [int.from_bytes(data[4 + 4 * i:8 + 4 * i], "big") for i in range(ndim)]
    return np.frombuffer(data, dtype=np.uint8, offset=4 + 4 * ndim).reshape(dims)


def _find(root: str, stem: str) -> Optional[str]:
    for name in (stem, stem + ".gz"):
        p = os.path.join(root, name)
        if os.path.exists(p):
            return p
    return None


def load_mnist(root: Optional[str] = None, split: str = "train", synthetic_size: int = 10000,
               seed: int = 0) -> Tuple[torch.Tensor, torch.Tensor]:
    """Returns (images float32 [N,1,28,28] in [0,1], labels int64 [N]).

    ``split='train'`` uses the train files if present, else the t10k files (the reference's fixture directory only
    ships the t10k images). Without files, a synthetic class-conditional dataset is generated.
    """
    candidates = [root] if root else []
    candidates += [os.environ.get("PCCL_MNIST_DIR", ""), "/root/reference/python/tests/end_to_end/data/MNIST/raw"]
    for r in candidates:
        if not r or not os.path.isdir(r):
            continue
        for prefix in (("train", "t10k") if split == "train" else ("t10k",)):
            ip, lp = _find(r, f"{prefix}-images-idx3-ubyte"), _find(r, f"{prefix}-labels-idx1-ubyte")
            if ip and lp:
                x = torch.from_numpy(_read_idx(ip).astype(np.float32) / 255.0).unsqueeze(1)
                y = torch.from_numpy(_read_idx(lp).astype(np.int64))
                return x, y
    return synthetic_mnist(synthetic_size, seed)


def synthetic_mnist(n: int, seed: int = 0) -> Tuple[torch.Tensor, torch.Tensor]:
    """Class-conditional blobs: each class has a fixed random 28x28 prototype plus noise (learnable, deterministic)."""
    g = torch.Generator().manual_seed(1234)
    protos = (torch.rand(10, 1, 28, 28, generator=g) > 0.7).float()
    g = torch.Generator().manual_seed(seed)
    y = torch.randint(0, 10, (n,), generator=g)
    x = (protos[y] * 0.8 + torch.rand(n, 1, 28, 28, generator=g) * 0.4).clamp(0, 1)
    return x, y


def batches(x: torch.Tensor, y: torch.Tensor, batch_size: int, seed: int = 0,
            device: Optional[torch.device] = None) -> Iterator[Tuple[torch.Tensor, torch.Tensor]]:
    """Endless shuffled mini-batches (epochs reshuffle with seed + epoch)."""
    epoch = 0
    if device is not None:
        x, y = x.to(device), y.to(device)
    while True:
        g = torch.Generator().manual_seed(seed + epoch)
        perm = torch.randperm(x.shape[0], generator=g)
        if device is not None:
            perm = perm.to(device)
        for i in range(0, x.shape[0] - batch_size + 1, batch_size):
            idx = perm[i:i + batch_size]
            yield x[idx], y[idx]
        epoch += 1


class TokenStream:
    """Random contiguous (x, y) windows from a uint16 token memmap, or synthetic tokens when no file is given."""

    def __init__(self, path: Optional[str] = None, vocab_size: int = 50304, synthetic_tokens: int = 1 << 22,
                 seed: int = 0):
        if path and os.path.exists(path):
            self.data = np.memmap(path, dtype=np.uint16, mode="r")
        else:
            rng = np.random.default_rng(seed)
            self.data = rng.integers(0, min(vocab_size, 50257), size=synthetic_tokens, dtype=np.uint16)
        self.rng = np.random.default_rng(seed + 1)

    def batch(self, batch_size: int, block_size: int, device: torch.device) -> Tuple[torch.Tensor, torch.Tensor]:
        ix = self.rng.integers(0, len(self.data) - block_size - 1, size=batch_size)
        x = torch.from_numpy(np.stack([self.data[i:i + block_size].astype(np.int64) for i in ix]))
        y = torch.from_numpy(np.stack([self.data[i + 1:i + 1 + block_size].astype(np.int64) for i in ix]))
        if device.type == "cuda":
            return x.pin_memory().to(device, non_blocking=True), y.pin_memory().to(device, non_blocking=True)
        return x.to(device), y.to(device)
