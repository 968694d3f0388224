"""Device-resident datasets (synthetic MNIST-shaped, or IDX files when present).

The reference reads MNIST through torchvision (PIL decode per sample, CPU
collate, pageable H2D copy every step; /root/reference/vae-hpo.py:133-158).
Here the whole split lives in HBM as one [N, C*H*W] fp32 tensor (60 000 x 784
x 4 B = 188 MB, trivially resident in 288 GB) and kernels gather batch rows by
sampler index, so there is no per-sample host work at all.

No network and no torchvision on the GPU box: ``synthetic_mnist`` produces a
deterministic MNIST-shaped stand-in (values in [0, 1], smooth stroke-like
blobs, so the VAE has structure to learn). If real IDX files exist under
``data_dir`` (``train-images-idx3-ubyte`` etc., optionally .gz) they are used.
"""

from __future__ import annotations

import gzip
import os
from dataclasses import dataclass
from typing import Optional

import numpy as np
import torch

__all__ = ["ImageSet", "synthetic_images", "load_idx_images", "mnist_like"]


@dataclass
class ImageSet:
    data: torch.Tensor          # [N, C*H*W] float32 in [0, 1]
    shape: tuple                # (C, H, W)
    synthetic: bool
    name: str = "mnist"

    def __len__(self):
        return self.data.shape[0]

    def to(self, device):
        return ImageSet(self.data.to(device, non_blocking=True).contiguous(), self.shape, self.synthetic, self.name)

    def images(self, idx) -> torch.Tensor:
        return self.data[idx].view(-1, *self.shape)


def synthetic_images(n: int, size: int = 28, channels: int = 1, seed: int = 0,
                     device: Optional[torch.device] = None) -> torch.Tensor:
    """n images of `size`x`size`: a sum of 2-4 anisotropic Gaussian strokes.

    Generated in chunks on ``device`` (fast on GPU, bounded memory on CPU).
    """
    dev = device or torch.device("cpu")
    g = torch.Generator(device="cpu").manual_seed(seed)
    out = torch.empty(n, channels * size * size, dtype=torch.float32, device=dev)
    yy, xx = torch.meshgrid(torch.linspace(-1, 1, size, device=dev), torch.linspace(-1, 1, size, device=dev),
                            indexing="ij")
    chunk = 4096
    for s in range(0, n, chunk):
        m = min(chunk, n - s)
        k = 4
        cx = (torch.rand(m, k, generator=g) * 1.2 - 0.6).to(dev)
        cy = (torch.rand(m, k, generator=g) * 1.2 - 0.6).to(dev)
        sx = (torch.rand(m, k, generator=g) * 0.25 + 0.05).to(dev)
        sy = (torch.rand(m, k, generator=g) * 0.25 + 0.05).to(dev)
        on = (torch.rand(m, k, generator=g) < 0.75).float().to(dev)
        on[:, 0] = 1.0
        img = torch.zeros(m, size, size, device=dev)
        for j in range(k):
            img += on[:, j, None, None] * torch.exp(
                -((xx[None] - cx[:, j, None, None]) ** 2) / (2 * sx[:, j, None, None] ** 2)
                - ((yy[None] - cy[:, j, None, None]) ** 2) / (2 * sy[:, j, None, None] ** 2))
        img = img.clamp_(0, 1)
        if channels > 1:
            img = img[:, None].expand(m, channels, size, size)
        out[s:s + m] = img.reshape(m, -1)
    return out


def _open(path):
    if os.path.exists(path):
        return open(path, "rb")
    if os.path.exists(path + ".gz"):
        return gzip.open(path + ".gz", "rb")
    return None


def load_idx_images(path: str) -> Optional[np.ndarray]:
    """Parse an IDX3 uint8 image file -> float32 [N, H*W] in [0, 1] (no pickle)."""
    f = _open(path)
    if f is None:
        return None
    with f:
        buf = f.read()
    magic = int.from_bytes(buf[0:4], "big")
    if magic != 2051:
        raise ValueError(f"{path}: bad IDX3 magic {magic}")
    n, h, w = (int.from_bytes(buf[4 + 4 * i: 8 + 4 * i], "big") for i in range(3))
    arr = np.frombuffer(buf, dtype=np.uint8, offset=16, count=n * h * w).reshape(n, h * w)
    return arr.astype(np.float32) / 255.0


def mnist_like(train: bool, data_dir: str = "data", device=None, size: int = 28,
               synthetic: Optional[bool] = None, seed: int = 0, n: Optional[int] = None) -> ImageSet:
    """MNIST split: real IDX files if present (and not forced synthetic), else synthetic."""
    ntot = n if n is not None else (60000 if train else 10000)
    if synthetic is not True and size == 28:
        stem = "train-images-idx3-ubyte" if train else "t10k-images-idx3-ubyte"
        for d in (data_dir, os.path.join(data_dir, "MNIST", "raw")):
            arr = load_idx_images(os.path.join(d, stem))
            if arr is not None:
                t = torch.from_numpy(arr[:ntot].copy())
                return ImageSet(t.to(device) if device is not None else t, (1, 28, 28), False)
        if synthetic is False:
            raise FileNotFoundError(f"MNIST IDX files not found under {data_dir}")
    t = synthetic_images(ntot, size=size, seed=seed + (0 if train else 1), device=device)
    return ImageSet(t, (1, size, size), True, f"synthetic{size}")
