"""Image-grid PNG writer (torchvision ``save_image`` equivalent; torchvision is
not installed on the build/GPU boxes).

Parity: the reference writes ``results-{rank}/reconstruction_{epoch}.png``
(8 originals + 8 reconstructions, ``nrow=8``) and ``sample_{epoch}.png`` (64
decoded latents) via ``torchvision.utils.save_image``
(/root/reference/vae-hpo.py:110-116, :166-170). ``make_grid`` below follows
torchvision's layout (padding 2, pad value 0, ``nrow`` images per row) and
its uint8 conversion (``x*255 + 0.5`` clamped); PNG encoding uses PIL when
importable, else a small zlib PNG encoder.
"""

from __future__ import annotations

import math
import struct
import zlib

import numpy as np
import torch

__all__ = ["make_grid", "save_image", "write_png", "save_image_async", "flush_images"]


def make_grid(t: torch.Tensor, nrow: int = 8, padding: int = 2, pad_value: float = 0.0) -> torch.Tensor:
    if t.dim() == 3:
        t = t.unsqueeze(0)
    if t.dim() != 4:
        raise ValueError("expected [N, C, H, W]")
    if t.shape[1] == 1:
        t = t.repeat(1, 3, 1, 1)
    n = t.shape[0]
    xmaps = min(nrow, n)
    ymaps = int(math.ceil(float(n) / xmaps))
    h, w = t.shape[2] + padding, t.shape[3] + padding
    grid = t.new_full((3, h * ymaps + padding, w * xmaps + padding), pad_value)
    k = 0
    for y in range(ymaps):
        for x in range(xmaps):
            if k >= n:
                break
            grid[:, y * h + padding: y * h + padding + t.shape[2],
                 x * w + padding: x * w + padding + t.shape[3]] = t[k]
            k += 1
    return grid


def write_png(path: str, rgb: np.ndarray):
    """Minimal RGB8 PNG encoder (no external deps)."""
    h, w, _ = rgb.shape
    raw = b"".join(b"\x00" + rgb[y].tobytes() for y in range(h))

    def chunk(tag, data):
        return struct.pack(">I", len(data)) + tag + data + struct.pack(">I", zlib.crc32(tag + data) & 0xFFFFFFFF)

    png = b"\x89PNG\r\n\x1a\n" + chunk(b"IHDR", struct.pack(">IIBBBBB", w, h, 8, 2, 0, 0, 0))
    png += chunk(b"IDAT", zlib.compress(raw, 6)) + chunk(b"IEND", b"")
    with open(path, "wb") as f:
        f.write(png)


def save_image(t: torch.Tensor, path: str, nrow: int = 8, padding: int = 2):
    grid = make_grid(t.detach().float().cpu(), nrow=nrow, padding=padding)
    arr = grid.mul(255).add_(0.5).clamp_(0, 255).permute(1, 2, 0).to(torch.uint8).numpy()
    try:
        from PIL import Image

        Image.fromarray(arr).save(path)
    except Exception:
        write_png(path, np.ascontiguousarray(arr))


# --------------------------------------------------------------------------
# Asynchronous writer: the grid is assembled and PNG-encoded on a background
# thread, so image output overlaps the next epoch's (asynchronous) graph
# replays instead of stalling the host between epochs. Order of writes to the
# same path is preserved (one worker).
_POOL = None


def save_image_async(t: torch.Tensor, path: str, nrow: int = 8, padding: int = 2):
    global _POOL
    if _POOL is None:
        from concurrent.futures import ThreadPoolExecutor

        _POOL = ThreadPoolExecutor(max_workers=1, thread_name_prefix="mdt-png")
    host = t.detach().float().cpu()  # snapshot now; the device buffer may be reused
    return _POOL.submit(save_image, host, path, nrow, padding)


def flush_images():
    """Block until every queued image is on disk (called before a run ends)."""
    global _POOL
    if _POOL is not None:
        _POOL.shutdown(wait=True)
        _POOL = None
