"""Host-side layout helpers of the conv implicit-GEMM kernels (csrc/kernels/conv_igemm.hip).

* weights are stored ``[CO][KH][KW][C]`` ("conv view": a transposed conv is the
  conv whose backward-data is its forward);
* the parity-class GEMM (conv backward-data / convT forward) reads a
  parity-ordered transpose ``[s][s][C][k/s][k/s][CO]``: class ``(a, b)`` holds
  the taps ``ky = a + s*ty``, ``kx = b + s*tx`` that reach the input pixels
  with ``(iy + P) % s == a`` — exactly the taps a stride-s transposed conv
  applies there, so no zero-insertion work is done;
* ``conv_desc`` is the 11-int geometry ``(N, H, W, C, OH, OW, CO, KH, KW, S, P)``.
"""

from __future__ import annotations

import torch

__all__ = ["parity_transpose", "conv_desc", "nhwc", "nchw", "torch_weight"]


def parity_transpose(w: torch.Tensor, s: int) -> torch.Tensor:
    """[CO, k, k, C] -> flat parity-ordered transpose [s, s, C, k/s, k/s, CO]."""
    co, k, k2, c = w.shape
    assert k == k2 and k % s == 0
    t = k // s
    # ky = a + s*ty  ->  view ky as (ty, a)
    v = w.reshape(co, t, s, t, s, c)            # [co, ty, a, tx, b, c]
    v = v.permute(2, 4, 5, 1, 3, 0)             # [a, b, c, ty, tx, co]
    return v.contiguous().reshape(-1)


def conv_desc(N, H, W, C, CO, k, s, p):
    OH = (H + 2 * p - k) // s + 1
    OW = (W + 2 * p - k) // s + 1
    return [N, H, W, C, OH, OW, CO, k, k, s, p]


def nhwc(x: torch.Tensor) -> torch.Tensor:
    return x.permute(0, 2, 3, 1).contiguous()


def nchw(x: torch.Tensor) -> torch.Tensor:
    return x.permute(0, 3, 1, 2).contiguous()


def torch_weight(w: torch.Tensor) -> torch.Tensor:
    """[CO, k, k, C] -> torch Conv2d weight [CO, C, k, k]."""
    return w.permute(0, 3, 1, 2).contiguous()
