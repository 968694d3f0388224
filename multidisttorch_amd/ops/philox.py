"""Host (numpy) Philox4x32-10 + Box-Muller, bit-identical in its integer part to
``csrc/kernels/common.h`` so the CPU reference path draws the same
reparameterisation noise as the HIP kernels for the same (seed, stream, step).
"""

from __future__ import annotations

import numpy as np

M0 = np.uint64(0xD2511F53)
M1 = np.uint64(0xCD9E8D57)
W0 = np.uint32(0x9E3779B9)
W1 = np.uint32(0xBB67AE85)
MASK = np.uint64(0xFFFFFFFF)


def philox4x32_10(c0, c1, c2, c3, k0, k1):
    c0 = np.asarray(c0, dtype=np.uint32)
    c1 = np.broadcast_to(np.asarray(c1, dtype=np.uint32), c0.shape).copy()
    c2 = np.broadcast_to(np.asarray(c2, dtype=np.uint32), c0.shape).copy()
    c3 = np.broadcast_to(np.asarray(c3, dtype=np.uint32), c0.shape).copy()
    k0 = np.uint32(k0)
    k1 = np.uint32(k1)
    with np.errstate(over="ignore"):
        for _ in range(10):
            p0 = c0.astype(np.uint64) * M0
            p1 = c2.astype(np.uint64) * M1
            lo0 = (p0 & MASK).astype(np.uint32)
            hi0 = (p0 >> np.uint64(32)).astype(np.uint32)
            lo1 = (p1 & MASK).astype(np.uint32)
            hi1 = (p1 >> np.uint64(32)).astype(np.uint32)
            c0, c1, c2, c3 = hi1 ^ c1 ^ k0, lo1, hi0 ^ c3 ^ k1, lo0
            k0 = np.uint32(k0 + W0)
            k1 = np.uint32(k1 + W1)
    return c0, c1, c2, c3


def normal_from_bits(a, b):
    a = a.astype(np.float32)
    b = b.astype(np.float32)
    u1 = (a + np.float32(1.0)) * np.float32(2.3283064365386963e-10)
    u2 = b * np.float32(2.3283064365386963e-10)
    return (np.sqrt(np.float32(-2.0) * np.log(u1)) * np.cos(np.float32(6.283185307179586) * u2)).astype(np.float32)


def reparam_eps(M: int, Z: int, seed: int, stream: int, step: int) -> np.ndarray:
    """eps[M, Z] exactly as kernel vae_f2 draws it (counter = row*Z + c)."""
    e = np.arange(M * Z, dtype=np.uint64).astype(np.uint32)
    s_lo = np.uint32(step & 0xFFFFFFFF)
    s_hi = np.uint32((step >> 32) & 0xFFFFFFFF)
    x, y, _, _ = philox4x32_10(e, np.uint32(stream), s_lo, s_hi, seed & 0xFFFFFFFF, (seed >> 32) & 0xFFFFFFFF)
    return normal_from_bits(x, y).reshape(M, Z)
