"""CPU checks of the index math behind the parity-class GEMM (conv_igemm.hip).

A pure-torch re-implementation of kModeTconv (class offsets oa/ea, tap
selection ky = a + s*ty, parity-ordered transposed weights) must equal
F.conv_transpose2d — this pins the kernel's address arithmetic without a GPU.
"""
import pytest
import torch
import torch.nn.functional as F

from multidisttorch_amd.ops.conv_layout import conv_desc, nchw, nhwc, parity_transpose, torch_weight


def test_parity_transpose_matches_definition():
    co, k, c, s = 5, 4, 3, 2
    w = torch.randn(co, k, k, c)
    t = parity_transpose(w, s).view(s, s, c, k // s, k // s, co)
    for a in range(s):
        for b in range(s):
            for ty in range(k // s):
                for tx in range(k // s):
                    torch.testing.assert_close(t[a, b, :, ty, tx, :], w[:, a + s * ty, b + s * tx, :].T)


def _parity_gemm(g_nhwc, w, d):
    """kModeTconv on the host: Y[n, iy, ix, ci] for every parity class."""
    N, H, W, C, OH, OW, CO, KH, KW, S, P = d
    T = KH // S
    wt = parity_transpose(w, S).view(S, S, C, T, T, CO)
    y = torch.zeros(N, H, W, C, dtype=torch.float64)
    for a in range(S):
        for b in range(S):
            oa, ob = (a - P) % S, (b - P) % S
            ea, eb = (oa + P - a) // S, (ob + P - b) // S
            assert (oa + P - a) % S == 0
            for j in range(H // S):
                for i in range(W // S):
                    iy, ix = S * j + oa, S * i + ob
                    acc = torch.zeros(N, C, dtype=torch.float64)
                    for ty in range(T):
                        for tx in range(T):
                            oy, ox = j + ea - ty, i + eb - tx
                            if 0 <= oy < OH and 0 <= ox < OW:
                                acc += g_nhwc[:, oy, ox, :].double() @ wt[a, b, :, ty, tx, :].double().T
                    y[:, iy, ix, :] = acc
    return y


@pytest.mark.parametrize("shape", [(2, 8, 3, 4, 4, 2, 1), (1, 6, 2, 5, 4, 2, 1), (2, 3, 4, 6, 1, 1, 0),
                                   (1, 9, 2, 3, 3, 3, 0)])
def test_parity_class_gemm_equals_conv_transpose(shape):
    N, H, C, CO, k, s, p = shape
    d = conv_desc(N, H, H, C, CO, k, s, p)
    OH = d[4]
    g = torch.randn(N, OH, OH, CO)
    w = torch.randn(CO, k, k, C)
    got = _parity_gemm(g, w, d)
    ref = F.conv_transpose2d(nchw(g).double(), torch_weight(w).double(), None, s, p,
                             output_padding=H - ((OH - 1) * s - 2 * p + k))
    torch.testing.assert_close(got, nhwc(ref))


def test_fastdiv_magic_numbers():
    """make_fastdiv (conv_igemm.h) replicated: q = (mulhi(n, mul) + n) >> shr."""
    def make(d):
        shr = 0
        while (1 << shr) < d:
            shr += 1
        mul = ((1 << 32) * ((1 << shr) - d)) // d + 1
        return mul & 0xFFFFFFFF, shr

    import random

    rng = random.Random(0)
    for d in [1, 2, 3, 7, 14, 49, 64, 196, 1000, 4096, 16384, 65535, 262144, 1 << 20]:
        mul, shr = make(d)
        for n in [0, 1, d - 1, d, d + 1, 2 * d - 1, (1 << 31) - 1] + [rng.randrange(1 << 31) for _ in range(200)]:
            q = (((n * mul) >> 32) + n) >> shr
            assert q == n // d, (d, n)
