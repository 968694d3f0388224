#!/usr/bin/env python3
"""Error pattern of the 128x128 thin_conv kernel (enc1 geometry) against a
float64 conv: per output channel, row and column, the elements beyond one bf16
rounding. Diagnostic for tests/gpu/test_conv_igemm.py::test_thin_conv_matches_conv2d."""
import os
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from multidisttorch_amd.ops import native  # noqa: E402
from multidisttorch_amd.ops.conv_layout import conv_desc, nchw, nhwc, torch_weight  # noqa: E402


def main():
    C = native.require()
    dev = torch.device("cuda")
    N, H, CO = 3, 128, 32
    OH = H // 2
    torch.manual_seed(3)
    for f32_in in (True, False):
        x = torch.rand(N, H, H, 1, device=dev)
        if not f32_in:
            x = x.bfloat16().float()
        w = torch.randn(CO, 4, 4, 1, device=dev) / 4
        b = torch.randn(CO, device=dev)
        d = conv_desc(N, H, H, 1, CO, 4, 2, 1)
        M = N * OH * OH
        y16 = torch.zeros(M * CO, device=dev, dtype=torch.bfloat16)
        xin = x if f32_in else x.bfloat16()
        C.thin_conv(xin, w.flatten(), d, b, False, y16)
        torch.cuda.synchronize()
        ref = nhwc(F.conv2d(nchw(x.float()).double(), torch_weight(w).double(), b.double(), 2, 1)).reshape(M, CO)
        y = y16.double().view(M, CO)
        flips = int((y16.view(M, CO) != ref.float().bfloat16()).sum())
        print(f"f32_in={f32_in}: bf16 outputs != bf16(f64 result): {flips}/{y.numel()} "
              f"(MDT_THIN_MFMA={os.environ.get('MDT_THIN_MFMA', 'default')})")
        err = (y - ref).abs()
        bad = err > ref.abs() * 2.0 ** -8 + 1e-6
        print(f"f32_in={f32_in}: bad {int(bad.sum())}/{bad.numel()}, max err {float(err.max()):.3e}, "
              f"max rel {float((err / (ref.abs() + 1e-3)).max()):.3e}")
        if bad.any():
            bv = bad.view(N, OH, OH, CO)
            print("  per co:", bv.sum((0, 1, 2)).tolist())
            print("  per oy:", bv.sum((0, 2, 3)).tolist())
            print("  per ox:", bv.sum((0, 1, 3)).tolist())
            idx = bad.nonzero()[:8].tolist()
            for p, c in idx:
                print(f"   pix {p} co {c}: kernel {float(y[p, c]):.6f} ref {float(ref[p, c]):.6f}")


if __name__ == "__main__":
    main()
