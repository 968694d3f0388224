"""Per-stage timeline of the direct conv k loop (csrc/kernels/conv_direct.h,
4-wave form), from a side build with -DMDT_DC_STAGE_STAMPS:

    MDT_BUILD_TAG=ss MDT_HIP_EXTRA_FLAGS=-DMDT_DC_STAGE_STAMPS python -c "from multidisttorch_amd import _build; _build.build()"
    MDT_NATIVE_SO=variants/ss/_C.so python bench/dconv_stage_stamps.py

Per stage the leader wave stamps (s_memrealtime, 10 ns): loop top, after
three k-steps' MFMAs were issued, after the wait for the next weight stage,
after the workgroup barrier. Prints median over workgroups / stages of:
top -> pre-wait (fragment loads + MFMA issue), wait, barrier, rest (refill
issue + next fragments + last MFMA) for the 16x16 <-> 8x8 geometries.
"""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    from multidisttorch_amd.ops import native

    C = native.require()
    dev = torch.device("cuda")
    N = 64
    for mode, H, Cc, OH, CO in ((0, 16, 128, 8, 256), (1, 16, 128, 8, 256), (0, 32, 64, 16, 128)):
        d = [N, H, H, Cc, OH, OH, CO, 4, 4, 2, 1]
        info = C.igemm_plan(mode, d, False, fwd=True)
        if mode == 0:
            A = torch.randn(N * H * H * Cc, device=dev).bfloat16()
            B = torch.randn(CO * 16 * Cc, device=dev).bfloat16()
            ny, K = N * OH * OH * CO, 16 * Cc
        else:
            A = torch.randn(N * OH * OH * CO, device=dev).bfloat16()
            B = torch.randn(4 * Cc * 4 * CO, device=dev).bfloat16()
            ny, K = N * H * H * Cc, 4 * CO
        nst = K // 64
        y16 = torch.empty(ny, device=dev, dtype=torch.bfloat16)
        bias = torch.zeros(Cc if mode else CO, device=dev)
        grid = info[7] * info[8]
        st = torch.zeros(grid * 8 + grid * nst * 4, dtype=torch.int64, device=dev)
        for _ in range(5):
            C.igemm(mode, A, B, d, bias, True, y16, None, fwd=True)
        torch.cuda.synchronize()
        C.dconv_stamps(st)
        C.igemm(mode, A, B, d, bias, True, y16, None, fwd=True)
        torch.cuda.synchronize()
        C.dconv_stamps(None)
        s = st[grid * 8:].view(grid, nst, 4).cpu().numpy().astype(np.float64) * 10.0  # ns
        ph = st[:grid * 8].view(grid, 8).cpu().numpy().astype(np.float64) * 10.0
        body = s[:, :-1, :]  # the last stage has no wait / barrier
        nxt = s[:, 1:, 0]
        parts = {"frags+mma": body[:, :, 1] - body[:, :, 0], "wait": body[:, :, 2] - body[:, :, 1],
                 "barrier": body[:, :, 3] - body[:, :, 2], "rest": nxt - body[:, :, 3]}
        tot = nxt - body[:, :, 0]
        print(f"mode{mode} {H}x{Cc}<->{OH}x{CO} cfg {info[0]} grid {grid} stages {nst}: "
              f"kloop median {np.median(ph[:, 2] - ph[:, 1]) / 1e3:.2f} us, per stage {np.median(tot):.0f} ns = "
              + ", ".join(f"{k} {np.median(v):.0f}" for k, v in parts.items()), flush=True)
        # stage-resolved (median over workgroups) for the first 8 stages
        print("   per-stage (ns, median over wgs) wait:", [int(np.median(parts['wait'][:, i])) for i in range(min(8, nst - 1))],
              "barrier:", [int(np.median(parts['barrier'][:, i])) for i in range(min(8, nst - 1))], flush=True)


if __name__ == "__main__":
    main()
