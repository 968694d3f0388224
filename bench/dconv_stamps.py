"""Per-phase timing of the direct conv kernels (csrc/kernels/conv_direct.h).

Each workgroup stamps s_memrealtime (100 MHz) at start, after its patch and
first weight stage landed, after the k loop and at the end. Prints, per
geometry, the kernel time (HIP events, mean of reps) and the median / max
phase durations over workgroups plus the dispatch skew.

    python bench/dconv_stamps.py [--batch 64]
"""
import argparse
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

CASES = [(0, 64, 32, 32, 64), (0, 32, 64, 16, 128), (1, 32, 64, 16, 128), (1, 64, 32, 32, 64),
         (0, 16, 128, 8, 256), (1, 16, 128, 8, 256)]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=64)
    ap.add_argument("--reps", type=int, default=50)
    ap.add_argument("--json", default=None)
    a = ap.parse_args()
    from multidisttorch_amd.ops import native

    C = native.require()
    dev = torch.device("cuda")
    N = a.batch
    out = {}
    for mode, H, Cc, OH, CO in CASES:
        d = [N, H, H, Cc, OH, OH, CO, 4, 4, 2, 1]
        info = C.igemm_plan(mode, d, False, fwd=True)
        if mode == 0:
            A = torch.randn(N * H * H * Cc, device=dev).bfloat16()
            B = torch.randn(CO * 16 * Cc, device=dev).bfloat16()
            ny = N * OH * OH * CO
            ncols = CO
        else:
            A = torch.randn(N * OH * OH * CO, device=dev).bfloat16()
            B = torch.randn(4 * Cc * 4 * CO, device=dev).bfloat16()
            ny = N * H * H * Cc
            ncols = Cc
        y16 = torch.empty(ny, device=dev, dtype=torch.bfloat16)
        bias = torch.zeros(ncols, device=dev)
        run = lambda: C.igemm(mode, A, B, d, bias, True, y16, None, fwd=True)
        for _ in range(5):
            run()
        torch.cuda.synchronize()
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        for _ in range(a.reps):
            run()
        e.record()
        torch.cuda.synchronize()
        us = s.elapsed_time(e) * 1e3 / a.reps
        grid = info[7] * info[8]
        st = torch.zeros(grid * 8, dtype=torch.int64, device=dev)
        C.dconv_stamps(st)
        run()
        torch.cuda.synchronize()
        C.dconv_stamps(None)
        t = st.view(grid, 8)[:, :4].cpu().numpy().astype(np.float64) * 0.01
        ph = {"load": t[:, 1] - t[:, 0], "kloop": t[:, 2] - t[:, 1], "epi": t[:, 3] - t[:, 2]}
        flops = 2.0 * info[3] * info[4] * info[5] * info[6]
        r = {"cfg": info[0], "grid": grid, "us": round(us, 2), "TF/s": round(flops / us * 1e-6, 1),
             "span_us": round(float(t[:, 3].max() - t[:, 0].min()), 2),
             "start_skew_us": round(float(t[:, 0].max() - t[:, 0].min()), 2)}
        for k, v in ph.items():
            r[k] = (round(float(np.median(v)), 2), round(float(v.max()), 2))
        out[f"mode{mode}_{H}x{Cc}_{OH}x{CO}"] = r
        print(f"mode{mode} {H}x{Cc} <-> {OH}x{CO}: {r}", flush=True)
    # direct weight gradient (conv_dwgrad.h): stamps 0 start, 1 stage 0 landed,
    # 2 half the stages done, 3 k loop done, 4 partial row stored
    for H, Cc, CO in ((64, 32, 64),):
        OH = H // 2
        d = [N, H, H, Cc, OH, OH, CO, 4, 4, 2, 1]
        info = C.wgrad_plan(d)
        if info[0] < 100:
            continue
        X = torch.randn(N * H * H * Cc, device=dev).bfloat16()
        G = torch.randn(N * OH * OH * CO, device=dev).bfloat16()
        o = torch.empty(N * CO * 16 * Cc, device=dev)
        run = lambda: C.wgrad(G, X, d, o)
        for _ in range(5):
            run()
        torch.cuda.synchronize()
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        for _ in range(a.reps):
            run()
        e.record()
        torch.cuda.synchronize()
        us = s.elapsed_time(e) * 1e3 / a.reps
        grid = N * 4
        st = torch.zeros(grid * 8, dtype=torch.int64, device=dev)
        C.dconv_stamps(st)
        run()
        torch.cuda.synchronize()
        C.dconv_stamps(None)
        t = st.view(grid, 8)[:, :5].cpu().numpy().astype(np.float64) * 0.01
        ph = {"first_stage": t[:, 1] - t[:, 0], "first_half": t[:, 2] - t[:, 1], "second_half": t[:, 3] - t[:, 2],
              "epi": t[:, 4] - t[:, 3]}
        r = {"cfg": info[0], "grid": grid, "us": round(us, 2), "span_us": round(float(t[:, 4].max() - t[:, 0].min()), 2),
             "start_skew_us": round(float(t[:, 0].max() - t[:, 0].min()), 2)}
        for k, v in ph.items():
            r[k] = (round(float(np.median(v)), 2), round(float(v.max()), 2))
        out[f"dwgrad_{H}x{Cc}_{OH}x{CO}"] = r
        print(f"dwgrad {H}x{Cc} -> {OH}x{CO}: {r}", flush=True)
    if a.json:
        with open(a.json, "w") as f:
            json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
