#!/usr/bin/env python3
"""Calibrate the conv GEMM kernels on plain GEMMs (1x1 images: no im2col).

Times igemm (conv mode, forward-type) and wgrad on square/rectangular bf16
problems and prints TFLOP/s, to separate kernel-structure limits from
gather/locality effects. usage: python bench/gemm_calib.py [--reps 20]
"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def timeit(f, reps):
    for _ in range(3):
        f()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    e0.record()
    for _ in range(reps):
        f()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1e3 / reps


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=20)
    a = ap.parse_args()
    from multidisttorch_amd.ops import native

    C = native.require()
    dev = "cuda"
    for (M, N, K) in [(4096, 4096, 4096), (16384, 1024, 1024), (16384, 128, 1024), (65536, 64, 512), (8192, 8192, 8192)]:
        A = torch.randn(M, K, device=dev).to(torch.bfloat16)
        W = torch.randn(N, K, device=dev).to(torch.bfloat16)
        y = torch.empty(M * N, device=dev, dtype=torch.bfloat16)
        d = [M, 1, 1, K, 1, 1, N, 1, 1, 1, 0]
        us = timeit(lambda: C.igemm(0, A, W.flatten(), d, None, False, y, None), a.reps)
        ref_us = timeit(lambda: torch.mm(A, W.t()), a.reps)
        plan = C.igemm_plan(0, d, False)
        fl = 2.0 * M * N * K
        print(f"igemm M={M} N={N} K={K}: {us:8.1f} us {fl / us / 1e6:7.1f} TF/s   torch.mm {ref_us:8.1f} us "
              f"{fl / ref_us / 1e6:7.1f} TF/s  plan={plan}", flush=True)
        # weight gradient: dW[N][K] = G^T X with the reduction over M
        G = torch.randn(M, N, device=dev).to(torch.bfloat16)
        info = C.wgrad_plan(d)
        out = torch.empty(info[6] * N * K, device=dev)
        us = timeit(lambda: C.wgrad(G, A, d, out), a.reps)
        ref_us = timeit(lambda: torch.mm(G.t(), A), a.reps)
        print(f"wgrad M={M} N={N} K={K}: {us:8.1f} us {fl / us / 1e6:7.1f} TF/s   torch.mm {ref_us:8.1f} us "
              f"{fl / ref_us / 1e6:7.1f} TF/s  plan={info}", flush=True)


if __name__ == "__main__":
    main()
