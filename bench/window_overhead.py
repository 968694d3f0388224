#!/usr/bin/env python3
"""Where the fixed cost of a short timed window goes (bench.py's driver command
times 20 steps between two device syncs).

Host wall time of K steps (K = 1 .. 80) bracketed exactly like bench.py, the
linear fit's intercept = fixed cost per window; plus device-side event times
of each of the first steps after an idle sync (first-step slowdown vs steady
state).

    python bench/window_overhead.py [--model conv28]
"""
import argparse
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--graph-steps", type=int, default=10)
    ap.add_argument("--spin", action="store_true", help="hipSetDeviceFlags(hipDeviceScheduleSpin) first")
    a = ap.parse_args()
    if a.spin:
        import ctypes

        rc = ctypes.CDLL("libamdhip64.so").hipSetDeviceFlags(1)  # hipDeviceScheduleSpin
        print("hipSetDeviceFlags(spin) ->", rc, flush=True)
    from multidisttorch_amd.data.datasets import mnist_like
    from multidisttorch_amd.models.conv_vae import ConvVaeTrainer

    dev = torch.device("cuda", 0)
    train = mnist_like(True, synthetic=True, device=dev, size=28)
    tr = ConvVaeTrainer(batch_size=128, image=28, z=32, device=dev, backend="hip", seed=1,
                        use_graphs=True, graph_steps=a.graph_steps)
    idx = torch.arange(len(train), device=dev, dtype=torch.int32)
    tr.bind_train_data(train.data, idx)
    tr.set_cursor(0, idx.numel() // 128)
    tr.prepare([128])
    tr.strict_graphs = True
    tr.train_steps(20)
    torch.cuda.synchronize()
    # 1. the bracket alone
    t0 = time.perf_counter()
    for _ in range(20):
        torch.cuda.synchronize()
    print(f"idle synchronize: {(time.perf_counter() - t0) / 20 * 1e6:.1f} us", flush=True)
    # 2. wall time of K steps between syncs (bench.py's bracket), 5 reps each
    pts = []
    for K in (1, 2, 5, 10, 20, 40, 80):
        best = []
        for _ in range(5):
            torch.cuda.synchronize()
            time.sleep(0.002)  # the bench's barrier / sync gap before t0
            t0 = time.perf_counter()
            tr.train_steps(K)
            torch.cuda.synchronize()
            best.append(time.perf_counter() - t0)
        best.sort()
        pts.append((K, best[len(best) // 2] * 1e6))
        print(f"K={K:3d}: median {best[len(best) // 2] * 1e6:8.1f} us  ({best[len(best) // 2] * 1e3 / K:.4f} ms/step)",
              flush=True)
    n = len(pts)
    sx = sum(k for k, _ in pts)
    sy = sum(t for _, t in pts)
    sxx = sum(k * k for k, _ in pts)
    sxy = sum(k * t for k, t in pts)
    slope = (n * sxy - sx * sy) / (n * sxx - sx * sx)
    icpt = (sy - slope * sx) / n
    print(f"fit: {slope:.2f} us/step + {icpt:.1f} us fixed per window", flush=True)
    # 3. device time of each of the first 10 steps after an idle gap (eager step launches with events)
    tr.use_graphs = False
    torch.cuda.synchronize()
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(11)]
    time.sleep(0.002)
    ev[0].record()
    for i in range(10):
        tr._step_hip(128)
        ev[i + 1].record()
    torch.cuda.synchronize()
    print("first steps after idle (device, us):", [round(ev[i].elapsed_time(ev[i + 1]) * 1e3, 1) for i in range(10)])


if __name__ == "__main__" and not os.getenv("FIRST_STEP"):
    main()


def first_step_launches(gaps=(0.0, 0.0002, 0.002, 0.02)):
    """Device time of each launch of the first step after an idle gap of each length."""
    from multidisttorch_amd.data.datasets import mnist_like
    from multidisttorch_amd.models.conv_vae import ConvVaeTrainer

    dev = torch.device("cuda", 0)
    train = mnist_like(True, synthetic=True, device=dev, size=28)
    tr = ConvVaeTrainer(batch_size=128, image=28, z=32, device=dev, backend="hip", seed=1, use_graphs=False)
    idx = torch.arange(len(train), device=dev, dtype=torch.int32)
    tr.bind_train_data(train.data, idx)
    tr.set_cursor(0, idx.numel() // 128)
    tr.train_steps(20)
    C = tr.C
    real = C

    class Rec:
        def __getattr__(self, n):
            f = getattr(real, n)
            if n not in ("f28_step", "launch_jobs_multi", "grad_finalize"):
                return f

            def w(*a, **k):
                r = f(*a, **k)
                evs.append((n, torch.cuda.Event(enable_timing=True)))
                evs[-1][1].record()
                return r
            return w

    for gap in gaps:
        torch.cuda.synchronize()
        time.sleep(gap)
        evs = []
        e0 = torch.cuda.Event(enable_timing=True)
        e0.record()
        tr.C = Rec()
        for _ in range(2):
            tr._step_hip(128)
        tr.C = real
        torch.cuda.synchronize()
        prev, out = e0, []
        for n, e in evs:
            out.append(f"{n[:10]} {prev.elapsed_time(e) * 1e3:.1f}")
            prev = e
        print(f"gap {gap * 1e3:5.1f} ms:", ", ".join(out), flush=True)


if __name__ == "__main__" and os.getenv("FIRST_STEP"):
    first_step_launches()
