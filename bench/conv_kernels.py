#!/usr/bin/env python3
"""Per-launch timing of one conv-VAE training step (kernel microbenchmark).

Records every native launch of one `_step_hip` of a ConvVaeTrainer, then
replays each launch alone `--reps` times between HIP events and reports the
mean time and (for the GEMM launches) the achieved TFLOP/s, so a kernel change
can be judged layer by layer. Launches are replayed on the same buffers, which
is safe because every kernel here is a pure function of its inputs apart from
the state/optimizer tail (which is replayed too, harmlessly, on a scratch run).

usage: python bench/conv_kernels.py [--image 128] [--batch 64] [--reps 20] [--json out.json]
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


class Recorder:
    def __init__(self, C):
        self._C = C
        self.calls = []

    def __getattr__(self, name):
        f = getattr(self._C, name)
        if not callable(f) or name in ("igemm_plan", "wgrad_plan", "TrialState", "make_grad_segs",
                                       "make_grad_units", "make_tr_units"):
            return f

        def wrap(*a, **k):
            self.calls.append((name, a, k))
            return f(*a, **k)

        return wrap


def flops(name, a, k):
    if name == "igemm":
        mode, d = a[0], a[3]
        N, H, W, C, OH, OW, CO, KH, KW, S, P = d
        if mode == 0:
            return 2.0 * N * OH * OW * CO * KH * KW * C
        return 2.0 * N * H * W * C * (KH // S) * (KW // S) * CO
    if name == "wgrad":
        N, H, W, C, OH, OW, CO, KH, KW, S, P = a[2]
        return 2.0 * N * OH * OW * CO * KH * KW * C
    return 0.0


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--image", type=int, default=128)
    ap.add_argument("--batch", type=int, default=64)
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--json", default=None)
    a = ap.parse_args()
    from multidisttorch_amd.models.conv_vae import ConvVaeTrainer
    from multidisttorch_amd.data.datasets import synthetic_images

    dev = torch.device("cuda")
    tr = ConvVaeTrainer(batch_size=a.batch, image=a.image, z=32 if a.image == 28 else 64, device=dev,
                        backend="hip", use_graphs=False)
    X = synthetic_images(max(4 * a.batch, 512), size=a.image, device=dev)
    idx = torch.arange(X.shape[0], device=dev, dtype=torch.int32)
    tr.bind_train_data(X, idx)
    tr.set_cursor(0, X.shape[0] // a.batch)
    tr.train_steps(2)
    rec = Recorder(tr.C)
    tr.C = rec
    tr._step_hip(a.batch)
    tr.C = rec._C
    torch.cuda.synchronize()
    out, total = [], 0.0
    for i, (name, args, kw) in enumerate(rec.calls):
        f = getattr(tr.C, name)
        for _ in range(3):
            f(*args, **kw)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        torch.cuda.synchronize()
        e0.record()
        for _ in range(a.reps):
            f(*args, **kw)
        e1.record()
        torch.cuda.synchronize()
        us = e0.elapsed_time(e1) * 1e3 / a.reps
        fl = flops(name, args, kw)
        desc = args[3] if name == "igemm" else (args[2] if name == "wgrad" else None)
        tag = f"mode{args[0]}" if name == "igemm" else ""
        row = dict(i=i, op=name, tag=tag, us=round(us, 2), tflops=round(fl / us / 1e6, 1) if fl else None,
                   desc=desc)
        if name == "igemm":
            row["plan"] = tr.C.igemm_plan(args[0], desc, kw.get("ws") is not None)
        if name == "wgrad":
            row["plan"] = tr.C.wgrad_plan(desc)
        out.append(row)
        total += us
        print(f"{i:3d} {name:14s} {tag:6s} {us:8.2f} us  {row['tflops'] or '':>7}  {desc or ''}  {row.get('plan', '')}",
              flush=True)
    print(f"sum of isolated launches: {total:.1f} us")
    if a.json:
        with open(a.json, "w") as fh:
            json.dump(dict(image=a.image, batch=a.batch, calls=out, total_us=total), fh, indent=1)


if __name__ == "__main__":
    main()
