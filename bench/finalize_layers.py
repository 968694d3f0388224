"""Finalize + Adam of each layer of a conv-VAE step timed alone (the optimizer
tail's pieces): per layer its parameter count, partial slabs, units and the
kernel time, plus the implied fabric rate of the compulsory bytes (slabs +
Adam's P/m/v read and written + the bf16 copy).

    python bench/finalize_layers.py [--image 128 --batch 64]
"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--image", type=int, default=128)
    ap.add_argument("--batch", type=int, default=64)
    ap.add_argument("--reps", type=int, default=20)
    a = ap.parse_args()
    from multidisttorch_amd.data.datasets import mnist_like
    from multidisttorch_amd.models.conv_vae import ConvVaeTrainer

    dev = torch.device("cuda", 0)
    os.environ.setdefault("MDT_CONV_F28", "0")
    train = mnist_like(True, synthetic=True, device=dev, size=a.image)
    tr = ConvVaeTrainer(batch_size=a.batch, image=a.image, device=dev, backend="hip", seed=1, use_graphs=False)
    idx = torch.arange(len(train), device=dev, dtype=torch.int32)
    tr.bind_train_data(train.data, idx)
    tr.set_cursor(0, idx.numel() // a.batch)
    tr.train_steps(3)
    torch.cuda.synchronize()
    M = a.batch
    p = tr._plan(M)
    lu = p["layer_units"]
    segs = tr._seg_rows(p["slabs"])
    tot_us = 0.0
    for i, l in enumerate(tr.spec):
        s0, s1 = segs[2 * i], segs[2 * i + 1]
        numel = s0[1] + s1[1]
        slab = s0[1] * s0[3] * (1 if s0[2] else 0) + s1[1] * s1[3] * (1 if s1[2] else 0)
        mb = (4 * slab + numel * (4 * 6 + 2)) / 1e6
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        tr._finalize_layers(M, i, i + 1)
        torch.cuda.synchronize()
        e0.record()
        for _ in range(a.reps):
            tr._finalize_layers(M, i, i + 1)
        e1.record()
        torch.cuda.synchronize()
        us = e0.elapsed_time(e1) * 1e3 / a.reps
        tot_us += us
        print(f"{l.name:10s} params {numel:9d}  slabs w {s0[3]:5d} b {s1[3]:5d}  units {lu[i + 1] - lu[i]:6d}  "
              f"{us:7.2f} us  {mb:7.1f} MB  {mb / us:5.2f} TB/s", flush=True)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(a.reps):
        tr._finalize_layers(M, 0, len(tr.spec))
    e1.record()
    torch.cuda.synchronize()
    print(f"sum of per-layer launches {tot_us:.1f} us; all layers in one launch "
          f"{e0.elapsed_time(e1) * 1e3 / a.reps:.1f} us", flush=True)


if __name__ == "__main__":
    main()
