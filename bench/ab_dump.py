#!/usr/bin/env python3
"""Bitwise A/B of a trainer across two native builds.

Trains a trainer for a few steps (eager, then graph-replayed, including a
tail batch and an eval pass) and dumps parameters, Adam moments, losses and
the eval loss; ``--compare`` checks two dumps for bitwise equality. Used to
show that a kernel restructuring (e.g. the MLP's F2 folded into F3, round 5)
changes no bit of the training trajectory:

    python bench/ab_dump.py --model mlp --out new.npz
    MDT_NATIVE_SO=variants/mlp_r4/_C.so python bench/ab_dump.py --model mlp --out old.npz
    python bench/ab_dump.py --compare old.npz new.npz
"""
from __future__ import annotations

import argparse
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def dump(model: str, out: str, steps: int):
    import torch

    from multidisttorch_amd.ops import native

    dev = torch.device("cuda", 0)
    B = 64 if model == "conv128" else 128
    D = 128 * 128 if model == "conv128" else 784
    n = 6 * B + 40  # six full batches and a tail of 40
    X = torch.rand(n, D, generator=torch.Generator().manual_seed(5)).to(dev)
    idx = torch.randperm(n, generator=torch.Generator().manual_seed(6)).to(torch.int32).to(dev)
    if model == "mlp":
        from multidisttorch_amd.models.mlp_trainer import MlpVaeTrainer

        tr = MlpVaeTrainer(batch_size=B, device=dev, backend="hip", seed=3, use_graphs=False)
    else:
        from multidisttorch_amd.models.conv_vae import ConvVaeTrainer

        im = 128 if model == "conv128" else 28
        tr = ConvVaeTrainer(batch_size=B, image=im, z=64 if im == 128 else 32, device=dev, backend="hip", seed=3,
                            use_graphs=False)
    tr.bind_train_data(X, idx)
    tr.set_cursor(0, 7)
    tr.train_steps(steps)  # eager
    tr.use_graphs = True
    tr.graph_steps = 2
    tr.train_steps(6 - steps % 6 if steps % 6 else 6)
    tr.train_steps(1, M=40)  # tail batch
    total, _ = tr.evaluate(X[:300], torch.arange(300, device=dev, dtype=torch.int32), want_first_recon=False)
    torch.cuda.synchronize()
    st = tr.read_state()
    np.savez(out, params=tr.params.cpu().numpy(), m=tr.exp_avg.cpu().numpy(), v=tr.exp_avg_sq.cpu().numpy(),
             loss=tr.loss_history()[: st["step"]], eval=np.array([total], np.float64),
             so=np.array([native.so_path() if hasattr(native, "so_path") else os.environ.get("MDT_NATIVE_SO", "")]))
    print(f"{out}: {st['step']} steps, eval {total}")


def compare(a: str, b: str) -> int:
    x, y = np.load(a), np.load(b)
    bad = []
    for k in ("params", "m", "v", "loss", "eval"):
        if x[k].shape != y[k].shape or not np.array_equal(x[k].view(np.uint8), y[k].view(np.uint8)):
            d = np.abs(x[k].astype(np.float64) - y[k].astype(np.float64)).max() if x[k].shape == y[k].shape else "shape"
            bad.append(f"{k}: max |diff| {d}")
    print("BITWISE EQUAL" if not bad else "DIFFER: " + "; ".join(bad))
    return 0 if not bad else 1


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="mlp", choices=["mlp", "conv28", "conv128"])
    ap.add_argument("--out")
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--compare", nargs=2)
    a = ap.parse_args()
    if a.compare:
        raise SystemExit(compare(*a.compare))
    dump(a.model, a.out, a.steps)


if __name__ == "__main__":
    main()
