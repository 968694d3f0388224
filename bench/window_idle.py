#!/usr/bin/env python3
"""Fixed cost of a timed window, by cause (round 5): host wall of one 20-step
graph replay bracketed by device syncs (bench.py's bracket) as a function of
(a) how long the device sat idle before t0 (host busy-wait, no sleep), and
(b) whether the graph had been replayed before (first replay of a freshly
captured + uploaded graph vs later ones).

    python bench/window_idle.py [--model conv28|mlp]
"""
import argparse
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def spin(sec):
    t = time.perf_counter()
    while time.perf_counter() - t < sec:
        pass


def window(tr, S, M, gap):
    torch.cuda.synchronize()
    spin(gap)
    t0 = time.perf_counter()
    tr._replay(S, M)
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) * 1e6


def make(model, dev, train, S):
    if model == "mlp":
        from multidisttorch_amd.models.mlp_trainer import MlpVaeTrainer

        tr = MlpVaeTrainer(batch_size=128, device=dev, backend="hip", seed=1, use_graphs=True, graph_steps=S)
    else:
        from multidisttorch_amd.models.conv_vae import ConvVaeTrainer

        tr = ConvVaeTrainer(batch_size=128, image=28, z=32, device=dev, backend="hip", seed=1, use_graphs=True,
                            graph_steps=S)
    idx = torch.arange(len(train), device=dev, dtype=torch.int32)
    tr.bind_train_data(train.data, idx)
    tr.set_cursor(0, idx.numel() // 128)
    tr.prepare([128])
    return tr


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="conv28")
    a = ap.parse_args()
    from multidisttorch_amd.data.datasets import mnist_like

    dev = torch.device("cuda", 0)
    train = mnist_like(True, synthetic=True, device=dev, size=28)
    S, M = 20, 128
    # (b) first replays of fresh trainers, right after prepare() + 5 single warm-up steps (bench.py's order)
    for rep in range(3):
        tr = make(a.model, dev, train, S)
        tr.train_steps(5)
        torch.cuda.synchronize()
        w = [window(tr, S, M, 0.0) for _ in range(4)]
        print(f"fresh trainer {rep}: replays 1..4 of the 20-step graph: " + ", ".join(f"{x:.1f}" for x in w) + " us",
              flush=True)
    # (a) idle gap before t0
    for gap in (0.0, 20e-6, 100e-6, 500e-6, 2e-3, 10e-3):
        ws = sorted(window(tr, S, M, gap) for _ in range(7))
        print(f"idle {gap * 1e6:7.0f} us before t0: window median {ws[3]:8.1f} us ({ws[3] / S:.2f} us/step), "
              f"min {ws[0]:.1f}", flush=True)


if __name__ == "__main__":
    main()
