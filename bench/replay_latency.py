#!/usr/bin/env python3
"""Host latency of a step-graph replay call (hipGraphLaunch of S fused 28x28
steps) and the wall time of one S-step window started from an idle device,
for S = 1, 10, 20: how much of a short timed window is graph submission."""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    from multidisttorch_amd.data.datasets import mnist_like
    from multidisttorch_amd.models.conv_vae import ConvVaeTrainer

    dev = torch.device("cuda", 0)
    train = mnist_like(True, synthetic=True, device=dev, size=28)
    idx = torch.arange(len(train), device=dev, dtype=torch.int32)
    for S in (1, 10, 20):
        tr = ConvVaeTrainer(batch_size=128, image=28, z=32, device=dev, backend="hip", seed=1,
                            use_graphs=True, graph_steps=S)
        tr.bind_train_data(train.data, idx)
        tr.set_cursor(0, idx.numel() // 128)
        tr.prepare([128])
        tr.train_steps(S * 3)
        torch.cuda.synchronize()
        g = tr._graphs[(S, 128)]
        calls, walls = [], []
        for _ in range(10):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            g.replay()
            t1 = time.perf_counter()
            torch.cuda.synchronize()
            t2 = time.perf_counter()
            calls.append((t1 - t0) * 1e6)
            walls.append((t2 - t0) * 1e6)
        calls.sort()
        walls.sort()
        print(f"S={S:2d}: replay() call {calls[5]:7.1f} us, window {walls[5]:8.1f} us = {walls[5] / S:6.1f} us/step",
              flush=True)


if __name__ == "__main__":
    main()
