#!/usr/bin/env python3
"""Trial packing on one MI355X: T independent trials, each on its own HIP
stream, replaying its captured step graphs concurrently.

Reports aggregate samples/s for T = 1, 2, 4, 8 (and per-trial ms/step).
usage: python bench/packing.py [--model mlp|conv28|conv128] [--steps 200]
"""
import argparse
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def make(model, dev, seed, B):
    if model == "mlp":
        from multidisttorch_amd.models.mlp_trainer import MlpVaeTrainer

        return MlpVaeTrainer(batch_size=B, device=dev, backend="hip", seed=seed, use_graphs=True, graph_steps=10)
    from multidisttorch_amd.models.conv_vae import ConvVaeTrainer

    img = 28 if model == "conv28" else 128
    return ConvVaeTrainer(batch_size=B, image=img, z=32 if img == 28 else 64, device=dev, backend="hip", seed=seed,
                          use_graphs=True, graph_steps=10)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="mlp")
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--batch", type=int, default=None)
    ap.add_argument("--trials", default="1,2,4,8")
    a = ap.parse_args()
    from multidisttorch_amd.data.datasets import mnist_like

    dev = torch.device("cuda", 0)
    B = a.batch or (128 if a.model != "conv128" else 64)
    img = 128 if a.model == "conv128" else 28
    data = mnist_like(True, synthetic=True, device=dev, size=img, n=None if img == 28 else 4096)
    out = []
    for T in [int(x) for x in a.trials.split(",")]:
        trs, streams = [], []
        for t in range(T):
            tr = make(a.model, dev, t, B)
            idx = torch.arange(t * 1000 % 2048, t * 1000 % 2048 + 2048, device=dev, dtype=torch.int32) % len(data)
            tr.bind_train_data(data.data, idx)
            tr.set_cursor(0, idx.numel() // B)
            s = torch.cuda.Stream()
            with torch.cuda.stream(s):
                tr.train_steps(20)  # capture + warm
            trs.append(tr)
            streams.append(s)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for tr, s in zip(trs, streams):
            with torch.cuda.stream(s):
                tr.train_steps(a.steps)
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        ok = all(tr.read_state()["step"] == 20 + a.steps for tr in trs)
        r = dict(model=a.model, trials=T, batch=B, steps=a.steps, seconds=round(dt, 4),
                 samples_per_s=round(T * B * a.steps / dt, 1), ms_per_step_per_trial=round(dt / a.steps * 1e3, 4),
                 valid=ok)
        out.append(r)
        print(json.dumps(r), flush=True)
        del trs, streams
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
