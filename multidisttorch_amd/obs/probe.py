"""Hardware probes: effective shader clock (idle / under a training load),
dependent-load latency per memory tier, and empty-kernel cost (eager vs graph).

Usage (GPU): python -m multidisttorch_amd.obs.probe [--json out.json]
"""

from __future__ import annotations

import argparse
import json
import time

import torch


def _C():
    from ..ops import native

    return native.require()


def clock_mhz(iters: int = 2_000_000, stream=None) -> float:
    C = _C()
    out = torch.zeros(3, dtype=torch.int64, device="cuda")
    with torch.cuda.stream(stream or torch.cuda.current_stream()):
        C.probe_clock(out, iters)
    torch.cuda.synchronize()
    cyc, ticks, _ = out.tolist()
    return cyc / (ticks / 100.0) if ticks else float("nan")  # s_memrealtime = 100 MHz


def latency_cycles(nbytes: int, hops: int = 20000, seed: int = 0) -> float:
    C = _C()
    n = max(2, nbytes // 4)
    g = torch.Generator().manual_seed(seed)
    # single random cycle over a strided subset so every hop is a new line
    stride = 32  # 128 B
    m = n // stride
    perm = torch.randperm(m, generator=g)
    idx = torch.zeros(n, dtype=torch.int32)
    nxt = torch.roll(perm, -1)
    idx[perm * stride] = (nxt * stride).to(torch.int32)
    idx = idx.cuda()
    out = torch.zeros(2, dtype=torch.int64, device="cuda")
    C.probe_latency(idx, 1000, out)  # warm
    C.probe_latency(idx, hops, out)
    torch.cuda.synchronize()
    return out[0].item() / hops


def empty_kernel_us(n: int = 2000, blocks: int = 256, threads: int = 512):
    C = _C()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(n):
        C.probe_empty(blocks, threads)
    torch.cuda.synchronize()
    eager = (time.perf_counter() - t0) / n * 1e6
    g = torch.cuda.CUDAGraph()
    s = torch.cuda.Stream()
    with torch.cuda.stream(s):
        C.probe_empty(blocks, threads)
    torch.cuda.synchronize()
    with torch.cuda.graph(g):
        for _ in range(200):
            C.probe_empty(blocks, threads)
    g.replay()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    reps = max(1, n // 200)
    for _ in range(reps):
        g.replay()
    torch.cuda.synchronize()
    graph = (time.perf_counter() - t0) / (reps * 200) * 1e6
    return eager, graph


def clock_under_training(steps: int = 400) -> float:
    """SCLK measured on a side stream while the fused MLP-VAE step replays."""
    from ..models.mlp_trainer import MlpVaeTrainer

    dev = torch.device("cuda")
    X = torch.rand(60000, 784, device=dev)
    idx = torch.randperm(60000, device=dev).to(torch.int32)
    tr = MlpVaeTrainer(batch_size=128, device=dev, backend="hip", seed=0)
    tr.bind_train_data(X, idx)
    tr.set_cursor(0, 468)
    tr.train_steps(20)
    torch.cuda.synchronize()
    side = torch.cuda.Stream()
    C = _C()
    out = torch.zeros(3, dtype=torch.int64, device="cuda")
    tr.train_steps(steps // 2)
    with torch.cuda.stream(side):
        C.probe_clock(out, 3_000_000)
    tr.train_steps(steps // 2)
    torch.cuda.synchronize()
    cyc, ticks, _ = out.tolist()
    return cyc / (ticks / 100.0)


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--json", default=None)
    a = ap.parse_args(argv)
    res = {}
    res["sclk_idle_mhz"] = clock_mhz()
    res["sclk_idle2_mhz"] = clock_mhz()
    res["lat_cycles_16KB"] = latency_cycles(16 << 10)
    res["lat_cycles_2MB"] = latency_cycles(2 << 20)
    res["lat_cycles_64MB"] = latency_cycles(64 << 20)
    res["lat_cycles_1GB"] = latency_cycles(1 << 30)
    e, g = empty_kernel_us()
    res["empty_kernel_eager_us"], res["empty_kernel_graph_us"] = e, g
    res["sclk_under_training_mhz"] = clock_under_training()
    print(json.dumps(res, indent=1))
    if a.json:
        with open(a.json, "w") as f:
            json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
