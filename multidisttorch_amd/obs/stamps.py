"""In-kernel phase timestamps of the fused MLP-VAE step (s_memrealtime, 100 MHz).

Runs a few eager steps with the engine's stamp buffer attached and reports,
per kernel: span (first wave start -> last wave end), gap to the next kernel,
and the median / max duration of each instrumented phase across waves.
Usage (GPU): python -m multidisttorch_amd.obs.stamps [--json out.json]
"""

from __future__ import annotations

import argparse
import json

import numpy as np
import torch

KERNELS = ["F1", "F2", "F3", "B1", "B2", "B3"]
SLOTS = 8
BLOCKS = 512
WAVES = 8


def collect(steps: int = 20, M: int = 128):
    from ..models.mlp_trainer import MlpVaeTrainer

    dev = torch.device("cuda")
    X = torch.rand(60000, 784, device=dev)
    idx = torch.randperm(60000, device=dev).to(torch.int32)
    tr = MlpVaeTrainer(batch_size=M, device=dev, backend="hip", seed=0, use_graphs=False)
    tr.bind_train_data(X, idx)
    tr.set_cursor(0, 468)
    buf = torch.zeros(len(KERNELS) * BLOCKS * WAVES * SLOTS, dtype=torch.int64, device=dev)
    tr.engine.set_stamps(buf)
    tr.train_steps(steps - 1)
    torch.cuda.synchronize()
    buf.zero_()
    tr.train_steps(1)
    torch.cuda.synchronize()
    tr.engine.set_stamps(torch.empty(0, dtype=torch.int64, device=dev))
    return buf.view(len(KERNELS), BLOCKS, WAVES, SLOTS).cpu().numpy().astype(np.int64)


def _ranges(M=128, D=784, H=400, Z=20, fuse=True):
    """Block index ranges of the grouped kernels (mirrors vae_grid in vae_mlp.hip)."""
    cd = lambda a, b: -(-a // b)
    ti = cd(M, 16)
    wg = lambda o, i: cd(cd(o, 32) * cd(i, 32), 2)
    b1 = ti * cd(H, 16)
    b2r = ti * cd(cd(H, 16), 8)
    b2w = wg(H, Z)
    b3w2, b3w1 = wg(2 * Z, H), wg(H, D)
    return {"B1": [("dh3", 0, b1), ("dW4", b1, b1 + wg(D, H))],
            "B2": [("rows", 0, b2r), ("dW3", b2r, b2r + b2w), ("loss", b2r + b2w, b2r + b2w + 1)],
            "B3": [("dW2", 0, b3w2), ("dW1", b3w2, b3w2 + b3w1), ("adam", b3w2 + b3w1, BLOCKS)]}


def analyse(st: np.ndarray) -> dict:
    out = {}
    rng = _ranges()
    spans = []
    for k, name in enumerate(KERNELS):
        s = st[k]
        valid = s[:, :, 0] > 0
        if not valid.any():
            continue
        starts = s[:, :, 0][valid]
        last = np.max(s, axis=2)[valid]
        t0, t1 = starts.min(), last.max()
        spans.append((name, t0, t1))
        phases = {}
        for sl in range(1, SLOTS):
            a, b = s[:, :, sl - 1], s[:, :, sl]
            m = valid & (a > 0) & (b > 0)
            if m.any():
                d = (b - a)[m] * 10e-3  # 10 ns ticks -> us
                phases[f"p{sl-1}->{sl}"] = dict(median_us=float(np.median(d)), max_us=float(d.max()), n=int(m.sum()))
        out[name] = dict(span_us=float((t1 - t0) * 10e-3), waves=int(valid.sum()),
                         start_skew_us=float((starts.max() - starts.min()) * 10e-3), phases=phases)
        for label, lo, hi in rng.get(name, []):
            sub = s[lo:hi]
            v2 = sub[:, :, 0] > 0
            if v2.any():
                dur = (np.max(sub, axis=2) - sub[:, :, 0])[v2] * 10e-3
                out[name][f"part_{label}"] = dict(median_us=float(np.median(dur)), max_us=float(dur.max()),
                                                  end_us=float((np.max(sub, axis=2)[v2].max() - t0) * 10e-3))
    for (n0, a0, b0), (n1, a1, b1) in zip(spans, spans[1:]):
        out[n0]["gap_to_next_us"] = float((a1 - b0) * 10e-3)
    if spans:
        out["step_span_us"] = float((spans[-1][2] - spans[0][1]) * 10e-3)
    return out


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--json", default=None)
    a = ap.parse_args(argv)
    res = analyse(collect())
    print(json.dumps(res, indent=1))
    if a.json:
        with open(a.json, "w") as f:
            json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
