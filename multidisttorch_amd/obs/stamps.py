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
    b2w4 = wg(D, H)
    return {"B1": [("dh3", 0, b1)],
            "B2": [("rows", 0, b2r), ("dW3", b2r, b2r + b2w), ("dW4", b2r + b2w, b2r + b2w + b2w4),
                   ("loss", b2r + b2w + b2w4, b2r + b2w + b2w4 + 1)],
            "B3": [("dW2", 0, b3w2), ("dW1", b3w2, b3w2 + b3w1), ("adam", b3w2 + b3w1, BLOCKS)]}


def placement(st: np.ndarray) -> dict:
    """Per kernel: how many CUs ran its blocks, and block durations split by
    whether another block of the same kernel overlapped it on the same CU
    (slot 7 = XCC/CU id of the wave, written with slot 0)."""
    out = {}
    for k, name in enumerate(KERNELS):
        s = st[k]
        v = s[:, 0, 0] > 0
        if not v.any():
            continue
        blocks = np.nonzero(v)[0]
        t0 = np.where(s[blocks, :, 0] > 0, s[blocks, :, 0], np.iinfo(np.int64).max).min(axis=1)
        t1 = s[blocks, :, :7].max(axis=(1, 2))
        cu = s[blocks, 0, 7]
        shared = np.zeros(len(blocks), bool)
        per_cu = {}
        for i, c in enumerate(cu):
            per_cu.setdefault(int(c), []).append(i)
        for idxs in per_cu.values():
            for i in idxs:
                for j in idxs:
                    if i != j and t0[i] < t1[j] and t0[j] < t1[i]:
                        shared[i] = True
        d = (t1 - t0) * 10e-3
        rec = dict(blocks=int(len(blocks)), cus=len(per_cu), max_blocks_per_cu=max(len(x) for x in per_cu.values()),
                   shared_blocks=int(shared.sum()))
        for lab, m in (("alone", ~shared), ("shared", shared)):
            if m.any():
                rec[f"dur_{lab}_median_us"] = float(np.median(d[m]))
                rec[f"dur_{lab}_max_us"] = float(d[m].max())
        for label, lo, hi in _ranges().get(name, []):
            m = (blocks >= lo) & (blocks < hi)
            if m.any():
                rec[f"{label}_shared"] = int((shared & m).sum())
                rec[f"{label}_n"] = int(m.sum())
                rec[f"{label}_start_last_us"] = float((t0[m].max() - t0.min()) * 10e-3)
        out[name] = rec
    return out


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
    ap.add_argument("--raw", default=None, help="save the raw stamp array (.npy)")
    a = ap.parse_args(argv)
    st = collect()
    if a.raw:
        np.save(a.raw, st)
    res = analyse(st)
    res["placement"] = placement(st)
    print(json.dumps(res, indent=1))
    if a.json:
        with open(a.json, "w") as f:
            json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
