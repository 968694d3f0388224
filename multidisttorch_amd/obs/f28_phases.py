"""Per-phase timing of the fused 28x28 step (csrc/kernels/conv28_fused.hip).

Every workgroup of f28_fwd_k / f28_bwd_k writes an s_memrealtime stamp
(100 MHz, chip-global) when it enters each phase; this tool runs a few eager
steps with stamping on and prints, per phase, the median and max duration
over the workgroups and the spread of the workgroups' start times (dispatch
skew). Phase boundaries are workgroup barriers, so a phase's duration
includes waiting for its slowest wave.

    python -m multidisttorch_amd.obs.f28_phases [--batch 128] [--steps 3] [--json out.json]
"""

from __future__ import annotations

import argparse
import json

import numpy as np
import torch

FWD = ["P0 gather+stage", "P1 enc1", "P2 enc2", "P3 head", "P4 reparam", "P5 dec_fc", "P6 dec1", "P7 dec2+BCE"]
BWD = ["Q0 load+stage", "Q1 dec2 bwd", "Q2 dec1 bwd", "Q3 dec_fc bwd", "Q4 reparam bwd", "Q5 head bwd",
       "Q6 enc2 bwd"]


def summarize(st: np.ndarray, names):
    """st: int64 [M][16] stamps (slots 0..len(names)). Returns a dict of µs stats."""
    st = st.astype(np.float64) * 0.01  # 100 MHz ticks -> µs
    out = {"start_skew_us": float(st[:, 0].max() - st[:, 0].min()),
           "kernel_us": float(st[:, len(names)].max() - st[:, 0].min())}
    for i, n in enumerate(names):
        d = st[:, i + 1] - st[:, i]
        out[n] = {"median_us": round(float(np.median(d)), 3), "max_us": round(float(d.max()), 3)}
    return out


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=128)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--json", default=None)
    a = ap.parse_args(argv)
    from multidisttorch_amd.data.datasets import synthetic_images
    from multidisttorch_amd.models.conv_vae import ConvVaeTrainer

    dev = torch.device("cuda", 0)
    B = a.batch
    tr = ConvVaeTrainer(batch_size=B, image=28, device=dev, backend="hip", seed=0, use_graphs=False)
    assert tr.f28, "fused 28x28 step disabled (MDT_CONV_F28=0?)"
    tr.f28_stamps = (torch.zeros(B * 16, dtype=torch.int64, device=dev),
                     torch.zeros(B * 16, dtype=torch.int64, device=dev))
    X = synthetic_images(8 * B, device=dev)
    tr.bind_train_data(X, torch.arange(8 * B, device=dev, dtype=torch.int32))
    tr.set_cursor(0, 8)
    res = []
    for _ in range(a.steps):
        tr.train_steps(1)
        torch.cuda.synchronize()
        f = tr.f28_stamps[0].view(B, 16).cpu().numpy()
        b = tr.f28_stamps[1].view(B, 16).cpu().numpy()
        r = {"fwd": summarize(f, FWD), "bwd": summarize(b, BWD),
             "fwd_end_to_bwd_start_us": float((b[:, 0].min() - f[:, len(FWD)].max()) * 0.01)}
        res.append(r)
    last = res[-1]
    for k in ("fwd", "bwd"):
        print(f"{k}: kernel {last[k]['kernel_us']:.2f} us, start skew {last[k]['start_skew_us']:.2f} us")
        for n in (FWD if k == "fwd" else BWD):
            v = last[k][n]
            print(f"   {n:18s} median {v['median_us']:7.2f}  max {v['max_us']:7.2f} us")
    print(f"fwd end -> bwd start: {last['fwd_end_to_bwd_start_us']:.2f} us")
    if a.json:
        with open(a.json, "w") as fh:
            json.dump(res, fh, indent=1)


if __name__ == "__main__":
    main()
