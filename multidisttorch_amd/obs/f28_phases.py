"""Per-phase timing of the fused 28x28 step (csrc/kernels/conv28_fused.hip).

Every workgroup writes an s_memrealtime stamp (100 MHz, chip-global) when it
enters each phase; this tool runs a few eager steps with stamping on and
prints, per phase, the median and max duration over the workgroups and the
spread of the workgroups' start times (dispatch skew). Phase boundaries are
workgroup barriers, so a phase's duration includes waiting for its slowest
wave. Default: the paired step (two workgroups per sample, conv28_pair.h;
slot 15 of a row records the workgroup's mode). ``--solo`` times the
two-launch one-workgroup-per-sample forward / backward instead.

    python -m multidisttorch_amd.obs.f28_phases [--batch 128] [--steps 3] [--solo] [--json out.json]
"""

from __future__ import annotations

import argparse
import json

import numpy as np
import torch

FWD = ["P0 gather+stage", "P1 enc1", "P2 enc2", "P3 head", "P4 reparam", "P5 dec_fc", "P6 dec1", "P7 dec2+BCE"]
BWD = ["Q0 load+stage", "Q1 dec2 bwd", "Q2 dec1 bwd", "Q3 dec_fc bwd", "Q4 reparam bwd", "Q5 head bwd",
       "Q6 enc2 bwd"]
PAIR = ["P0 gather+stage", "P1 enc1", "P2 enc2 (half)", "P3 head (K half)", "X1+P4 reparam", "P5 dec_fc+X2",
        "P6 dec1 (half)", "P7 dec2+X3+BCE", "Q1 dec2 bwd+X4", "Q2 dec1 bwd (half)", "Q3 dec_fc bwd (half)",
        "X5+Q4 reparam bwd", "Q5 head bwd+X6", "Q6 enc2 bwd (half)"]
MODES = {0: "solo", 1: "role0", 2: "role1", 3: "exit"}


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
    ap.add_argument("--solo", action="store_true")
    a = ap.parse_args(argv)
    from multidisttorch_amd.data.datasets import synthetic_images
    from multidisttorch_amd.models.conv_vae import ConvVaeTrainer

    dev = torch.device("cuda", 0)
    B = a.batch
    tr = ConvVaeTrainer(batch_size=B, image=28, device=dev, backend="hip", seed=0, use_graphs=False)
    assert tr.f28, "fused 28x28 step disabled (MDT_CONV_F28=0?)"
    tr.f28_stamps = (torch.zeros(2 * B * 16, dtype=torch.int64, device=dev),
                     torch.zeros(2 * B * 16, dtype=torch.int64, device=dev))
    if a.solo:
        tr.f28_merge = False
    X = synthetic_images(8 * B, device=dev)
    tr.bind_train_data(X, torch.arange(8 * B, device=dev, dtype=torch.int32))
    tr.set_cursor(0, 8)
    res = []
    if not a.solo:
        return _pair(tr, B, a)
    for _ in range(a.steps):
        tr.train_steps(1)
        torch.cuda.synchronize()
        f = tr.f28_stamps[0].view(2 * B, 16)[:B].cpu().numpy()
        b = tr.f28_stamps[1].view(2 * B, 16)[:B].cpu().numpy()
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


def _pair(tr, B, a):
    res = []
    for _ in range(a.steps):
        tr.f28_stamps[0].zero_()
        tr.train_steps(1)
        torch.cuda.synchronize()
        st = tr.f28_stamps[0].view(2 * B, 16).cpu().numpy()
        modes, near = st[:, 15] & 15, st[:, 15] >> 4
        counts = {MODES[int(m)]: int((modes == m).sum()) for m in np.unique(modes)}
        paired = st[(modes == 1) | (modes == 2)]
        r = {"modes": counts, "err": int(tr.f28_err.item()), "same_xcd": int(near[(modes == 1) | (modes == 2)].sum())}
        if len(paired):
            r["pair"] = summarize(paired, PAIR)
        res.append(r)
    last = res[-1]
    print("workgroup modes:", last["modes"], "same-XCD paired workgroups:", last["same_xcd"],
          "exchange timeouts:", last["err"])
    if "pair" in last:
        pr = last["pair"]
        print(f"pair: kernel {pr['kernel_us']:.2f} us, start skew {pr['start_skew_us']:.2f} us")
        for n in PAIR:
            v = pr[n]
            print(f"   {n:22s} median {v['median_us']:7.2f}  max {v['max_us']:7.2f} us")
    if a.json:
        with open(a.json, "w") as fh:
            json.dump(res, fh, indent=1)
    return res


if __name__ == "__main__":
    main()
