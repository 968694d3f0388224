"""Per-workgroup start / end stamps of the 28x28 step's finalize + Adam work:
how long one finalize unit's workgroup runs against how long the launch spans.

    python bench/finalize_stamps.py [--reps 6]

The finalize units of a real plan are packed as ONE job of a stamped
jobs_multi_k launch (the same grad_finalize_body the stand-alone
grad_finalize_k runs) and launched after real steps; the parameters it
updates are restored afterwards, so this is timing only. Stamps are
s_memrealtime (100 MHz) at workgroup entry and exit, relative to the first
entry; the launch is also timed with events around it.
"""
import argparse
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=6)
    a = ap.parse_args()
    from multidisttorch_amd.data.datasets import synthetic_images
    from multidisttorch_amd.models.conv_vae import ConvVaeTrainer

    dev = torch.device("cuda", 0)
    B = 128
    tr = ConvVaeTrainer(batch_size=B, image=28, device=dev, backend="hip", seed=0, use_graphs=False)
    X = synthetic_images(8 * B, device=dev)
    tr.bind_train_data(X, torch.arange(8 * B, device=dev, dtype=torch.int32))
    tr.set_cursor(0, 8)
    tr.train_steps(2)
    torch.cuda.synchronize()
    C, p, st = tr.C, tr._plan28(B), tr.state
    j = C.Job()
    C.grad_finalize(tr.params, tr.grads, tr.exp_avg, tr.exp_avg_sq, tr.w16, p["segs"], p["units"], p["nunits"],
                    st.train_state, st.hparams, True, job=j)
    grid = j.nblk
    stamps = torch.zeros(2 * grid, dtype=torch.int64, device=dev)
    pack, g2 = C.pack_jobs_multi([j], stamps=stamps)
    assert g2 == grid
    pack = pack.to(dev)
    keep = [t.clone() for t in (tr.params, tr.exp_avg, tr.exp_avg_sq, tr.w16)]
    durs, starts, spans, ev_us = [], [], [], []
    for _ in range(a.reps):
        tr.train_steps(1)
        stamps.zero_()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        C.launch_jobs_multi(pack, grid)
        e1.record()
        torch.cuda.synchronize()
        s = stamps.view(grid, 2).cpu().numpy().astype(np.int64)
        t0 = s[:, 0].min()
        us = (s - t0) * 10 / 1000.0
        durs.append(us[:, 1] - us[:, 0])
        starts.append(us[:, 0])
        spans.append(us[:, 1].max())
        ev_us.append(e0.elapsed_time(e1) * 1000.0)
    for t, v in zip((tr.params, tr.exp_avg, tr.exp_avg_sq, tr.w16), keep):
        t.copy_(v)
    d = np.stack(durs[1:])
    print(f"finalize units: {grid} workgroups")
    print(f"  workgroup duration us: median {np.median(d):.2f}  p90 {np.percentile(d, 90):.2f}  max {np.median(d.max(1)):.2f}")
    print(f"  workgroup start us: median {np.median(np.stack(starts[1:])):.2f}  last {np.median(np.stack(starts[1:]).max(1)):.2f}")
    print(f"  first entry -> last exit us: {np.median(spans[1:]):.2f}")
    print(f"  event-timed launch us: {np.median(ev_us[1:]):.2f}")
    lu = p["layer_units"]
    for i, l in enumerate(tr.spec):
        u0, u1 = lu[i], lu[i + 1]
        dl = d[:, u0:u1]
        print(f"  {l.name:9s} units {u1 - u0:4d}  duration median {np.median(dl):.2f}  max {np.median(dl.max(1)):.2f}")


if __name__ == "__main__":
    main()
