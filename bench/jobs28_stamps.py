"""Per-workgroup start / end stamps of the 28x28 step's weight-gradient launch
(`jobs_multi_k`: the six weight-gradient jobs + the loss/step job), taken
inside real eager steps: which job's workgroups finish last, and how long the
blocks of each job run.

    python bench/jobs28_stamps.py [--steps 6] [--json out.json]

Stamps are s_memrealtime (100 MHz) written by every workgroup at entry and
exit (`pack_jobs_multi(..., stamps=)`), relative to the earliest start.
"""
import argparse
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=6)
    ap.add_argument("--json", default=None)
    ap.add_argument("--merged", action="store_true", help="the merged table: + gather + per-layer finalize jobs")
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
    C, p = tr.C, tr._plan28(B)
    names = ["enc1", "enc2", "enc_head", "dec_fc", "dec1", "dec2", "loss"]
    if a.merged:
        tr.f28_fin_merge = True  # MDT_F28_FIN_MERGE's form for this trainer
        _, _, jobs, wait = tr._merged_pack28(p)
        names += (["gather"] if tr.f28_prefetch else []) + ["fin_" + n for n in tr._FIN_ORDER28]
    else:
        tr.f28_fin_merge = False
        jobs, wait = p["jobs"], []
    nblk = [j.nblk for j in jobs]
    grid0 = sum(nblk)
    stamps = torch.zeros(2 * grid0, dtype=torch.int64, device=dev)
    pack, grid = C.pack_jobs_multi(jobs, stamps=stamps, wait=wait, dep_ctr=tr.f28_dep if wait else None)
    assert grid == grid0
    if a.merged:
        p[("merged", True, bool(tr.f28_prefetch))] = (pack.to(dev), grid, jobs, wait)
    else:
        p["jobs_pack"], p["jobs_grid"] = pack.to(dev), grid
    runs = []
    for _ in range(a.steps):
        stamps.zero_()
        tr.train_steps(1)
        torch.cuda.synchronize()
        s = stamps.view(grid, 2).cpu().numpy().astype(np.int64)
        t0 = s[:, 0].min()
        runs.append(((s - t0) * 10).astype(np.float64) / 1000.0)  # us
    res = {"grid": grid, "jobs": {}}
    per = np.stack(runs[1:])  # [steps-1][grid][2], first step dropped
    off = 0
    for n, k in zip(names, nblk):
        blk = per[:, off:off + k]
        dur = blk[..., 1] - blk[..., 0]
        res["jobs"][n] = dict(blocks=k, start_med=float(np.median(blk[..., 0])), end_max=float(np.median(blk[..., 1].max(1))),
                              dur_med=float(np.median(dur)), dur_max=float(np.median(dur.max(1))))
        off += k
    res["kernel_us"] = float(np.median(per[..., 1].max(1)))
    print(f"jobs_multi_k grid {grid}: kernel (first start -> last end) {res['kernel_us']:.2f} us")
    for n, r in res["jobs"].items():
        print(f"  {n:12s} blocks {r['blocks']:4d}  start med {r['start_med']:5.2f}  block dur med {r['dur_med']:5.2f} "
              f"max {r['dur_max']:5.2f}  last end {r['end_max']:5.2f} us")
    if a.json:
        with open(a.json, "w") as f:
            json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
