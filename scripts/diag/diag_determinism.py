"""Run-to-run determinism of the fused 28x28 step (paired and solo forms).

Trains the same trial N times from scratch (eager, 8 steps), optionally with a
stream of unrelated GEMMs beside it, and reports how many distinct results
(loss history + parameters) came out, and -- for the paired launch -- how many
samples fell back to the one-workgroup form in each step (stamp slot 15).

    python scripts/diag/diag_determinism.py [--runs 6] [--json out.json]
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--runs", type=int, default=6)
    ap.add_argument("--steps", type=int, default=8)
    ap.add_argument("--json", default=None)
    a = ap.parse_args()
    from multidisttorch_amd.models.conv_vae import ConvVaeTrainer

    dev = torch.device("cuda", 0)
    X = torch.rand(4 * 128, 784, generator=torch.Generator().manual_seed(3)).to(dev)
    idx = torch.arange(4 * 128, device=dev, dtype=torch.int32)
    out = {}
    for pair in (True, False):
        for noisy in (False, True):
            results, fallbacks, nears = [], [], []
            for r in range(a.runs):
                tr = ConvVaeTrainer(batch_size=128, image=28, z=32, device=dev, backend="hip", seed=4, lr=2e-3,
                                    use_graphs=False)
                tr.f28_pair = pair
                stamps = torch.zeros(2 * 128 * 16, dtype=torch.int64, device=dev)
                tr.f28_stamps = (stamps, None)
                tr.bind_train_data(X, idx)
                tr.set_cursor(0, 4)
                side = torch.cuda.Stream()
                junk = torch.rand(2048, 2048, device=dev)
                fb, nr = [], []
                for _ in range(a.steps):
                    if noisy:
                        with torch.cuda.stream(side):
                            for _ in range(4):
                                junk = junk @ junk
                                junk = junk / junk.norm()
                    tr.train_steps(1)
                    if pair:
                        s = stamps.view(256, 16)[:, 15].cpu()
                        modes = s & 15
                        fb.append(int((modes == 0).sum()))
                        nr.append(int(((s >> 4) & 1).sum()))
                torch.cuda.synchronize()
                results.append((tr.loss_history()[:a.steps].tolist(), tr.params.clone()))
                fallbacks.append(fb)
                nears.append(nr)
            distinct = []
            for h, p in results:
                if not any(h == h2 and torch.equal(p, p2) for h2, p2 in distinct):
                    distinct.append((h, p))
            key = f"pair{int(pair)}_noisy{int(noisy)}"
            out[key] = {"distinct_results": len(distinct), "runs": a.runs,
                        "solo_fallbacks_per_step": fallbacks if pair else None,
                        "near_workgroups_per_step": nears if pair else None,
                        "max_param_spread": max((p - results[0][1]).abs().max().item() for _, p in results)}
            print(key, json.dumps({k: v for k, v in out[key].items() if k != "near_workgroups_per_step"}), flush=True)
    if a.json:
        with open(a.json, "w") as f:
            json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
