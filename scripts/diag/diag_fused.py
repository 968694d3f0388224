"""Diagnostic: where do the fused-reducer and reducer-free 28x28 steps differ?

Per-segment comparison of the f32 gradient arena after ONE step with
f28_skip_adam (finalize only), and of the fused kernel's backward outputs, for
the paired and the solo step; plus the solo step with an extra LDS-dirtying
launch before it (uninitialised-LDS check).

    python scripts/diag/diag_fused.py
"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))


def main():
    from multidisttorch_amd.models.conv_vae import ConvVaeTrainer

    dev = torch.device("cuda", 0)
    X = torch.rand(4 * 128, 784, generator=torch.Generator().manual_seed(3)).to(dev)
    idx = torch.arange(4 * 128, device=dev, dtype=torch.int32)

    def make(pair, fused, overlap=True, skip=True):
        tr = ConvVaeTrainer(batch_size=128, image=28, z=32, device=dev, backend="hip", seed=4, lr=2e-3,
                            use_graphs=False)
        tr.f28_pair = pair
        tr.ddp_overlap = overlap
        tr.f28_skip_adam = skip
        if fused:
            tr.attach_reducer(tr.C.XgmiP2PReducer(0, 1, tr.grads, tr.default_bucket_bounds(), True, 0.0, 64, 20.0,
                                                  -1, True))
        tr.bind_train_data(X, idx)
        tr.set_cursor(0, 4)
        return tr

    def snap(tr):
        d = {n: g.clone() for n, g in tr.named_grads().items()}
        d.update({"gact." + k: v.float().clone() for k, v in tr.gacts.items()})
        d["dmulv"] = tr.dmulv.clone()
        d["f28_bias"] = tr.f28_bias.clone()
        d["f28_part"] = tr.f28_part.clone()
        d["params"] = tr.params.clone()
        return d

    def diff(a, b):
        out = {}
        for k in a:
            m = (a[k] - b[k]).abs().max().item()
            if m != 0.0:
                out[k] = m
        return out

    res = {}
    for pair in (True, False):
        for steps in (1, 2):
            runs = {}
            for name, fused, overlap in (("free", False, True), ("fused_ov", True, True), ("fused_noov", True, False)):
                tr = make(pair, fused, overlap, skip=steps == 1)
                tr.train_steps(steps)
                torch.cuda.synchronize()
                runs[name] = snap(tr)
            res[f"pair{int(pair)}_steps{steps}"] = {k: diff(runs["free"], v) for k, v in runs.items() if k != "free"}
        # uninitialised-LDS probe: same reducer-free trial, with an LDS-heavy launch in front of each step
        a, b = make(pair, False, skip=False), make(pair, False, skip=False)
        for _ in range(3):
            a.train_steps(1)
            b._transpose_weights()  # wtrans_k: fills LDS with weight tiles
            b.train_steps(1)
        torch.cuda.synchronize()
        res[f"pair{int(pair)}_lds_dirty"] = diff(snap(a), snap(b))
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
