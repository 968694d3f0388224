"""Diagnostic: two reducer-free 28x28 trainers stepped in lockstep (eager),
every per-step buffer compared after each step; the first buffer that
differs (in pipeline order) names the launch whose result moved.

Context first (what test_fused_comm does before its failing cases): fused
-reducer trainers built and run, kept alive.

    python scripts/diag/diag_lockstep.py [--pairs 10] [--pair 0]
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--pairs", type=int, default=10)
    ap.add_argument("--pair", type=int, default=0)
    ap.add_argument("--context", type=int, default=1)
    a = ap.parse_args()
    from multidisttorch_amd.models.conv_vae import ConvVaeTrainer

    dev = torch.device("cuda", 0)
    nb, steps = 4, 8
    X = torch.rand(nb * 128, 784, generator=torch.Generator().manual_seed(3)).to(dev)
    idx = torch.arange(nb * 128, device=dev, dtype=torch.int32)

    def make(pair, graphs=False, fused=False, overlap=True):
        tr = ConvVaeTrainer(batch_size=128, image=28, z=32, device=dev, backend="hip", seed=4, lr=2e-3,
                            use_graphs=graphs, graph_steps=4)
        tr.f28_pair = pair
        tr.ddp_overlap = overlap
        if fused:
            tr.attach_reducer(tr.C.XgmiP2PReducer(0, 1, tr.grads, tr.default_bucket_bounds(), True, 0.0, 64, 20.0,
                                                  -1, True))
        tr.bind_train_data(X, idx)
        tr.set_cursor(0, nb)
        return tr

    keep = []
    if a.context:
        for pair in (True, False):
            for graphs in (False, True):
                t = make(pair, graphs, fused=True)
                t.train_steps(steps)
                keep.append(t)
        torch.cuda.synchronize()

    def buffers(tr):
        p = tr._plan28(128)
        b = {"xb": tr.xb, "mulv": tr.mulv, "eps": tr.eps, "z16": tr.z16, "dlog32": tr.dlog32}
        b.update({"act." + k: v for k, v in tr.acts.items()})
        b.update({"gact." + k: v for k, v in tr.gacts.items()})
        b.update({"dmulv": tr.dmulv, "f28_bias": tr.f28_bias, "f28_part": tr.f28_part})
        b.update({"slab." + k: t for k, (t, _) in p["slabs"].items() if k.endswith(".weight")})
        b.update({"params": tr.params, "exp_avg": tr.exp_avg, "exp_avg_sq": tr.exp_avg_sq, "w16": tr.w16,
                  "state": tr.state.train_state})
        return b

    events = []
    for r in range(a.pairs):
        A, B = make(bool(a.pair)), make(bool(a.pair))
        for s in range(steps):
            A.train_steps(1)
            torch.cuda.synchronize()
            B.train_steps(1)
            torch.cuda.synchronize()
            ba, bb = buffers(A), buffers(B)
            diff = [k for k in ba if not torch.equal(ba[k], bb[k])]
            if diff:
                detail = {k: float((ba[k].float() - bb[k].float()).abs().max()) for k in diff if ba[k].is_floating_point()}
                nz = {k: int((ba[k] != bb[k]).sum()) for k in diff}
                ev = {"pair_run": r, "step": s, "differ": diff, "max_abs": detail, "count": nz}
                events.append(ev)
                print(json.dumps(ev), flush=True)
                break
    print(json.dumps({"runs": a.pairs, "diverged": len(events)}))


if __name__ == "__main__":
    main()
