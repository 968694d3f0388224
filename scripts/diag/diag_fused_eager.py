"""Diagnostic: which side of test_fused_comm's eager comparison moves?

For each (overlap, pair) it trains the same 8-step trial four ways --
reducer-free eager, reducer-free graphs, fused-reducer eager, fused-reducer
graphs -- three times each (fresh trainers), and prints how many distinct
results each way produced and which ways agree with each other.

    python scripts/diag/diag_fused_eager.py
"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))


def main():
    from multidisttorch_amd.models.conv_vae import ConvVaeTrainer

    dev = torch.device("cuda", 0)
    nb, steps = 4, 8
    X = torch.rand(nb * 128, 784, generator=torch.Generator().manual_seed(3)).to(dev)
    idx = torch.arange(nb * 128, device=dev, dtype=torch.int32)

    def run(graphs, pair, overlap, fused):
        tr = ConvVaeTrainer(batch_size=128, image=28, z=32, device=dev, backend="hip", seed=4, lr=2e-3,
                            use_graphs=graphs, graph_steps=4)
        tr.f28_pair = pair
        tr.ddp_overlap = overlap
        if fused:
            red = tr.C.XgmiP2PReducer(0, 1, tr.grads, tr.default_bucket_bounds(), True, 0.0, 64, 20.0, -1, True)
            tr.attach_reducer(red)
        tr.bind_train_data(X, idx)
        tr.set_cursor(0, nb)
        tr.train_steps(steps)
        torch.cuda.synchronize()
        return tr.loss_history()[:steps].tolist(), tr.params.clone()

    out = {}
    for overlap in (True, False):
        for pair in (True, False):
            ways = {}
            for name, graphs, fused in (("free_eager", False, False), ("free_graph", True, False),
                                        ("fused_eager", False, True), ("fused_graph", True, True)):
                ways[name] = [run(graphs, pair, overlap, fused) for _ in range(3)]
            reps = {}
            classes = []  # distinct results over every run of every way
            for name, runs in ways.items():
                ids = []
                for h, p in runs:
                    for ci, (h2, p2) in enumerate(classes):
                        if h == h2 and torch.equal(p, p2):
                            ids.append(ci)
                            break
                    else:
                        classes.append((h, p))
                        ids.append(len(classes) - 1)
                reps[name] = ids
            key = f"overlap{int(overlap)}_pair{int(pair)}"
            out[key] = {"result_class_per_run": reps, "distinct": len(classes),
                        "first_loss_diffs": [[round(a - b, 4) for a, b in zip(c[0], classes[0][0])]
                                             for c in classes[1:]]}
            print(key, json.dumps(out[key]), flush=True)
    print(json.dumps({k: v["result_class_per_run"] for k, v in out.items()}))


if __name__ == "__main__":
    main()
