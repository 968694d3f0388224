"""Diagnostic: does any buffer of the fused 28x28 step get read before it is
written, anywhere in the trainer (not only the buffers diag_garbage.py
knows by name)? Fills the CUDA caching allocator's free blocks with a
pattern (quiet NaN, then a large finite value) before the trainer is built,
so every torch.empty allocation of the trainer starts with that garbage,
and compares the trained result bitwise with a clean run, for the solo and
paired forms, eager and graph-replayed.

    python scripts/diag/diag_alloc_poison.py
"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))


def poison_allocator(value):
    """Allocate, fill and free blocks of many sizes (small and large pools)."""
    keep = []
    for nbytes in [4096, 65536, 262144, 1 << 20] * 64 + [4 << 20, 16 << 20, 64 << 20] * 8:
        t = torch.empty(nbytes // 4, dtype=torch.float32, device="cuda")
        t.fill_(value)
        keep.append(t)
    torch.cuda.synchronize()
    del keep  # blocks return to the caching allocator's free lists, contents intact


def main():
    from multidisttorch_amd.models.conv_vae import ConvVaeTrainer

    dev = torch.device("cuda", 0)
    nb, steps = 4, 8
    X = torch.rand(nb * 128, 784, generator=torch.Generator().manual_seed(3)).to(dev)
    idx = torch.arange(nb * 128, device=dev, dtype=torch.int32)

    def run(pair, graphs):
        tr = ConvVaeTrainer(batch_size=128, image=28, z=32, device=dev, backend="hip", seed=4, lr=2e-3,
                            use_graphs=graphs, graph_steps=4)
        tr.f28_pair = pair
        tr.bind_train_data(X, idx)
        tr.set_cursor(0, nb)
        tr.train_steps(steps)
        torch.cuda.synchronize()
        out = tr.loss_history()[:steps].tolist(), tr.params.clone()
        del tr
        torch.cuda.synchronize()
        return out

    res = {}
    for pair in (False, True):
        for graphs in (False, True):
            clean = run(pair, graphs)
            r = {}
            for name, val in (("nan", float("nan")), ("big", 8388608.0), ("neg", -3.0e38)):
                poison_allocator(val)
                h, p = run(pair, graphs)
                r[name] = {"bitwise": h == clean[0] and torch.equal(p, clean[1]),
                           "finite": bool(torch.isfinite(p).all().item())}
            key = f"pair{int(pair)}_graphs{int(graphs)}"
            res[key] = r
            print(key, json.dumps(r), flush=True)
    print(json.dumps({k: all(v["bitwise"] for v in r.values()) for k, r in res.items()}))


if __name__ == "__main__":
    main()
