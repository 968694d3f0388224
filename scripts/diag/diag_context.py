"""Diagnostic: which earlier activity in the process makes the reducer-free
28x28 step stop being run-to-run bitwise (test_fused_comm.py saw the solo
eager reference give a different result on every run in some phases)?

Stages, each followed by three solo eager reference runs compared with the
baseline result of stage 0:
  0 nothing before (baseline)
  1 a fused-reducer trainer, eager, run and deleted (gc)
  2 a fused-reducer trainer, graphs + overlap schedule, run and deleted
  3 a reducer-free trainer with graphs, run and deleted
  4 a fused reducer constructed, never launched, kept alive
  5 gc.collect() + torch.cuda.empty_cache()

    python scripts/diag/diag_context.py
"""
import gc
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

    def make(pair, graphs=False, fused=False, overlap=False):
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

    def ref():
        tr = make(False)
        tr.train_steps(steps)
        torch.cuda.synchronize()
        return tr.loss_history()[:steps].tolist(), tr.params.clone()

    base = ref()
    out = {}
    keep = []

    def check(stage):
        res = [ref() for _ in range(3)]
        eq = [h == base[0] and torch.equal(p, base[1]) for h, p in res]
        out[stage] = eq
        print(stage, eq, flush=True)

    check("0_nothing")
    t = make(True, fused=True)
    t.train_steps(steps)
    torch.cuda.synchronize()
    del t
    gc.collect()
    check("1_fused_eager")
    t = make(True, graphs=True, fused=True, overlap=True)
    t.train_steps(steps)
    torch.cuda.synchronize()
    del t
    gc.collect()
    check("2_fused_graphs_overlap")
    t = make(False, graphs=True)
    t.train_steps(steps)
    torch.cuda.synchronize()
    del t
    gc.collect()
    check("3_free_graphs")
    t = make(True)
    keep.append(t.C.XgmiP2PReducer(0, 1, t.grads, t.default_bucket_bounds(), True, 0.0, 64, 20.0, -1, True))
    check("4_reducer_alive")
    gc.collect()
    torch.cuda.empty_cache()
    check("5_gc_empty_cache")
    print(json.dumps(out))


if __name__ == "__main__":
    main()
