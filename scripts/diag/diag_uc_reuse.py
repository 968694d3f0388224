"""Diagnostic: after a fused-reducer trainer with captured graphs has lived
and died, do later trainers' buffers land inside the address range of its
freed uncached (hipDeviceMallocUncached) reducer region, and which per-step
buffer of a reducer-free solo step first differs from a clean run?

    python scripts/diag/diag_uc_reuse.py
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
    nb = 4
    X = torch.rand(nb * 128, 784, generator=torch.Generator().manual_seed(3)).to(dev)
    idx = torch.arange(nb * 128, device=dev, dtype=torch.int32)

    def trainer(graphs=False, pair=False, fused=False):
        tr = ConvVaeTrainer(batch_size=128, image=28, z=32, device=dev, backend="hip", seed=4, lr=2e-3,
                            use_graphs=graphs, graph_steps=4)
        tr.f28_pair = pair
        tr.ddp_overlap = True
        red = None
        if fused:
            red = tr.C.XgmiP2PReducer(0, 1, tr.grads, tr.default_bucket_bounds(), True, 0.0, 64, 20.0, -1, True)
            tr.attach_reducer(red)
        tr.bind_train_data(X, idx)
        tr.set_cursor(0, nb)
        return tr, red

    def bufs(tr):
        p = tr._plan28(128)
        b = {"xb": tr.xb, "mulv": tr.mulv, "eps": tr.eps, "z16": tr.z16, "dlog32": tr.dlog32}
        b.update({"act." + k: v for k, v in tr.acts.items()})
        b.update({"gact." + k: v for k, v in tr.gacts.items()})
        b.update({"dmulv": tr.dmulv, "f28_bias": tr.f28_bias, "f28_part": tr.f28_part})
        b.update({"slab." + k: t for k, (t, _) in p["slabs"].items() if k.endswith(".weight")})
        b.update({"params": tr.params, "exp_avg": tr.exp_avg, "exp_avg_sq": tr.exp_avg_sq, "w16": tr.w16,
                  "w16t": tr.w16t, "state": tr.state.train_state})
        return b

    STEPS = 8

    def snapshots():
        """Per-step buffer snapshots of one fresh reducer-free solo trainer
        (device copies only: no host sync between the steps)."""
        tr, _ = trainer()
        out = []
        for _ in range(STEPS):
            tr.train_steps(1)
            out.append({k: v.clone() for k, v in bufs(tr).items()})
        torch.cuda.synchronize()
        addrs = {k: (v.data_ptr(), v.numel() * v.element_size()) for k, v in bufs(tr).items()}
        return out, addrs

    def first_diff(a, b):
        for s in range(STEPS):
            d = [k for k in a[s] if not torch.equal(a[s][k], b[s][k])]
            if d:
                return s, d
        return None, []

    clean, _ = snapshots()
    clean2, _ = snapshots()
    print("clean vs clean:", first_diff(clean, clean2), flush=True)

    tr, red = trainer(graphs=True, pair=True, fused=True)
    tr.train_steps(8)
    torch.cuda.synchronize()
    base, nbytes = red.local_base(), red.region_bytes()
    print(f"fused reducer region [{base:#x}, {base + nbytes:#x}) {nbytes / 1e6:.1f} MB", flush=True)
    del tr, red
    gc.collect()

    for r in range(4):
        snap, addrs = snapshots()
        s, diff = first_diff(clean, snap)
        inside = [k for k, (a, n) in addrs.items() if a < base + nbytes and a + n > base]
        print(json.dumps({"run": r, "first_differing_step": s, "differ": diff, "buffers_in_freed_uc_range": inside}),
              flush=True)


if __name__ == "__main__":
    main()
