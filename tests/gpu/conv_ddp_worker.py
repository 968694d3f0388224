"""Worker for tests/gpu/test_conv_ddp.py: s processes share the box's single
MI355X and train the conv-VAE HIP path data-parallel through the one-shot
p2p bucket reducer (hipIpc regions exchanged over the gloo world) -- the
intra-group DDP of /root/reference/vae-hpo.py:129-131 on our fused step.

Phase 1 (same eps on every replica): the averaged gradient equals each
replica's own gradient, so every replica must match a reducer-free run of
the same trainer (rank 0 computes it afterwards) and all replicas must be
bitwise identical. Phase 2 (independent eps per replica, rng_stream = group
rank, as the reference's unseeded replicas): replicas still bitwise identical
after every step, while their per-replica losses differ.

argv: image graphs(0|1) bucket_mb [reducer kind] [mode] [tail]  -> prints RESULT json
  mode "split" (default for xgmi at 28x28 before round 5): push and reduce in
  separate eager launches with a host barrier between them; "prod": the
  production schedule exactly (graphs as given, the in-kernel wait, no split
  tail, no host barrier; run with MDT_CU_SPLIT=1 so ranks sharing the GPU
  never starve each other). tail > 0: every epoch ends with a partial batch of
  that many samples (full and tail steps alternate: different finalize-unit
  decompositions of the same arena).
"""
import hashlib
import json
import os
import sys

import numpy as np
import torch
import torch.distributed as dist

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))


def main():
    image, graphs = int(sys.argv[1]), sys.argv[2] == "1"
    bucket_mb = None if sys.argv[3] == "none" else float(sys.argv[3])
    kind = sys.argv[4] if len(sys.argv) > 4 else "p2p"
    mode = sys.argv[5] if len(sys.argv) > 5 else ("split" if kind == "xgmi" and image == 28 else "prod")
    tail = int(sys.argv[6]) if len(sys.argv) > 6 else 0
    from multidisttorch_amd.runtime.env import apply_cu_split

    apply_cu_split()  # MDT_CU_SPLIT=1: disjoint CU shares per rank (before HIP initialises)
    dist.init_process_group("gloo")
    r, s = dist.get_rank(), dist.get_world_size()
    torch.cuda.set_device(0)
    dev = torch.device("cuda", 0)
    os.environ["MDT_P2P_TIMEOUT_S"] = "20"
    from multidisttorch_amd.models.conv_vae import ConvVaeTrainer
    from multidisttorch_amd.parallel.ddp import SELFTEST_LOG, broadcast_params, make_arena_reducer

    B = 128 if image == 28 else 16
    z = 32 if image == 28 else 64
    nb = 4
    D = image * image
    n = nb * B + tail
    X = torch.rand(n, D, generator=torch.Generator().manual_seed(11)).to(dev)
    idx = torch.arange(n, device=dev, dtype=torch.int32)
    per_epoch = nb + (1 if tail else 0)
    steps = 2 * per_epoch

    def epoch(tr):
        tr.train_steps(nb)
        if tail:
            tr.train_steps(1, M=tail)

    def make(stream):
        return ConvVaeTrainer(batch_size=B, image=image, z=z, device=dev, backend="hip", seed=7, lr=2e-3,
                              rng_stream=stream, use_graphs=graphs, graph_steps=4)

    def gather_same(t):
        out = [torch.empty_like(t) for _ in range(s)]
        dist.all_gather(out, t)
        return all(torch.equal(out[0], o) for o in out)

    res = {"rank": r}
    for phase, stream in (("same_eps", 0), ("indep_eps", r)):
        tr = make(stream)
        broadcast_params([tr.params], dist.group.WORLD)  # DDP ctor broadcast (gloo: via host copy)
        tr.refresh_weights()
        n_log = len(SELFTEST_LOG)
        red = make_arena_reducer(dist.group.WORLD, tr.grads, tr.bucket_bounds(bucket_mb), kind=kind)
        selftest = SELFTEST_LOG[-1] if len(SELFTEST_LOG) > n_log else None
        tr.attach_reducer(red)
        if kind == "xgmi" and image == 28 and mode == "split":
            # push and reduce in separate launches with a host barrier between
            # (eager steps): the pre-CU-split rehearsal form, kept as a variant
            tr.comm_split_tail = True
            tr.comm_phase_hook = lambda: (torch.cuda.synchronize(), dist.barrier())
        assert mode == "split" or not tr.comm_split_tail
        tr.bind_train_data(X, idx)
        tr.set_cursor(0, per_epoch)
        same_each = []
        for _ in range(2):
            epoch(tr)
            torch.cuda.synchronize()
            same_each.append(gather_same(tr.params.cpu()))
        hist = tr.loss_history()[:steps].astype(np.float64)
        res[phase] = dict(reducer=type(red).__name__, same=same_each,
                          phash=hashlib.sha1(tr.params.cpu().numpy().tobytes()).hexdigest(),
                          two_shot=bool(red.fused_two_shot()) if hasattr(red, "fused_two_shot") else None, split=bool(tr.comm_split_tail), pair=bool(getattr(tr, "f28_pair", False)),
                          cu_mask=os.environ.get("HSA_CU_MASK"), status=int(red.status()) if hasattr(red, "status") else 0, nb=int(red.num_buckets()),
                          launched=int(red.launched_count()), loss=hist.tolist(), selftest=selftest,
                          finite=bool(torch.isfinite(tr.params).all().item()))
        if phase == "same_eps" and r == 0:
            ref = make(0)
            ref.bind_train_data(X, idx)
            ref.set_cursor(0, per_epoch)
            epoch(ref)
            epoch(ref)
            torch.cuda.synchronize()
            d = (tr.params - ref.params).abs().max().item()
            scale = ref.params.abs().max().item()
            res["single"] = dict(max_param_diff=d, param_scale=scale,
                                 loss=ref.loss_history()[:steps].astype(np.float64).tolist())
        dist.barrier()  # peers stop writing into our region before it is freed
        tr.attach_reducer(None)  # also drops the graphs that reference the peer regions
        del red, tr
        torch.cuda.synchronize()
        dist.barrier()
    print("RESULT " + json.dumps(res), flush=True)
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
