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

argv: image graphs(0|1) bucket_mb [reducer kind]  -> prints RESULT json
"""
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
    from multidisttorch_amd.runtime.env import apply_cu_split

    apply_cu_split()  # MDT_CU_SPLIT=1: disjoint CU shares per rank (before HIP initialises)
    dist.init_process_group("gloo")
    r, s = dist.get_rank(), dist.get_world_size()
    torch.cuda.set_device(0)
    dev = torch.device("cuda", 0)
    os.environ["MDT_P2P_TIMEOUT_S"] = "20"
    from multidisttorch_amd.models.conv_vae import ConvVaeTrainer
    from multidisttorch_amd.parallel.ddp import broadcast_params, make_arena_reducer

    B = 128 if image == 28 else 16
    z = 32 if image == 28 else 64
    nb = 4
    D = image * image
    X = torch.rand(nb * B, D, generator=torch.Generator().manual_seed(11)).to(dev)
    idx = torch.arange(nb * B, device=dev, dtype=torch.int32)
    steps = 8

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
        red = make_arena_reducer(dist.group.WORLD, tr.grads, tr.bucket_bounds(bucket_mb), kind=kind)
        tr.attach_reducer(red)
        if kind == "xgmi" and image == 28:
            # ranks share one GPU: a reduce spinning on a peer's push could hold the CUs that
            # peer needs, so push and reduce go in separate launches with a host barrier between
            # (eager steps; on a node every rank owns its GPU and the reduce waits in-kernel)
            tr.comm_split_tail = True
            tr.comm_phase_hook = lambda: (torch.cuda.synchronize(), dist.barrier())
        tr.bind_train_data(X, idx)
        tr.set_cursor(0, nb)
        same_each = []
        for _ in range(2):
            tr.train_steps(steps // 2)
            torch.cuda.synchronize()
            same_each.append(gather_same(tr.params.cpu()))
        hist = tr.loss_history()[:steps].astype(np.float64)
        res[phase] = dict(same=same_each, status=int(red.status()), nb=int(red.num_buckets()),
                          launched=int(red.launched_count()), loss=hist.tolist(),
                          finite=bool(torch.isfinite(tr.params).all().item()))
        if phase == "same_eps" and r == 0:
            ref = make(0)
            ref.bind_train_data(X, idx)
            ref.set_cursor(0, nb)
            ref.train_steps(steps)
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
