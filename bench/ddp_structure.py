"""Structure cost of intra-group DDP on the fused 28x28 step, one MI355X.

The verdict's bar for configs #4/#5: with a reducer on a group of ONE rank
(collectives forced: RCCL PreMulSum scale 2 / the fused xGMI jobs, which
always run), the DDP step should cost <= 1.15x the reducer-free step, and the
encoder weight gradients must run while the decoder bucket's all-reduce is in
flight. Variants (20-step graphs, best of `--reps` replays, us per step):

  none          reducer-free step (f28_step_k | weight gradients | finalize+Adam)
  rccl_overlap  RCCL on its own stream, decoder bucket issued before the
                encoder weight gradients (two streams, event fences)
  rccl_inline   RCCL on the compute stream after the whole backward (no events)
  xgmi_overlap  fused all-reduce jobs (comm_jobs.h): decoder push inside the
                encoder weight-gradient launch, push+reduce+Adam tail
  xgmi_flat     fused jobs, no overlap: weight gradients | push+reduce+Adam

For xgmi_overlap it also records per-workgroup start/end stamps of the three
job launches and prints, per job, the span of its workgroups: the decoder push
and the encoder weight gradients share a launch and run at the same time.

    python bench/ddp_structure.py [--reps 7] [--json out.json]
"""
import argparse
import json
import os
import socket
import sys
import time

import torch
import torch.distributed as dist

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=7)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--json", default=None)
    ap.add_argument("--model", default="conv28", choices=["conv28", "conv128", "mlp"],
                    help="conv128: the layer-by-layer 128x128 step at B=64 (config #5 model); "
                         "mlp: the reference's MLP-VAE step at B=128 (fc4 bucket | rest)")
    ap.add_argument("--bucket-mb", type=float, default=None, help="RCCL bucket cap (default: decoder | encoder)")
    a = ap.parse_args()
    from multidisttorch_amd.models.conv_vae import ConvVaeTrainer
    from multidisttorch_amd.parallel.ddp import make_arena_reducer

    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ["MASTER_PORT"] = str(free_port())
    torch.cuda.set_device(0)
    dev = torch.device("cuda", 0)
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=dev)
    pg = dist.group.WORLD
    if a.model == "mlp":
        return mlp_variants(a, pg, dev)
    img = 28 if a.model == "conv28" else 128
    B, nb = (128, 16) if img == 28 else (64, 8)
    X = torch.rand(nb * B, img * img, generator=torch.Generator().manual_seed(3)).to(dev)
    idx = torch.arange(nb * B, device=dev, dtype=torch.int32)

    def make(kind, overlap=True):
        tr = ConvVaeTrainer(batch_size=B, image=img, z=32 if img == 28 else 64, device=dev, backend="hip", seed=4,
                            lr=2e-3, use_graphs=True, graph_steps=a.steps)
        tr.ddp_overlap = overlap
        bounds = tr.bucket_bounds(a.bucket_mb)
        if kind == "rccl":
            tr.attach_reducer(make_arena_reducer(pg, tr.grads, bounds, kind="rccl", scale=2.0))
            tr.set_hparams(grad_scale=0.5)
        elif kind == "xgmi":
            tr.attach_reducer(make_arena_reducer(pg, tr.grads, bounds, kind="xgmi"))
        tr.bind_train_data(X, idx)
        tr.set_cursor(0, nb)
        return tr

    def timeit(tr):
        tr.prepare([B])
        tr.strict_graphs = True
        tr.train_steps(a.steps)
        torch.cuda.synchronize()
        best = float("inf")
        for _ in range(a.reps):
            t0 = time.perf_counter()
            tr.train_steps(a.steps)
            torch.cuda.synchronize()
            best = min(best, (time.perf_counter() - t0) / a.steps)
        assert tr.health_error() is None, tr.health_error()
        return best * 1e6

    out = {"model": a.model, "batch": B}
    variants = (("none", None, True), ("rccl_overlap", "rccl", True), ("rccl_inline", "rccl", False),
                ("xgmi_overlap", "xgmi", True), ("xgmi_flat", "xgmi", False))
    if img == 128:  # layer path: RCCL buckets on their own stream as layers complete; fused pushes in the launches
        variants = (("none", None, True), ("rccl", "rccl", True), ("xgmi", "xgmi", True))
    for name, kind, ov in variants:
        tr = make(kind, ov)
        out[name] = round(timeit(tr), 2)
        print(f"{name:14s} {out[name]:8.2f} us/step  ratio {out[name] / out['none']:.3f}", flush=True)
        del tr
    out["ratio"] = {k: round(v / out["none"], 3) for k, v in out.items() if isinstance(v, float)}
    if img != 28:
        if a.json:
            with open(a.json, "w") as f:
                json.dump(out, f, indent=1)
        dist.destroy_process_group()
        return

    # in-launch overlap evidence: per-workgroup stamps of the fused-reducer step's job launches
    tr = make("xgmi", True)
    p = tr._plan28(B)
    sizes = [g for _, g in tr._comm_packs28(B, p)]
    tr._comm_packs.clear()
    tr.comm_stamps = [torch.zeros(2 * g, dtype=torch.int64, device=dev) for g in sizes]
    tr.use_graphs = False
    tr.train_steps(3)
    torch.cuda.synchronize()
    # job order = _comm_packs28's tables
    names = [["dec_fc wgrad", "dec1 wgrad", "dec2 wgrad", "loss/step"],
             ["enc1 wgrad", "enc2 wgrad", "enc_head wgrad", "decoder push (all-reduce)"],
             ["encoder push+reduce+Adam", "decoder reduce+Adam"]]
    packs = tr._comm_packs28(B, p)
    tables = tr._comm_tables[(B, True, True, False)]  # (M, Adam, overlap, split tail)
    lines, t_base = [], None
    stamps = [st.view(-1, 2).cpu().tolist() for st in tr.comm_stamps]
    t_base = min(x[0] for s in stamps for x in s)
    for li, (s, jobs) in enumerate(zip(stamps, tables)):
        b0 = 0
        for ji, j in enumerate(jobs):
            seg = s[b0:b0 + j.nblk]
            lines.append({"launch": li, "job": names[li][ji] if ji < len(names[li]) else str(ji),
                          "blocks": j.nblk, "start_us": round((min(x[0] for x in seg) - t_base) / 100.0, 2),
                          "end_us": round((max(x[1] for x in seg) - t_base) / 100.0, 2)})
            b0 += j.nblk
    assert len(packs) == len(stamps)
    out["xgmi_overlap_job_spans"] = lines
    for l in lines:
        print(f"  launch {l['launch']}  {l['job']:28s} {l['blocks']:5d} WGs  {l['start_us']:7.2f} .. {l['end_us']:7.2f} us")
    if a.json:
        with open(a.json, "w") as f:
            json.dump(out, f, indent=1)
    dist.destroy_process_group()


def mlp_variants(a, pg, dev):
    """MLP-VAE step with its two buckets (fc4 | rest): side-stream overlap vs
    everything inline on the compute stream, for RCCL and the p2p one-shot
    kernel (scale 2 + grad_scale 0.5 force the collective on one rank)."""
    from multidisttorch_amd.models.mlp_trainer import MlpVaeTrainer
    from multidisttorch_amd.parallel.ddp import make_arena_reducer

    B, nb = 128, 16
    X = torch.rand(nb * B, 784, generator=torch.Generator().manual_seed(3)).to(dev)
    idx = torch.arange(nb * B, device=dev, dtype=torch.int32)
    out = {"model": "mlp", "batch": B}
    for name, kind, ov in (("none", None, None), ("rccl_overlap", "rccl", True), ("rccl_inline", "rccl", False),
                           ("xgmi_overlap", "xgmi", True), ("xgmi_inline", "xgmi", False)):
        tr = MlpVaeTrainer(batch_size=B, device=dev, seed=4, lr=1e-3, use_graphs=True, graph_steps=a.steps)
        if kind is not None:
            tr.attach_reducer(make_arena_reducer(pg, tr.grads, tr.bucket_bounds(None), kind=kind, scale=2.0))
            tr.set_hparams(grad_scale=0.5)
            tr.ddp_overlap = ov
        tr.bind_train_data(X, idx)
        tr.set_cursor(0, nb)
        tr.prepare([B])
        tr.strict_graphs = True
        tr.train_steps(a.steps)
        torch.cuda.synchronize()
        best = float("inf")
        for _ in range(a.reps):
            t0 = time.perf_counter()
            tr.train_steps(a.steps)
            torch.cuda.synchronize()
            best = min(best, (time.perf_counter() - t0) / a.steps)
        out[name] = round(best * 1e6, 2)
        print(f"{name:14s} {out[name]:8.2f} us/step  ratio {out[name] / out['none']:.3f}", flush=True)
        del tr
    out["ratio"] = {k: round(v / out["none"], 3) for k, v in out.items() if isinstance(v, float)}
    if a.json:
        with open(a.json, "w") as f:
            json.dump(out, f, indent=1)
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
