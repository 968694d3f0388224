#!/usr/bin/env python3
"""Headline benchmark: aggregate VAE samples/s across K concurrent HPO trials.

Metric / config from BASELINE.json: the global world (one process per MI355X)
is carved into K trial groups (default K = N: one trial per GPU, BASELINE
config #3 shape "8 subgroups x 1 GPU"; at N = 1 this is config #2 "1 subgroup
of 1 MI355X; conv-VAE bf16 on 28x28"). ``--ngroups`` gives e.g. 4x2 with
intra-group gradient all-reduce (config #4). Every trial trains the conv-VAE
(bf16 MFMA kernels, fp32 master weights + Adam) at batch 128 on its
DistributedSampler shard of a synthetic MNIST-shaped dataset, with its own
(lr, beta) hyper-parameters. ``--model mlp`` runs the reference's own MLP-VAE
(784-400-20, /root/reference/vae-hpo.py:19-45, fp32); ``--model conv128`` the
128x128 conv-VAE of config #5.

A step = one full training iteration (fwd + bwd + [all-reduce] + Adam) of every
trial. Timing: ``prepare`` captures the step hipGraphs (S = --graph-steps and the
S = 1 remainder graph) before anything is timed and the trainers are then
locked (``strict_graphs``: a missing graph raises rather than being captured
inside the timer); W warm-up replays, then a barrier +
device sync, exactly K steps, barrier + device sync; the max over ranks is
reported. ``value`` = sum over trials of (batch x steps) / max_time (samples are
counted once per trial, not per replica -- SURVEY.md section 6 metric).

Run: python bench.py --gpus N --steps K --warmup W   (N>1 via torch.distributed.run)
"""

from __future__ import annotations

import argparse
import json
import os
import sys
import time

import torch
import torch.distributed as dist

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

# Reference-equivalent throughput on the SAME MI355X: the
# reference's training loop (DDP + DataLoader + loss.item() per step + torch
# Adam, bench/ref_torch_baseline.py) in stock PyTorch-ROCm eager mode, per
# trial, for each model. The conv anchors run the reference loop with the
# conv-VAE swapped in, in fp32 (the reference's dtype; torch's bf16 autocast
# path faulted inside MIOpen on this stack for the 28x28 model).
# baseline(K) = K x anchor (generous to the reference: perfect scaling).
REF_SAMPLES_PER_S_PER_TRIAL = {"mlp": 93465.0, "conv28": 42924.0, "conv128": 18788.0}


def _timing_barrier(world, dev):
    """Barrier that brackets the timed steps. With one GPU per local rank on an
    RCCL world it is a one-element all-reduce over xGMI (tens of microseconds),
    so the bracket does not add the ~1 ms of a gloo TCP barrier across 8 ranks
    (measured on loopback) to a 25 ms timed window; otherwise (CPU, or ranks
    sharing a GPU, which RCCL rejects) the gloo control-plane barrier."""
    from multidisttorch_amd.runtime import global_barrier

    if world == 1:
        return (lambda: None), "none"
    local_n = int(os.environ.get("LOCAL_WORLD_SIZE", world))
    if dev.type == "cuda" and dist.get_backend() == "nccl" and torch.cuda.device_count() >= local_n:
        flag = torch.ones(1, device=dev)

        def bar():
            dist.all_reduce(flag)

        return bar, "rccl"
    return global_barrier, "gloo"


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--batch-size", type=int, default=128)
    ap.add_argument("--ngroups", type=int, default=None, help="trials K (default: world size)")
    ap.add_argument("--model", default="conv28", choices=["mlp", "conv28", "conv128"],
                    help="conv28 = conv-VAE bf16 28x28 (BASELINE configs #2/#3, headline); conv128 = 128x128 "
                         "(config #5); mlp = the reference's MLP-VAE in fp32")
    ap.add_argument("--graph-steps", type=int, default=20,
                    help="steps per captured hipGraph (one replay covers the driver's 20-step window)")
    ap.add_argument("--no-graphs", action="store_true")
    ap.add_argument("--backend", default=None, help="hip|torch (default: hip on GPU)")
    ap.add_argument("--json-out", default=None)
    ap.add_argument("--bucket-mb", default=None, help="intra-group buckets: MiB cap, 0 = one bucket")
    ap.add_argument("--trials-per-gpu", type=int, default=1,
                    help="trial packing: T concurrent trials per single-rank group (one HIP stream each); "
                         "the headline config is T=1 (K = N trials)")
    a = ap.parse_args(argv)

    from multidisttorch_amd.runtime.env import apply_cu_split

    apply_cu_split()  # one-GPU multi-rank rehearsals only (MDT_CU_SPLIT=1), before HIP initialises
    from multidisttorch_amd.runtime import setup_ddp, global_barrier, control_group
    from multidisttorch_amd.parallel.groups import setup_ddp_groups
    from multidisttorch_amd.hpo.trial import default_sweep
    from multidisttorch_amd.data.datasets import mnist_like
    from multidisttorch_amd.data.sampler import shard_indices
    from multidisttorch_amd.models.mlp_trainer import MlpVaeTrainer
    from multidisttorch_amd.parallel.ddp import SELFTEST_LOG, make_arena_reducer

    from multidisttorch_amd.runtime.bootstrap import _stdout_to_stderr

    # One trial per rank (the headline K = N layout): the trial groups never
    # communicate, so the device-bound world with one eager ncclCommSplit per
    # group (the HPO runner's default, runtime/bootstrap.py) buys nothing here;
    # the bench keeps the plain lazy RCCL world, whose single communicator the
    # first timing barrier opens outside the timed region. An explicit
    # MDT_EAGER_COMM still wins.
    world_env = int(os.environ.get("WORLD_SIZE", "1"))
    if (a.ngroups is None or a.ngroups >= world_env) and "MDT_EAGER_COMM" not in os.environ:
        os.environ["MDT_EAGER_COMM"] = "0"
    with _stdout_to_stderr():  # keep stdout for the single JSON line (gloo prints connect banners)
        world, rank = setup_ddp(verbose=False)
        K = a.ngroups or world
        handles = setup_ddp_groups(K, verbose=False)
        ctrl = control_group()
    dev = torch.device("cuda", torch.cuda.current_device()) if torch.cuda.is_available() else torch.device("cpu")
    if dev.type == "cpu":
        # CPU ranks (config #1): split the host's cores between the ranks of this
        # node instead of every rank spinning up one thread per core
        local_n = int(os.environ.get("LOCAL_WORLD_SIZE", world))
        torch.set_num_threads(max(1, (os.cpu_count() or 1) // max(1, local_n)))
    n_per = world // K
    gid = rank // n_per if rank < K * n_per else None


    T = max(1, a.trials_per_gpu)
    if T > 1 and n_per != 1:
        raise SystemExit("--trials-per-gpu > 1 needs single-rank groups (no intra-group all-reduce)")
    specs = default_sweep(K * T)

    def make_trainer(spec, grank):
        if a.model == "mlp":
            return MlpVaeTrainer(batch_size=a.batch_size, device=dev, backend=a.backend,
                                 seed=spec.seed, lr=spec.lr, kl_beta=spec.beta, rng_stream=grank,
                                 use_graphs=not a.no_graphs, graph_steps=a.graph_steps)
        from multidisttorch_amd.models.conv_vae import ConvVaeTrainer

        im = 28 if a.model == "conv28" else 128
        tr = ConvVaeTrainer(batch_size=a.batch_size, image=im, z=32 if im == 28 else 64, device=dev,
                            backend=a.backend, seed=spec.seed, lr=spec.lr, kl_beta=spec.beta,
                            rng_stream=grank, use_graphs=not a.no_graphs, graph_steps=a.graph_steps)
        if T > 1:  # packed trials already fill the chip: one workgroup per sample (deterministic form)
            tr.f28_pair = False
        return tr

    trainers, streams = [], []
    selftest = None
    img = 28 if a.model in ("mlp", "conv28") else 128
    if gid is not None:
        pg = handles[gid]
        grank = dist.get_rank(pg)
        train = mnist_like(True, synthetic=True, device=dev, size=img,
                           n=None if img == 28 else 4096 * max(1, a.batch_size // 32))
        for t in range(T):
            tid = gid * T + t
            trainer = make_trainer(specs[tid], grank)
            # replicas of a group start from group rank 0's weights (DDP broadcast)
            if n_per > 1:
                dist.broadcast(trainer.params, src=dist.get_global_rank(pg, 0), group=pg)
                trainer.refresh_weights()
                mb = None if a.bucket_mb in (None, "") else float(a.bucket_mb)
                n_log = len(SELFTEST_LOG)
                trainer.attach_reducer(make_arena_reducer(pg, trainer.grads, trainer.bucket_bounds(mb),
                                                          comm_jobs=getattr(trainer, "comm_jobs", False)))
                if len(SELFTEST_LOG) > n_log:  # the fused xGMI data plane's construction-time self-test
                    st = SELFTEST_LOG[-1]
                    selftest = {"result": st["result"], "ms": st["ms"], "two_shot": st["two_shot"],
                                "form": st.get("form"), "marks_ms": st.get("marks_ms")}
            # reference sampler replicas W // group size (vae-hpo.py:146); packing: one shard per trial
            idx = shard_indices(len(train), (world // n_per) * T, tid)
            trainer.bind_train_data(train.data, idx)
            trainer.set_cursor(0, idx.numel() // a.batch_size)  # full batches only
            # capture every step graph the timed loop replays (S = graph_steps and
            # the S = 1 remainder) BEFORE warm-up; afterwards a missing graph is
            # an error, never a capture inside the timed region
            trainer.prepare([a.batch_size])
            trainer.strict_graphs = trainer.use_graphs
            s = torch.cuda.Stream(dev) if (T > 1 and dev.type == "cuda") else None
            if s is not None:
                with torch.cuda.stream(s):
                    trainer.train_steps(a.warmup)
            else:
                trainer.train_steps(a.warmup)
            trainers.append(trainer)
            streams.append(s)
    trainer = trainers[0] if trainers else None

    def run_all(n):
        for tr, s in zip(trainers, streams):
            if s is not None:
                with torch.cuda.stream(s):
                    tr.train_steps(n)
            else:
                tr.train_steps(n)

    if dev.type == "cuda":
        torch.cuda.synchronize()
    global_barrier()  # coarse: every rank has finished set-up and warm-up
    tbar, tbar_kind = _timing_barrier(world, dev)
    tbar()  # opens the RCCL world communicator (lazy init) outside the timer
    if dev.type == "cuda":
        torch.cuda.synchronize()
    tbar()
    if dev.type == "cuda":
        torch.cuda.synchronize()
    t0 = time.perf_counter()
    run_all(a.steps)
    if dev.type == "cuda":
        torch.cuda.synchronize()
    tbar()
    if dev.type == "cuda":
        torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([dt], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX, group=ctrl)
        dt = float(t.item())
    samples = K * T * a.batch_size * a.steps
    value = samples / dt
    # sanity: training actually progressed and the loss is finite
    ok = True
    health = []
    for tr in trainers:
        st = tr.read_state()
        hist = tr.loss_history()
        last = float(hist[(st["step"] - 1) % len(hist)])
        ok = ok and st["step"] == a.warmup + a.steps and last == last and last < 1e9
        # in-kernel failures that do not show up in the loss: a paired-workgroup
        # exchange or an xGMI all-reduce wait that timed out (health_error)
        msg = tr.health_error() if hasattr(tr, "health_error") else None
        if msg:
            health.append(msg)
            ok = False
    # intra-group data parallelism: every replica of a trial must hold bitwise the
    # same parameters after the timed steps (the averaged gradient is identical on
    # every member; tests/gpu/conv_ddp_worker.py asserts the same)
    replicas_equal = None
    if n_per > 1 and gid is not None:
        replicas_equal = True
        pg = handles[gid]
        on_dev = dist.get_backend(pg) == "nccl"
        for tr in trainers:
            p = tr.params.detach().clone() if on_dev else tr.params.detach().cpu()
            got = [torch.empty_like(p) for _ in range(n_per)]
            dist.all_gather(got, p, group=pg)
            replicas_equal = replicas_equal and all(torch.equal(got[0], g) for g in got)
        ok = ok and replicas_equal
    flag = torch.tensor([1.0 if ok else 0.0])
    if world > 1:
        dist.all_reduce(flag, op=dist.ReduceOp.MIN, group=ctrl)
    if rank == 0:
        out = {
            "metric": "aggregate VAE samples/sec across K concurrent HPO trials",
            "value": round(value, 1),
            "unit": "samples/s",
            "n_gpus": world,
            "steps": a.steps,
            "warmup": a.warmup,
            "ms_per_step": round(dt / a.steps * 1e3, 4),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": round(value / (REF_SAMPLES_PER_S_PER_TRIAL[a.model] * K * T), 2),
            "dtype": "fp32" if a.model == "mlp" else "bf16",
            "data": ("synthetic (MNIST-shaped 60000x1x28x28, random-init weights)" if a.model != "conv128"
                     else "synthetic (1x128x128 images, random-init weights)"),
            "config": {
                "model": {"mlp": "MLP-VAE 784-400-20 (reference vae-hpo.py topology)",
                          "conv28": "conv-VAE 28x28 (2 conv + 2 deconv, z=32)",
                          "conv128": "conv-VAE 128x128 (4 conv + 4 deconv, z=64)"}[a.model],
                "global_batch": a.batch_size * K * T,
                "per_trial_batch": a.batch_size,
                "seq_len": None,
                "image": img,
                "parallelism": f"groups{K}x{n_per}" + (f"+pack{T}" if T > 1 else ""),
                "trials": K * T,
                "backend": trainer.backend if trainer is not None else None,
                "graphs": (not a.no_graphs),
                "timing_barrier": tbar_kind,
                "valid": bool(flag.item() > 0),
                "health": health or None,
                "replicas_bitwise_equal": replicas_equal,
                "reducer_selftest": selftest,
                "reducer": (type(trainer.reducer).__name__ if trainer is not None
                            and getattr(trainer, "reducer", None) is not None else None),
                # vs_baseline: the reference publishes no numbers (BASELINE.json
                # "published": {}); the divisor is a builder-measured anchor
                "baseline": ("NOT a published baseline: builder-measured reference-equivalent torch-eager "
                             f"loop on one MI355X ({'fp32' if a.model != 'conv128' else 'bf16 autocast'}), "
                             f"{REF_SAMPLES_PER_S_PER_TRIAL[a.model]:.0f} samples/s per trial x trials"),
            },
        }
        line = json.dumps(out)
        print(line, flush=True)
        if a.json_out:
            with open(a.json_out, "w") as f:
                f.write(line + "\n")
    if dist.is_initialized():
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
