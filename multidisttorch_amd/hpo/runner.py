"""Per-trial driver: one HPO trial trained by one group of ranks.

Parity map (/root/reference/vae-hpo.py):
  * ``run(group_id, batch_size, epochs, group)`` :122-174  -> ``run_trial``
  * ``train`` :61-92 / ``test`` :95-119                     -> ``_train_epoch`` / ``_test_epoch``
  * stdout formats (``[W:G] Train Epoch: ...``, ``====> Epoch: ...``,
    ``====> Test set loss: ...``, ``"{rank} Done. time: ..."``) are byte
    compatible; ``results-{group_rank}/reconstruction_{e}.png`` and
    ``sample_{e}.png`` keep the reference's layout (SURVEY.md Q7 collision
    included unless ``per_group_results``).
  * the DistributedSampler shard (``rank=group_id, num_replicas=W//group_size``)
    and its fixed epoch order (no ``set_epoch``) are reproduced exactly.

MI355X-first differences: the whole epoch runs as replays of a captured
hipGraph over device-resident data (no DataLoader, no per-step ``.item()``);
the loss history is read once per epoch to print the same log lines; global
barriers run on the gloo control plane so uneven trials never trip the RCCL
watchdog; replicas of a group (size > 1) all-reduce gradients through the
native bucket reducer, overlapped with the tail of the backward pass.
"""

from __future__ import annotations

import math
import os
import sys
import time
from dataclasses import dataclass, field
from typing import Optional

import torch
import torch.distributed as dist

from ..ckpt import checkpoint as ckpt
from ..data.sampler import reference_num_replicas, shard_indices
from ..obs.metrics import TrialMetrics
from ..obs import trace
from ..parallel.autotune import autotune_comm
from ..parallel.ddp import broadcast_params, make_arena_reducer
from ..parallel.groups import print0
from ..runtime.bootstrap import bound_device, global_barrier
from ..runtime.faults import (InjectedFault, TrialCorrupted, TrialTimeout, agree_healthy, fault_step, group_timeout_s, guarded,
                              heartbeat_s, maybe_inject, trial_watch)
from ..utils.images import flush_images, save_image_async
from .trial import TrialSpec

__all__ = ["RunOptions", "TrialResult", "run_trial", "run_packed_trials", "idle_rank"]


@dataclass
class RunOptions:
    batch_size: int = 128
    log_interval: int = 10
    model: str = "mlp"
    backend: Optional[str] = None          # hip | torch (default: hip on GPU)
    use_graphs: bool = True
    graph_steps: int = 10
    ckpt_dir: Optional[str] = None
    resume: bool = False
    metrics_dir: Optional[str] = None
    results: bool = True                   # write PNGs like the reference
    per_group_results: bool = False        # opt-in fix for the results-0 collision (Q7)
    eval_each_epoch: bool = True
    quiet_train_log: bool = False
    train_samples: Optional[int] = None    # synthetic dataset size (default 60000)
    test_samples: Optional[int] = None     # (default 10000)
    image_size: int = 28
    data_dir: str = "data"
    synthetic: Optional[bool] = None       # None: IDX files when present, else synthetic; True/False force
    bucket_mb: Optional[object] = None     # None: model default; 0: one bucket; float: MiB cap; "auto": measured
    profile: bool = False                  # roctx ranges + device-synced phase timings in the metrics JSONL


@dataclass
class TrialResult:
    group_id: int
    epochs: int
    shard: int
    samples: int
    wall_s: float
    final_train_loss: float = float("nan")
    final_test_loss: float = float("nan")
    failed: bool = False
    error: str = ""
    extra: dict = field(default_factory=dict)


def _results_dir(opts: RunOptions, group_id: int, group_rank: int) -> str:
    if opts.per_group_results:
        return f"results-g{group_id}-{group_rank}"
    return f"results-{group_rank}"


def _make_trainer(spec: TrialSpec, opts: RunOptions, device, group_rank: int, D: int):
    if opts.model == "mlp":
        from ..models.mlp_trainer import MlpVaeTrainer

        return MlpVaeTrainer(batch_size=opts.batch_size, D=D, device=device, backend=opts.backend,
                             seed=spec.seed, lr=spec.lr, kl_beta=spec.beta, rng_stream=group_rank,
                             use_graphs=opts.use_graphs, graph_steps=opts.graph_steps)
    if opts.model == "conv":
        from ..models.conv_vae import ConvVaeTrainer

        return ConvVaeTrainer(batch_size=opts.batch_size, image=opts.image_size,
                              z=32 if opts.image_size == 28 else 64, device=device, backend=opts.backend,
                              seed=spec.seed, lr=spec.lr, kl_beta=spec.beta, rng_stream=group_rank,
                              use_graphs=opts.use_graphs, graph_steps=opts.graph_steps)
    raise ValueError(f"unknown model {opts.model!r}")


def _load_data(opts: RunOptions, device):
    from ..data.datasets import mnist_like

    train = mnist_like(True, data_dir=opts.data_dir, device=device, size=opts.image_size,
                       synthetic=opts.synthetic, n=opts.train_samples)
    test = mnist_like(False, data_dir=opts.data_dir, device=device, size=opts.image_size,
                      synthetic=opts.synthetic, n=opts.test_samples)
    return train, test


LOSS_RING = 4096  # per-step loss history ring of the trainers (kLossHist, csrc/kernels/vae_mlp.h)


def _steps(trainer, n: int, B: int, events):
    """``train_steps(n)``; with an ``events`` list, in chunks of about 64 steps
    (a whole number of captured graphs) each followed by a recorded event, so
    a waiter can tell a slow epoch that is still completing steps from a stuck
    one."""
    if events is None:
        trainer.train_steps(n, B)
        return
    gs = max(1, int(getattr(trainer, "graph_steps", 1)))
    chunk = gs * max(1, 64 // gs)
    done = 0
    while done < n:
        k = min(chunk, n - done)
        trainer.train_steps(k, B)
        done += k
        ev = torch.cuda.Event()
        ev.record()
        events.append(ev)


def _launch_epoch(trainer, epoch: int, n_shard: int, opts: RunOptions, fault_at: Optional[int] = None,
                  events=None):
    """Enqueue one epoch of steps on the current stream; returns (step counter
    before the epoch, {batch_idx: loss} of log lines whose ring slots were read
    early). No host sync unless the epoch is longer than the loss ring: then
    the ring is read after every LOSS_RING steps, before it wraps (batch sizes
    below 15 on a 60000-sample shard). ``fault_at`` (MDT_FAULT step=) stops
    issuing steps at that optimizer step and raises, mid-epoch. ``events``
    (a list) receives progress events (see ``_steps``)."""
    B = opts.batch_size
    full, tail = n_shard // B, n_shard % B
    nb = full + (1 if tail else 0)
    trainer.set_cursor(0, nb)
    trainer.reset_loss()
    step0 = trainer.step_count
    early = {}
    stop = None if fault_at is None or not step0 <= fault_at < step0 + nb else fault_at - step0
    with trace.range(f"train_epoch_{epoch}"):
        c = 0
        while c < full:
            n = min(full - c, LOSS_RING) if nb > LOSS_RING else full - c
            if stop is not None and c + n > stop:
                _steps(trainer, stop - c, B, events)
                raise InjectedFault(f"injected fault at step {fault_at} (epoch {epoch})")
            _steps(trainer, n, B, events)
            if nb > LOSS_RING:
                hist = trainer.loss_history()
                assert len(hist) == LOSS_RING
                for bi in range(c - c % opts.log_interval, c + n, opts.log_interval):
                    if bi >= c:
                        early[bi] = float(hist[(step0 + bi) % LOSS_RING])
            c += n
        if tail:
            if stop is not None and stop == full:
                raise InjectedFault(f"injected fault at step {fault_at} (epoch {epoch})")
            _steps(trainer, 1, tail, events)
    return step0, early


def _abort(group, device, trainer=None):
    """Give up on the group's data plane: the trainer's xGMI reducer (its
    in-kernel waits see the host-mapped abort word, so the steps still queued
    drain at once instead of one MDT_P2P_TIMEOUT_S each) and the group's RCCL
    communicator (its kernels observe the abort flag and exit)."""
    red = getattr(trainer, "reducer", None)
    if red is not None and hasattr(red, "abort"):
        red.abort()
    try:
        be = group._get_backend(device)
        if hasattr(be, "abort"):
            be.abort()
    except Exception:  # noqa: BLE001 - best effort, we are failing anyway
        pass


def _drain(events, limit_s: float):
    """After an abort: wait (bounded) until the queued steps have left the
    stream, so the process can sync, checkpoint or exit. Seconds taken, or
    None if the stream is still busy after ``limit_s``."""
    t = time.monotonic()
    while events and not events[-1].query():
        if time.monotonic() - t > limit_s:
            return None
        time.sleep(0.001)
    return time.monotonic() - t


def _fail_epoch(trainer, group, device, events, msg):
    _abort(group, device, trainer)
    limit = float(os.getenv("MDT_ABORT_DRAIN_S", "30"))
    d = _drain(events, limit)
    trainer.drain_s = d
    tail = f"stream drained in {d:.2f} s" if d is not None else f"stream still busy after {limit:.0f} s"
    raise TrialTimeout(f"{msg} ({tail})")


def _wait_epoch(trainer, group, device, events, watch=None):
    """Wait for this replica's enqueued epoch (groups > 1 on GPU).

    The bucket collectives run inside replayed graphs, out of sight of
    ProcessGroupNCCL's watchdog: if a peer died mid-epoch they would never
    complete. So: poll the epoch's progress events; meanwhile beat on the
    trial's ``TrialWatch`` and check the peers (a published failure or a
    silent peer ends the wait within ~0.5 s / ``MDT_HEARTBEAT_S``); and if no
    chunk of steps completes for ``MDT_GROUP_TIMEOUT_S`` the epoch is stuck.
    Either way abort the group's data plane (``_abort``: the xGMI reducer's
    waits and the RCCL communicator give up), let the queued steps drain
    (bounded by ``MDT_ABORT_DRAIN_S``) and fail the trial."""
    if device.type != "cuda" or group is None or not dist.is_initialized() or dist.get_world_size(group) == 1:
        return
    ev = torch.cuda.Event()
    ev.record()
    events.append(ev)
    stall, hb = group_timeout_s(), heartbeat_s()
    now = time.monotonic()
    last_progress, next_beat, done = now, now, 0
    if watch is not None:
        watch.reset()
    while True:
        while done < len(events) and events[done].query():
            done += 1
            last_progress = time.monotonic()
        if done == len(events):
            break
        now = time.monotonic()
        if now - last_progress > stall:
            _fail_epoch(trainer, group, device, events, f"no step of the epoch completed for {stall:.0f} s (peer lost?)")
        if watch is not None and now >= next_beat:
            next_beat = now + 0.5
            try:
                watch.beat()
                msg = watch.check(hb)
            except Exception as e:  # noqa: BLE001 - the store (on world rank 0) is unreachable
                msg = f"control store unreachable: {type(e).__name__}: {e}"
            if msg:
                _fail_epoch(trainer, group, device, events, msg)
        time.sleep(0.0005)
    red = getattr(trainer, "reducer", None)
    if red is not None and hasattr(red, "status") and int(red.status()) != 0:
        raise TrialTimeout(f"p2p all-reduce gave up waiting for a peer (status {int(red.status())})")


def _check_health(trainer):
    """Fail the trial on a kernel-reported corruption (ConvVaeTrainer.health_error)."""
    fn = getattr(trainer, "health_error", None)
    msg = fn() if fn is not None else None
    if msg:
        raise TrialCorrupted(msg)


def _train_epoch(trainer, epoch: int, n_shard: int, n_dataset: int, opts: RunOptions, group,
                 step0: Optional[int] = None, tag: str = "", fault_at: Optional[int] = None, watch=None) -> float:
    B = opts.batch_size
    full, tail = n_shard // B, n_shard % B
    nb = full + (1 if tail else 0)
    early = {}
    if step0 is None:
        device = getattr(trainer, "device", torch.device("cpu"))
        multi = device.type == "cuda" and group is not None and dist.is_initialized() and \
            dist.get_world_size(group) > 1
        events = [] if multi else None
        step0, early = _launch_epoch(trainer, epoch, n_shard, opts, fault_at, events)
        _wait_epoch(trainer, group, device, events, watch)
    elif nb > LOSS_RING:
        raise ValueError(f"{nb} batches per epoch exceed the {LOSS_RING}-entry loss ring of a packed trial; "
                         f"use a larger --batch-size or --trials-per-group 1")
    _check_health(trainer)
    hist = trainer.loss_history()
    st = trainer.read_state()
    if not opts.quiet_train_log:
        for batch_idx in range(0, nb, opts.log_interval):
            bsz = B if batch_idx < full else tail
            loss_b = early.get(batch_idx)
            if loss_b is None:
                loss_b = float(hist[(step0 + batch_idx) % len(hist)])
            print0(tag + "Train Epoch: {} [{}/{} ({:.0f}%)]\tLoss: {:.6f}".format(
                epoch, batch_idx * bsz, n_dataset, 100.0 * batch_idx / nb, loss_b / bsz), process_group=group)
    # The reference divides by the FULL dataset size, not the shard (Q6).
    print0(tag + "====> Epoch: {} Average loss: {:.4f}".format(epoch, st["epoch_loss"] / n_dataset),
           process_group=group)
    return st["epoch_loss"]


def _test_epoch(trainer, epoch: int, test, opts: RunOptions, group, rdir: Optional[str], shape,
                tag: str = "") -> float:
    idx = torch.arange(len(test), dtype=torch.int32, device=test.data.device)
    with trace.range(f"test_epoch_{epoch}"):
        total, first = trainer.evaluate(test.data, idx, want_first_recon=rdir is not None)
    if rdir is not None and first is not None:
        m = first.shape[0]
        n = min(m, 8)
        data = test.data[:n].view(n, *shape).float().cpu()
        comparison = torch.cat([data, first[:n].view(n, *shape).float().cpu()])
        os.makedirs(rdir, exist_ok=True)
        save_image_async(comparison, f"{rdir}/reconstruction_" + str(epoch) + ".png", nrow=n)
    test_loss = total / len(test)
    print0(tag + "====> Test set loss: {:.4f}".format(test_loss), process_group=group)
    return test_loss


def run_trial(spec: TrialSpec, group, opts: RunOptions, data=None, num_trials: Optional[int] = None) -> TrialResult:
    """Train one trial on the ranks of ``group`` (this rank is a member)."""
    world_rank = dist.get_rank() if dist.is_initialized() else 0
    world_size = dist.get_world_size() if dist.is_initialized() else 1
    grank = dist.get_rank(group) if dist.is_initialized() else 0
    gsize = dist.get_world_size(group) if dist.is_initialized() else 1
    # sampler replicas exactly as the reference (vae-hpo.py:146): W // group size,
    # which differs from the trial count K when W % K != 0 (leftover idle ranks)
    n_rep = reference_num_replicas(world_size, gsize)
    device = bound_device()

    train, test = data if data is not None else _load_data(opts, device)
    if grank == 0:  # stderr: stdout stays byte-compatible with the reference
        print(f"[mdt] trial {spec.group_id}: train data {train.name} ({'synthetic' if train.synthetic else 'IDX'}, "
              f"{len(train)} x {tuple(train.shape)})", file=sys.stderr, flush=True)
    D = int(train.data.shape[1])
    trainer = _make_trainer(spec, opts, device, grank, D)
    if gsize > 1:
        # DDP's _sync_module_states: replicas start from group rank 0's weights
        broadcast_params([trainer.params], group)
        trainer.refresh_weights()
        if opts.bucket_mb == "auto":
            idx0 = shard_indices(len(train), n_rep, spec.group_id)
            key = f"{opts.model}-{opts.image_size}-b{opts.batch_size}-n{trainer.numel}-s{gsize}"
            bounds, kind, timings = autotune_comm(lambda: _make_trainer(spec, opts, device, grank, D), group,
                                                  train.data, idx0, key=key)
            print0(f"bucket autotune (group of {gsize}): {timings} -> {kind or 'default'} {bounds}",
                   process_group=group)
        else:
            bounds, kind = trainer.bucket_bounds(opts.bucket_mb), None
        trainer.attach_reducer(make_arena_reducer(group, trainer.grads, bounds, kind=kind,
                                                  comm_jobs=getattr(trainer, "comm_jobs", False)))
    start_epoch = 1
    if opts.ckpt_dir and opts.resume:
        # only group rank 0 writes checkpoints, so only it reads one; the
        # replicas receive weights, Adam moments, the step counter and the
        # epoch to resume from (no shared filesystem needed). Rank 0's load
        # outcome goes first, so a load error (arch mismatch, corrupt file)
        # raises on every member together instead of stranding the replicas
        # in the parameter broadcast.
        prog, err = None, None
        if grank == 0:
            try:
                prog = ckpt.load_latest(opts.ckpt_dir, spec.group_id, trainer)
            except Exception as e:  # noqa: BLE001 - re-raised below on every member
                err = e
        if prog is not None:
            start_epoch = prog["epoch"] + 1
            print0(f"resumed trial {spec.group_id} from {prog['path']} (epoch {prog['epoch']})", process_group=group)
        if gsize > 1:
            meta = torch.tensor([0 if err is None else 1, start_epoch, trainer.step_count], dtype=torch.int64,
                                device=device if dist.get_backend(group) == "nccl" else "cpu")
            broadcast_params([meta], group)
            if int(meta[0].item()) != 0:
                if err is not None:
                    raise err
                raise RuntimeError(f"trial {spec.group_id}: group rank 0 could not load its checkpoint; "
                                   f"stopping every member")
            broadcast_params([trainer.params, trainer.exp_avg, trainer.exp_avg_sq], group)
            start_epoch = int(meta[1].item())
            trainer.set_step(int(meta[2].item()))
            trainer.refresh_weights()
        elif err is not None:
            raise err
    metrics = TrialMetrics(opts.metrics_dir, spec.group_id, enabled=(grank == 0))

    idx = shard_indices(len(train), n_rep, spec.group_id)
    trainer.bind_train_data(train.data, idx)
    n_shard = idx.numel()
    # capture the step graphs and the test-set eval graphs and load the
    # decode kernels now, like the reference's model/DDP construction before
    # its timer starts (vae-hpo.py:159)
    trainer.prepare([opts.batch_size, n_shard % opts.batch_size], test.data if opts.eval_each_epoch else None)

    # Parity with the reference's download barrier (vae-hpo.py:133-144).
    global_barrier()
    rdir = _results_dir(opts, spec.group_id, grank) if opts.results else None
    shape = (1, opts.image_size, opts.image_size)
    gen = torch.Generator(device="cpu").manual_seed(spec.seed * 7919 + 17)

    t0 = time.time()
    train_loss = test_loss = float("nan")
    failure = {}
    epochs_done = 0

    watch = trial_watch(spec.group_id) if gsize > 1 else None

    def _fail(e):
        failure["error"] = f"{type(e).__name__}: {e}"
        metrics.log(event="trial_failed", error=failure["error"])
        if watch is not None:  # peers waiting on their epoch see it within ~0.5 s
            watch.fail(failure["error"])

    fault_at = fault_step(trial=spec.group_id, rank=world_rank)
    checked_in = False  # this member's "not ok" has been delivered to the group
    with guarded(f"trial {spec.group_id} (world rank {world_rank})", group, _fail):
        for epoch in range(start_epoch, spec.epochs + 1):
            # group members agree on health before every epoch (see faults.py)
            if not agree_healthy(spec.group_id, True):
                checked_in = True
                raise RuntimeError("a replica of this trial failed; stopping the trial on every member")
            maybe_inject(trial=spec.group_id, epoch=epoch, rank=world_rank)
            train_loss, test_loss = _run_epoch(trainer, epoch, n_shard, train, test, opts, group, rdir, shape,
                                               gen, device, spec, grank, metrics, fault_at=fault_at, watch=watch)
            epochs_done += 1
        if not agree_healthy(spec.group_id, True):
            checked_in = True
            raise RuntimeError("a replica of this trial failed in its last epoch")
    if failure and not checked_in:
        agree_healthy(spec.group_id, False)

    flush_images()
    global_barrier()  # parity: vae-hpo.py:172 (waits for the slowest trial)
    t1 = time.time()
    print(world_rank, "Done. time: %f" % (t1 - t0), flush=True)
    return TrialResult(spec.group_id, epochs_done, n_shard, epochs_done * n_shard, t1 - t0,
                       train_loss / len(train), test_loss, failed=bool(failure), error=failure.get("error", ""))


def _run_epoch(trainer, epoch, n_shard, train, test, opts, group, rdir, shape, gen, device, spec, grank, metrics,
               step0=None, t_train=None, tag="", fault_at=None, watch=None):
    te = time.perf_counter()
    train_loss = _train_epoch(trainer, epoch, n_shard, len(train), opts, group, step0=step0, tag=tag,
                              fault_at=fault_at, watch=watch)
    if t_train is None:
        t_train = time.perf_counter() - te
    phases = {}

    def _mark(name, t):
        if opts.profile and device.type == "cuda":
            torch.cuda.synchronize(device)
        phases[name] = round(time.perf_counter() - t, 6)
        return time.perf_counter()

    t = time.perf_counter()
    test_loss = float("nan")
    if opts.eval_each_epoch:
        test_loss = _test_epoch(trainer, epoch, test, opts, group, rdir, shape, tag=tag)
    t = _mark("eval_s", t)
    if rdir is not None:
        with torch.no_grad(), trace.range(f"sample_{epoch}"):
            sample = torch.randn(64, trainer.Z, generator=gen).to(device)
            sample = trainer.decode(sample).cpu()
            os.makedirs(rdir, exist_ok=True)
            save_image_async(sample.view(64, *shape), f"{rdir}/sample_" + str(epoch) + ".png")
    t = _mark("sample_s", t)
    if opts.ckpt_dir and grank == 0:
        with trace.range(f"ckpt_{epoch}"):
            ckpt.save_trial(opts.ckpt_dir, trainer, spec, epoch)
    _mark("ckpt_s", t)
    metrics.log(epoch=epoch, train_loss_sum=train_loss, train_loss=train_loss / len(train),
                test_loss=test_loss, epoch_train_s=t_train, samples=n_shard,
                train_samples_per_s=n_shard / max(t_train, 1e-9), lr=spec.lr, beta=spec.beta, **phases)
    return train_loss, test_loss


def run_packed_trials(specs, group, opts: RunOptions, data=None, num_trials: Optional[int] = None):
    """Train several trials concurrently on this rank's GPU (trial packing).

    MI355X-first extension (no reference counterpart): one small VAE step
    fills only part of the 256 CUs, so T trials of a size-1 group each get a
    HIP stream and their captured step graphs are replayed concurrently
    (measured 1.6-1.8x aggregate throughput at T = 2, profiles/r1_packing).
    Per epoch: every live trial's steps are enqueued on its stream, one
    device sync, then per-trial logging / eval / samples / checkpoints exactly
    as ``run_trial`` does (lines carry a ``(trial t)`` tag). Each trial is
    failure-isolated; uneven epoch counts are handled per trial.
    """
    world_rank = dist.get_rank() if dist.is_initialized() else 0
    world_size = dist.get_world_size() if dist.is_initialized() else 1
    gsize = dist.get_world_size(group) if dist.is_initialized() else 1
    if gsize != 1:
        raise ValueError("trial packing runs independent trials: it needs groups of one rank")
    total = num_trials if num_trials is not None else world_size * len(specs)
    device = bound_device()
    train, test = data if data is not None else _load_data(opts, device)
    D = int(train.data.shape[1])
    shape = (1, opts.image_size, opts.image_size)
    tr = []
    for spec in specs:
        trainer = _make_trainer(spec, opts, device, 0, D)
        if len(specs) > 1 and hasattr(trainer, "f28_pair"):
            # packed trials fill the chip already; the one-workgroup-per-sample
            # step keeps their numerics independent of how the trials interleave
            trainer.f28_pair = False
        start = 1
        if opts.ckpt_dir and opts.resume:
            prog = ckpt.load_latest(opts.ckpt_dir, spec.group_id, trainer)
            if prog is not None:
                start = prog["epoch"] + 1
        idx = shard_indices(len(train), total, spec.group_id)  # packing extension: one shard per trial
        trainer.bind_train_data(train.data, idx)
        trainer.prepare([opts.batch_size, idx.numel() % opts.batch_size], test.data if opts.eval_each_epoch else None)
        rdir = (f"results-t{spec.group_id}-0" if opts.results else None)
        tr.append(dict(spec=spec, trainer=trainer, start=start, n_shard=idx.numel(), rdir=rdir,
                       stream=torch.cuda.Stream(device) if device.type == "cuda" else None,
                       metrics=TrialMetrics(opts.metrics_dir, spec.group_id, enabled=True),
                       gen=torch.Generator(device="cpu").manual_seed(spec.seed * 7919 + 17),
                       done=0, train_loss=float("nan"), test_loss=float("nan"), failure={}))
    for t in tr:  # a packed epoch is enqueued whole: its losses must fit the ring (checked before any launch)
        nb = -(-t["n_shard"] // opts.batch_size)
        if nb > LOSS_RING:
            raise ValueError(f"{nb} batches per epoch exceed the {LOSS_RING}-entry loss ring of a packed trial; "
                             f"use a larger --batch-size or --trials-per-group 1")
    global_barrier()
    t0 = time.time()
    last = max(t["spec"].epochs for t in tr)
    for epoch in range(1, last + 1):
        live = [t for t in tr if t["start"] <= epoch <= t["spec"].epochs and not t["failure"]]
        te = time.perf_counter()
        for t in live:  # enqueue every trial's epoch on its own stream
            with guarded(f"trial {t['spec'].group_id} (world rank {world_rank})", None,
                         lambda e, t=t: t["failure"].setdefault("error", f"{type(e).__name__}: {e}")):
                maybe_inject(trial=t["spec"].group_id, epoch=epoch, rank=world_rank)
                if t["stream"] is not None:
                    with torch.cuda.stream(t["stream"]):
                        t["step0"], _ = _launch_epoch(t["trainer"], epoch, t["n_shard"], opts)
                else:
                    t["step0"], _ = _launch_epoch(t["trainer"], epoch, t["n_shard"], opts)
        if device.type == "cuda":
            torch.cuda.synchronize(device)
        t_train = time.perf_counter() - te
        for t in live:
            if t["failure"]:
                continue
            spec = t["spec"]
            with guarded(f"trial {spec.group_id} (world rank {world_rank})", None,
                         lambda e, t=t: t["failure"].setdefault("error", f"{type(e).__name__}: {e}")):
                t["train_loss"], t["test_loss"] = _run_epoch(
                    t["trainer"], epoch, t["n_shard"], train, test, opts, group, t["rdir"], shape, t["gen"], device,
                    spec, 0, t["metrics"], step0=t["step0"], t_train=t_train, tag=f"(trial {spec.group_id}) ")
                t["done"] += 1
    flush_images()
    global_barrier()
    t1 = time.time()
    print(world_rank, "Done. time: %f" % (t1 - t0), flush=True)
    return [TrialResult(t["spec"].group_id, t["done"], t["n_shard"], t["done"] * t["n_shard"], t1 - t0,
                        t["train_loss"] / len(train), t["test_loss"], failed=bool(t["failure"]),
                        error=t["failure"].get("error", "")) for t in tr]


def idle_rank():
    """Leftover ranks (W % K) own no trial but join both global barriers, so the
    members never block on them (fixes the reference's crash)."""
    global_barrier()
    t0 = time.time()
    global_barrier()
    return time.time() - t0
