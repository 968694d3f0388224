"""Multi-process test worker (launched by tests via multidisttorch_amd.launch).

Each mode prints one line ``RESULT <json>`` per rank that the test parses.
"""
import json
import faulthandler
faulthandler.enable()
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402


def _finish():
    """Control-plane barrier, then process-group teardown: no rank exits while
    a peer still talks to it (the reference's example-subgroup.py exits
    without teardown; that raced gloo's threads at exit)."""
    from multidisttorch_amd.runtime.bootstrap import global_barrier, shutdown

    global_barrier()
    shutdown()


def out(**kw):
    print("RESULT " + json.dumps(kw), flush=True)


def mode_groups(k):
    from utils import setup_ddp, setup_ddp_groups, print0
    from multidisttorch_amd.runtime.bootstrap import control_group, global_barrier

    ws, wr = setup_ddp()
    groups = setup_ddp_groups(k)
    control_group()
    member = [g for g, pg in enumerate(groups) if dist.get_rank(pg) >= 0]
    grank = [dist.get_rank(pg) for pg in groups]
    gathered = None
    for g in member:
        t = torch.tensor([wr])
        lst = [torch.zeros_like(t) for _ in range(dist.get_world_size(groups[g]))]
        dist.all_gather(lst, t, group=groups[g])
        gathered = [int(x) for x in lst]
        print0("hello from group", g, process_group=groups[g])
    global_barrier()
    out(world=ws, rank=wr, member=member, grank=grank, gathered=gathered)
    _finish()


def mode_reducer():
    from multidisttorch_amd.runtime.bootstrap import setup_ddp
    from multidisttorch_amd.parallel.ddp import make_arena_reducer, PyBucketReducer

    ws, wr = setup_ddp(verbose=False)
    pg = dist.new_group(list(range(ws)))
    res = {}
    for native in (True, False):
        flat = torch.arange(1000, dtype=torch.float32) * (wr + 1)
        red = make_arena_reducer(pg, flat, [0, 300, 1000], average=True, prefer_native=native)
        red.launch(1)
        red.launch(0)
        red.wait_all()
        expect = torch.arange(1000, dtype=torch.float32) * (sum(range(1, ws + 1)) / ws)
        res["native" if native else "py"] = float((flat - expect).abs().max())
        res["type_" + ("native" if native else "py")] = type(red).__name__
        # readiness mode
        flat2 = torch.ones(128) * (wr + 1)
        red2 = make_arena_reducer(pg, flat2, [0, 64, 128], average=False, prefer_native=native)
        red2.set_param_map([0, 0, 1])
        red2.mark_ready(2)
        red2.mark_ready(0)
        red2.mark_ready(1)
        red2.wait_all()
        res["ready_" + ("native" if native else "py")] = float(flat2[0]), float(flat2[100])
    out(rank=wr, **res)
    _finish()


def mode_disagree(what):
    """Members build reducers that do not agree (rank 1's arena one element
    larger, other bucket bounds, or another reducer kind): EVERY member must
    raise before any gradient moves, naming the differing rank."""
    from multidisttorch_amd.runtime.bootstrap import setup_ddp
    from multidisttorch_amd.parallel.ddp import make_arena_reducer

    ws, wr = setup_ddp(verbose=False)
    pg = dist.new_group(list(range(ws)))
    n = 1000 + (1 if what == "numel" and wr == 1 else 0)
    bounds = [0, 300 if what == "bounds" and wr == 1 else 200, n]
    kind = "python" if what == "kind" and wr == 1 else "c10d"
    err = None
    try:
        make_arena_reducer(pg, torch.zeros(n), bounds, kind=kind)
    except RuntimeError as e:
        err = str(e)
    # the agreement check itself keeps the group usable: one more collective works
    t = torch.ones(1)
    dist.all_reduce(t, group=pg)
    out(rank=wr, err=err, after=float(t.item()))
    _finish()


def mode_arena_ddp():
    """ArenaDDP grads == torch DDP grads on the same model/data (gloo, fp32)."""
    from multidisttorch_amd.runtime.bootstrap import setup_ddp
    from multidisttorch_amd.parallel.ddp import ArenaDDP
    from multidisttorch_amd.models.mlp_vae import VAE, loss_function

    ws, wr = setup_ddp(verbose=False)
    torch.manual_seed(0)
    base = VAE(D=64, H=32, Z=4)
    m1 = VAE(D=64, H=32, Z=4)
    m2 = VAE(D=64, H=32, Z=4)
    m1.load_state_dict(base.state_dict())
    m2.load_state_dict(base.state_dict())
    ddp_ref = torch.nn.parallel.DistributedDataParallel(m1)
    ours = ArenaDDP(m2, None, bucket_cap_mb=0.002, first_bucket_mb=0.001)
    g = torch.Generator().manual_seed(100 + wr)
    x = torch.rand(16, 64, generator=g)
    eps = torch.randn(16, 4, generator=g)
    for model, fin in ((ddp_ref, None), (ours, ours.finish_gradient_sync)):
        r, mu, lv = model(x, eps=eps)
        loss = loss_function(r, x, mu, lv)
        loss.backward()
        if fin:
            fin()
    err = max(float((p1.grad - p2.grad).abs().max()) for p1, p2 in zip(m1.parameters(), m2.parameters()))
    nb = len(ours.bucket_bounds) - 1
    out(rank=wr, err=err, buckets=nb)
    _finish()


def mode_trainer_ddp():
    """Two replicas of one trial (group of 2) stay bit-identical and match a
    single process training on the same data with averaged gradients."""
    from multidisttorch_amd.runtime.bootstrap import setup_ddp
    from multidisttorch_amd.parallel.ddp import make_arena_reducer, broadcast_params
    from multidisttorch_amd.models.mlp_trainer import MlpVaeTrainer

    ws, wr = setup_ddp(verbose=False)
    pg = dist.new_group(list(range(ws)))
    tr = MlpVaeTrainer(batch_size=32, D=64, H=32, Z=4, backend="torch", seed=3 + wr, rng_stream=wr)
    broadcast_params([tr.params], pg)
    tr.attach_reducer(make_arena_reducer(pg, tr.grads, [0, tr.split, tr.numel]))
    X = torch.rand(256, 64, generator=torch.Generator().manual_seed(9))
    idx = torch.arange(256, dtype=torch.int32)
    tr.bind_train_data(X, idx)
    tr.set_cursor(0, 8)
    tr.train_steps(5)
    p = tr.params.clone()
    allp = [torch.zeros_like(p) for _ in range(ws)]
    dist.all_gather(allp, p)
    out(rank=wr, maxdiff=float(max((a - allp[0]).abs().max() for a in allp)), step=tr.step_count)
    _finish()


def mode_autotune():
    """Bucket autotune over a group of 2 (gloo, CPU): both members must pick
    the same layout; conv-VAE replicas with per-layer buckets stay in sync."""
    from multidisttorch_amd.runtime.bootstrap import setup_ddp
    from multidisttorch_amd.parallel.autotune import autotune_buckets
    from multidisttorch_amd.parallel.ddp import make_arena_reducer, broadcast_params
    from multidisttorch_amd.models.conv_vae import ConvVaeTrainer

    ws, wr = setup_ddp(verbose=False)
    pg = dist.new_group(list(range(ws)))
    X = torch.rand(64, 784, generator=torch.Generator().manual_seed(4))
    idx = torch.arange(64, dtype=torch.int32)
    make = lambda: ConvVaeTrainer(batch_size=16, image=28, backend="torch", seed=1, rng_stream=wr)
    cache = os.environ["MDT_BUCKET_CACHE"]
    best, timings = autotune_buckets(make, pg, X, idx, candidates=(None, 0, 0.05), steps=2, warmup=1,
                                     key="test-key", cache=cache)
    tr = make()
    broadcast_params([tr.params], pg)
    tr.refresh_weights()
    tr.attach_reducer(make_arena_reducer(pg, tr.grads, best))
    tr.bind_train_data(X, idx)
    tr.set_cursor(0, 4)
    tr.train_steps(3)
    p = tr.params.clone()
    allp = [torch.zeros_like(p) for _ in range(ws)]
    dist.all_gather(allp, p)
    out(rank=wr, best=best, n=len(timings), maxdiff=float(max((a - allp[0]).abs().max() for a in allp)),
        cached=os.path.exists(cache))
    _finish()


def mode_health(k):
    """Health groups + trial watch on W ranks, K groups (leftover ranks idle):
    built without any further ``dist.new_group`` (patched to raise), agreement
    over each trial, a published failure and a silent peer are detected."""
    import time

    from multidisttorch_amd.runtime import faults
    from multidisttorch_amd.runtime.bootstrap import global_barrier, setup_ddp
    from multidisttorch_amd.parallel.groups import GroupPlan, setup_ddp_groups

    ws, wr = setup_ddp(verbose=False)
    setup_ddp_groups(k, verbose=False)
    global_barrier()

    def _no_new_group(*a, **kw):
        raise AssertionError("create_health_groups must not call dist.new_group")

    real = dist.new_group
    dist.new_group = _no_new_group
    try:
        faults.create_health_groups(k)
    finally:
        dist.new_group = real
    plan = GroupPlan(ws, k)
    g = plan.group_of(wr)
    res = dict(rank=wr, group=g, has_pg=faults.health_group(g) is not None if g is not None else False)
    if g is not None and plan.ranks_per_group > 1:
        grank = wr - plan.ranks(g)[0]
        res["agree_all_ok"] = faults.agree_healthy(g, True)
        res["agree_one_bad"] = faults.agree_healthy(g, grank != 1)
        w = faults.trial_watch(g)
        w.reset()
        if grank == 0:
            # peers beat for 1 s, then rank 1 publishes a failure
            t0 = time.monotonic()
            msg = None
            while msg is None and time.monotonic() - t0 < 20:
                w.beat()
                msg = w.check(60.0)
                time.sleep(0.05)
            res["failure_seen"] = msg
        else:
            for _ in range(20):
                w.beat()
                time.sleep(0.05)
            if grank == 1:
                w.fail("boom")
        faults.agree_healthy(g, True)  # resync before the silence check
        if grank == 0:
            # now nobody else beats: a 0.5 s heartbeat bound flags a silent peer
            w2 = faults.TrialWatch(w.store, 0, w.size)
            w2.store.delete_key("failed")
            t0 = time.monotonic()
            msg = None
            while msg is None and time.monotonic() - t0 < 20:
                msg = w2.check(0.5)
                time.sleep(0.05)
            res["silence_seen"] = msg
            res["silence_after_s"] = round(time.monotonic() - t0, 2)
    global_barrier()
    out(**res)
    _finish()


if __name__ == "__main__":
    mode = sys.argv[1]
    if mode == "groups":
        mode_groups(int(sys.argv[2]))
    elif mode == "reducer":
        mode_reducer()
    elif mode == "disagree":
        mode_disagree(sys.argv[2])
    elif mode == "arena_ddp":
        mode_arena_ddp()
    elif mode == "trainer_ddp":
        mode_trainer_ddp()
    elif mode == "autotune":
        mode_autotune()
    elif mode == "health":
        mode_health(int(sys.argv[2]))
    else:
        raise SystemExit(f"unknown mode {mode}")
