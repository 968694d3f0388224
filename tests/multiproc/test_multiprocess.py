"""Multi-process CPU/gloo tests (BASELINE config #1 plumbing), launched with the
framework's own launcher under emulated SLURM / Open MPI / torchrun env."""
import json
import os
import re
import sys

import pytest
import torch

from multidisttorch_amd.launch import launch

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
WORKER = os.path.join(HERE, "worker.py")
ENV = {"DDP_BACKEND": "gloo", "OMP_NUM_THREADS": "1", "PYTHONPATH": ROOT}


def _results(outs):
    res = []
    for o in outs:
        for line in (o or "").splitlines():
            if line.startswith("RESULT "):
                res.append(json.loads(line[7:]))
    return res


def _run(args, n, emulate="torchrun", timeout=180, cwd=None, extra_env=None):
    cmd = [sys.executable] + args
    old = os.getcwd()
    if cwd:
        os.chdir(cwd)
    try:
        rc, outs = launch(cmd, n, emulate=emulate, timeout=timeout, extra_env={**ENV, **(extra_env or {})},
                          capture=True)
    finally:
        os.chdir(old)
    return rc, outs


@pytest.mark.parametrize("w,k,emulate", [(2, 2, "slurm"), (4, 2, "ompi"), (5, 2, "torchrun"), (3, 1, "slurm")])
def test_group_carving(w, k, emulate):
    rc, outs = _run([WORKER, "groups", str(k)], w, emulate)
    assert rc == 0, "\n".join(outs)
    res = sorted(_results(outs), key=lambda r: r["rank"])
    assert len(res) == w
    n = w // k
    for r in res:
        g = r["rank"] // n
        if g < k:
            assert r["member"] == [g]
            assert r["gathered"] == list(range(g * n, g * n + n))
            assert r["grank"][g] == r["rank"] - g * n
        else:  # leftover rank: idle but joins the control-plane barrier (no crash, Q3)
            assert r["member"] == [] and r["gathered"] is None
    text = "\n".join(outs)
    # reference print formats (utils.py:149, :161, :174)
    assert f"world_size, world_rank: {w} 0" in text
    assert "Rank 0 is in group 0" in text
    assert re.search(r"^\[0:0\] hello from group 0$", text, re.M)


def test_native_and_python_reducer():
    rc, outs = _run([WORKER, "reducer"], 2)
    assert rc == 0, "\n".join(outs)
    for r in _results(outs):
        assert r["native"] == 0.0 and r["py"] == 0.0
        assert r["type_native"] == "BucketReducer"
        assert r["ready_native"] == [3.0, 3.0] and r["ready_py"] == [3.0, 3.0]


@pytest.mark.parametrize("what,field", [("numel", "numel"), ("bounds", "bounds"), ("kind", "kind")])
def test_reducer_disagreement_raises_on_every_member(what, field):
    """Construction-time agreement (DDP ctor X3/X4 analogue):
    a member whose arena is one element larger (or whose bucket bounds or
    reducer kind differ) makes EVERY member raise, naming group rank 1, before
    any peer memory is mapped or any gradient moves."""
    rc, outs = _run([WORKER, "disagree", what], 2)
    assert rc == 0, "\n".join(outs)
    res = _results(outs)
    assert len(res) == 2
    for r in res:
        assert r["err"] and "group rank 1 differs in" in r["err"] and field in r["err"], r
        assert r["after"] == 2.0


def test_arena_ddp_matches_torch_ddp():
    rc, outs = _run([WORKER, "arena_ddp"], 2)
    assert rc == 0, "\n".join(outs)
    res = _results(outs)
    assert len(res) == 2
    for r in res:
        assert r["err"] < 1e-5 and r["buckets"] >= 2


def test_trainer_replicas_stay_in_sync():
    rc, outs = _run([WORKER, "trainer_ddp"], 2)
    assert rc == 0, "\n".join(outs)
    for r in _results(outs):
        assert r["maxdiff"] == 0.0 and r["step"] == 5


def test_bucket_autotune_agrees_across_group(tmp_path):
    old = dict(ENV)
    ENV["MDT_BUCKET_CACHE"] = str(tmp_path / "buckets.json")
    try:
        rc, outs = _run([WORKER, "autotune"], 2)
    finally:
        ENV.clear()
        ENV.update(old)
    assert rc == 0, "\n".join(outs)
    res = _results(outs)
    assert len(res) == 2 and res[0]["best"] == res[1]["best"]
    assert res[0]["n"] == 3 and res[0]["cached"]
    assert all(r["maxdiff"] == 0.0 for r in res)


def test_example_subgroup_world4(tmp_path):
    old = dict(ENV)
    ENV["MDT_EXAMPLE_WORLD"] = "4"
    try:
        rc, outs = _run([os.path.join(ROOT, "example-subgroup.py")], 4, "slurm", cwd=str(tmp_path))
    finally:
        ENV.clear()
        ENV.update(old)
    text = "\n".join(outs)
    assert rc == 0, text
    assert "0 gather_list: [tensor([0]), tensor([1])]" in text
    assert "2 gather_list: [tensor([2]), tensor([3])]" in text


def _vae_hpo(tmp_path, n, *args, emulate="slurm"):
    return _run([os.path.join(ROOT, "vae-hpo.py"), "--train-samples", "1024", "--test-samples", "256",
                 "--batch-size", "64"] + list(args), n, emulate, timeout=300, cwd=str(tmp_path))


def test_vae_hpo_two_trials_config1(tmp_path):
    rc, outs = _vae_hpo(tmp_path, 2, "--epochs", "1", "--ngroups", "2", "--metrics-dir", "m")
    text = "\n".join(outs)
    assert rc == 0, text
    # trial g trains epochs+g epochs (vae-hpo.py:202): trial 1 logs epoch 2
    assert re.search(r"^\[1:0\] ====> Epoch: 2 Average loss: \d+\.\d{4}$", text, re.M)
    assert not re.search(r"^\[0:0\] ====> Epoch: 2", text, re.M)
    assert re.search(r"^\[0:0\] Train Epoch: 1 \[0/1024 \(0%\)\]\tLoss: \d+\.\d{6}$", text, re.M)
    assert re.search(r"^\[0:0\] ====> Test set loss: \d+\.\d{4}$", text, re.M)
    assert re.search(r"^0 Done\. time: \d+\.\d{6}$", text, re.M)
    agg = json.loads(re.search(r"MDT_AGGREGATE (.*)", text).group(1))
    assert agg["trials"] == 2 and agg["samples"] == 512 * 1 + 512 * 2
    assert (tmp_path / "results-0" / "sample_1.png").exists()
    assert (tmp_path / "m" / "trial-1.jsonl").exists()


def test_vae_hpo_intra_group_ddp_and_resume(tmp_path):
    rc, outs = _vae_hpo(tmp_path, 2, "--epochs", "1", "--ngroups", "1", "--ckpt-dir", "ck", "--no-results")
    assert rc == 0, "\n".join(outs)
    assert (tmp_path / "ck" / "trial-0" / "epoch-1.pt").exists()
    rc, outs = _vae_hpo(tmp_path, 2, "--epochs", "2", "--ngroups", "1", "--ckpt-dir", "ck", "--resume",
                        "--no-results")
    text = "\n".join(outs)
    assert rc == 0, text
    assert "resumed trial 0" in text and "Epoch: 2 Average" in text and "Epoch: 1 Average" not in text
    ck = torch.load(str(tmp_path / "ck" / "trial-0" / "epoch-2.pt"), weights_only=True)
    assert ck["progress"]["epoch"] == 2


def test_vae_hpo_idle_leftover_rank(tmp_path):
    rc, outs = _vae_hpo(tmp_path, 3, "--epochs", "1", "--ngroups", "2", "--no-results", emulate="torchrun")
    text = "\n".join(outs)
    assert rc == 0, text  # the reference crashes here
    assert "Rank 2 is in group" not in text


def test_failed_trial_is_isolated(tmp_path):
    """An injected failure in trial 1 does not stop trial 0 (reference: crash/hang)."""
    old = dict(ENV)
    ENV["MDT_FAULT"] = "trial=1,epoch=1"
    try:
        rc, outs = _vae_hpo(tmp_path, 2, "--epochs", "1", "--ngroups", "2", "--no-results")
    finally:
        ENV.clear()
        ENV.update(old)
    text = "\n".join(outs)
    assert rc == 0, text
    assert "trial 1 (world rank 1) FAILED: InjectedFault" in text
    assert re.search(r"^\[0:0\] ====> Test set loss", text, re.M)
    agg = json.loads(re.search(r"MDT_AGGREGATE (.*)", text).group(1))
    assert agg["failed_trials"] == [1] and agg["samples"] == 512


def test_vae_hpo_packed_trials(tmp_path):
    """Two single-rank groups x two packed trials = four concurrent trials."""
    rc, outs = _vae_hpo(tmp_path, 2, "--epochs", "1", "--ngroups", "2", "--trials-per-group", "2",
                        "--metrics-dir", "m")
    text = "\n".join(outs)
    assert rc == 0, text
    agg = json.loads(re.search(r"MDT_AGGREGATE (.*)", text).group(1))
    # trial t trains 1+t epochs on a 1/4 shard (256 samples)
    assert agg["trials"] == 4 and agg["samples"] == 256 * (1 + 2 + 3 + 4) and agg["failed_trials"] == []
    assert re.search(r"^\[1:0\] \(trial 3\) ====> Epoch: 4 Average loss: \d+\.\d{4}$", text, re.M)
    assert (tmp_path / "results-t2-0" / "sample_3.png").exists()
    assert (tmp_path / "m" / "trial-3.jsonl").exists()


def test_vae_hpo_profile_and_dtype_flags(tmp_path):
    rc, outs = _vae_hpo(tmp_path, 1, "--epochs", "1", "--ngroups", "1", "--profile", "--dtype", "fp32")
    assert rc == 0, "\n".join(outs)
    rec = [json.loads(l) for l in open(tmp_path / "metrics" / "trial-0.jsonl")]
    ep = [r for r in rec if r.get("epoch") == 1][0]
    assert {"eval_s", "sample_s", "ckpt_s", "epoch_train_s"} <= set(ep)
    rc, outs = _vae_hpo(tmp_path, 1, "--epochs", "1", "--ngroups", "1", "--dtype", "bf16")
    assert rc != 0 and "computes in fp32" in "\n".join(outs)


@pytest.mark.parametrize("n,k", [(2, None), (4, 2)])
def test_bench_contract_multirank(tmp_path, n, k):
    """bench.py under torchrun-style env (the driver's N>1 launch): rank 0 prints ONE
    JSON line with the BASELINE metric, n_gpus = N, trials = K, samples counted once
    per trial (K x batch x steps / max-rank time)."""
    args = [os.path.join(ROOT, "bench.py"), "--gpus", str(n), "--steps", "2", "--warmup", "1",
            "--model", "mlp", "--batch-size", "64"]
    if k:
        args += ["--ngroups", str(k)]
    rc, outs = _run(args, n, "torchrun", timeout=240, cwd=str(tmp_path))
    text = "\n".join(outs)
    assert rc == 0, text
    lines = [l for l in text.splitlines() if l.startswith("{\"metric\"")]
    assert len(lines) == 1, text
    out = json.loads(lines[0])
    K = k or n
    assert out["n_gpus"] == n and out["steps"] == 2 and out["warmup"] == 1
    assert out["config"]["trials"] == K and out["config"]["parallelism"] == f"groups{K}x{n // K}"
    assert out["config"]["valid"] is True
    assert out["config"]["replicas_bitwise_equal"] is (True if n // K > 1 else None)
    assert abs(out["value"] - K * 64 * 2 / (out["ms_per_step"] * 2e-3)) / out["value"] < 0.01


@pytest.mark.parametrize("model,k,bs", [("conv28", 4, 128), ("conv128", 2, 8)])
def test_bench_contract_conv_groups_n8(tmp_path, model, k, bs):
    """BASELINE configs #4/#5 shape at n = 8 (torch backend, gloo): K trial
    groups of 8 // K ranks each run intra-group DDP; one JSON line with the
    group layout and samples counted once per trial."""
    args = [os.path.join(ROOT, "bench.py"), "--gpus", "8", "--steps", "2", "--warmup", "1", "--model", model,
            "--ngroups", str(k), "--batch-size", str(bs), "--backend", "torch"]
    rc, outs = _run(args, 8, "torchrun", timeout=400, cwd=str(tmp_path), extra_env={"OMP_NUM_THREADS": "1"})
    text = "\n".join(o or "" for o in outs)
    assert rc == 0, text[-4000:]
    lines = [l for l in text.splitlines() if l.startswith("{\"metric\"")]
    assert len(lines) == 1, text[-4000:]
    out = json.loads(lines[0])
    assert out["n_gpus"] == 8 and out["config"]["trials"] == k
    assert out["config"]["parallelism"] == f"groups{k}x{8 // k}"
    assert out["config"]["model"].startswith("conv")
    assert abs(out["value"] - k * bs * 2 / (out["ms_per_step"] * 2e-3)) / out["value"] < 0.01
    # every replica of every trial ends bitwise equal (bench gathers the parameters)
    assert out["config"]["replicas_bitwise_equal"] is True and out["config"]["valid"] is True


def test_vae_hpo_conv_ckpt_and_resume(tmp_path):
    """--model conv --ckpt-dir then --resume (the conv checkpoint
    path crashed on int(trainer.H) and silently failed the trial)."""
    rc, outs = _vae_hpo(tmp_path, 2, "--model", "conv", "--epochs", "1", "--ngroups", "1", "--ckpt-dir", "ck",
                        "--no-results")
    text = "\n".join(outs)
    assert rc == 0, text
    assert "FAILED" not in text
    assert (tmp_path / "ck" / "trial-0" / "epoch-1.pt").exists()
    rc, outs = _vae_hpo(tmp_path, 2, "--model", "conv", "--epochs", "2", "--ngroups", "1", "--ckpt-dir", "ck",
                        "--resume", "--no-results")
    text = "\n".join(outs)
    assert rc == 0, text
    assert "FAILED" not in text
    assert "resumed trial 0" in text and "Epoch: 2 Average" in text and "Epoch: 1 Average" not in text
    ck = torch.load(str(tmp_path / "ck" / "trial-0" / "epoch-2.pt"), weights_only=True)
    assert ck["progress"]["epoch"] == 2 and ck["arch"]["kind"] == "conv"
    agg = json.loads(re.search(r"MDT_AGGREGATE (.*)", text).group(1))
    assert agg["failed_trials"] == []


def test_failure_inside_multi_rank_group(tmp_path):
    """Group of 2 + a rank-specific mid-epoch fault (isolation only
    held for single-rank groups). Rank 1 stops issuing steps at step 3 while
    its peer is inside the step-3 all-reduce: the peer times out, both members
    agree the trial failed, the other trial finishes, everyone exits 0."""
    old = dict(ENV)
    ENV["MDT_FAULT"] = "rank=3,step=3"
    ENV["MDT_GROUP_TIMEOUT_S"] = "8"
    try:
        rc, outs = _vae_hpo(tmp_path, 4, "--epochs", "1", "--ngroups", "2", "--no-results")
    finally:
        ENV.clear()
        ENV.update(old)
    text = "\n".join(outs)
    assert rc == 0, text
    assert "trial 1 (world rank 3) FAILED: InjectedFault" in text
    assert "trial 1 (world rank 2) FAILED" in text
    assert re.search(r"^\[0:0\] ====> Test set loss", text, re.M)
    agg = json.loads(re.search(r"MDT_AGGREGATE (.*)", text).group(1))
    assert agg["failed_trials"] == [1] and agg["trials"] == 2


def test_health_groups_idle_rank_and_watch():
    """W=5, K=2 (rank 4 idle): health groups come up without any world-
    collective new_group (on a device-bound RCCL world that path made an idle
    rank issue one ncclCommSplit more than the members: ADVICE r2), members
    agree, and the store heartbeat reports a published failure and a silent
    peer."""
    rc, outs = _run([WORKER, "health", "2"], 5, "torchrun", timeout=120)
    text = "\n".join(o or "" for o in outs)
    assert rc == 0, text
    res = {r["rank"]: r for r in _results(outs)}
    assert sorted(res) == [0, 1, 2, 3, 4], text
    assert res[4]["group"] is None and not res[4]["has_pg"]
    for r in range(4):
        assert res[r]["has_pg"] and res[r]["agree_all_ok"] is True and res[r]["agree_one_bad"] is False
    for r in (0, 2):
        assert "rank 1: boom" in res[r]["failure_seen"], res[r]
        assert "sent no heartbeat" in res[r]["silence_seen"] and res[r]["silence_after_s"] < 5, res[r]


def test_resume_arch_mismatch_fails_every_member_together(tmp_path):
    """A 2-rank trial resuming from a checkpoint of another architecture: only
    group rank 0 reads it, and its load error reaches the replica before the
    parameter broadcast, so BOTH members raise (the replica used to
    wait in the broadcast until the collective timeout)."""
    rc, outs = _vae_hpo(tmp_path, 2, "--epochs", "1", "--ngroups", "1", "--ckpt-dir", "ck", "--no-results")
    assert rc == 0, "\n".join(outs)
    t0 = __import__("time").monotonic()
    rc, outs = _vae_hpo(tmp_path, 2, "--model", "conv", "--epochs", "2", "--ngroups", "1", "--ckpt-dir", "ck",
                        "--resume", "--no-results")
    took = __import__("time").monotonic() - t0
    text = "\n".join(o or "" for o in outs)
    assert rc != 0, text
    assert "could not load its checkpoint" in text, text[-3000:]
    assert took < 120, took
