"""Intra-group DDP of the flagship conv-VAE on the HIP path (BASELINE configs
#4/#5; reference: ``DistributedDataParallel(model, process_group=group)`` at
/root/reference/vae-hpo.py:129-131 and the per-step all-reduce at :72).

``ConvVaeTrainer`` with a reducer attached runs a different step from the
single-replica one: per-bucket gradient finalize -> bucket all-reduce launched
while the rest of the backward is still being issued -> wait -> Adam + bf16
cast -> transposed copies. These tests run that step on the GPU:
  * a 1-rank RCCL world (the real RcclBucketReducer on torch's communicator):
    bucket layouts None / 0 / 0.5 MiB, eager and graph-replayed, 28x28 and
    128x128; results must equal the reducer-free step (the all-reduce over one
    rank is an identity) and the bucket launches must interleave with the
    backward GEMM launches;
  * s = 2 and 4 processes sharing the GPU through the p2p reducer
    (conv_ddp_worker.py): replicas bitwise identical, and equal to the
    single-process run when every replica draws the same eps.
Plus the bench/autotune graph-capture hygiene: after ``prepare`` a timed
``train_steps`` never captures.
"""
import json
import os
import socket
import sys

import numpy as np
import pytest
import torch
import torch.distributed as dist

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.fixture()
def nccl_world():
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ["MASTER_PORT"] = str(_free_port())
    torch.cuda.set_device(0)
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))
    yield dist.group.WORLD
    dist.destroy_process_group()


def _data(image, nb, B, dev):
    X = torch.rand(nb * B, image * image, generator=torch.Generator().manual_seed(3)).to(dev)
    return X, torch.arange(nb * B, device=dev, dtype=torch.int32)


def _trainer(image, B, dev, graphs, **kw):
    from multidisttorch_amd.models.conv_vae import ConvVaeTrainer

    return ConvVaeTrainer(batch_size=B, image=image, z=32 if image == 28 else 64, device=dev, backend="hip",
                          seed=4, lr=2e-3, use_graphs=graphs, graph_steps=4, **kw)


class _CallLog:
    """Proxy of the native module recording the order of launch-issuing calls."""

    def __init__(self, C, log):
        self._C, self._log = C, log

    def __getattr__(self, name):
        f = getattr(self._C, name)
        if not callable(f) or name[0].isupper():
            return f

        def wrap(*a, **k):
            self._log.append(name)
            return f(*a, **k)

        return wrap


class _RedLog:
    def __init__(self, red, log):
        self._red, self._log = red, log

    def bounds(self):
        return self._red.bounds()

    def launch(self, k):
        self._log.append(f"bucket{k}")
        return self._red.launch(k)

    def wait_all(self):
        self._log.append("wait_all")
        return self._red.wait_all()

    def __getattr__(self, n):
        return getattr(self._red, n)


@pytest.mark.parametrize("image", [28, 128])
def test_conv_trainer_rccl_reducer_matches_single(nccl_world, native_ext, image):
    from multidisttorch_amd.parallel.ddp import make_arena_reducer

    dev = torch.device("cuda", 0)
    B = 128 if image == 28 else 32
    nb, steps = 4, 8
    X, idx = _data(image, nb, B, dev)
    runs = {}
    for graphs in (False, True):
        for mb in ("single", None, 0, 0.5):
            tr = _trainer(image, B, dev, graphs)
            if mb != "single":
                red = make_arena_reducer(nccl_world, tr.grads, tr.bucket_bounds(mb))
                assert type(red).__name__ == "RcclBucketReducer"
                tr.attach_reducer(red)
            tr.bind_train_data(X, idx)
            tr.set_cursor(0, nb)
            tr.train_steps(steps)
            torch.cuda.synchronize()
            runs[(graphs, mb)] = (tr.params.clone(), tr.loss_history()[:steps].copy(), tr.read_state()["step"])
            if mb != "single":
                # host-side launches: every step eagerly, or the capture-time
                # warm-up step + the 4 captured steps of the S=4 graph
                assert red.launched_count() == (5 if graphs else steps) * red.num_buckets()
                assert red.pending() == 0
    p0, h0, s0 = runs[(False, "single")]
    assert s0 == steps and np.isfinite(h0).all()
    for key, (p, h, s) in runs.items():
        assert s == steps, key
        # one rank: the all-reduce is an identity; only where Adam runs differs
        # (fused into the finalize vs one flat launch after the all-reduce)
        np.testing.assert_allclose(h, h0, rtol=1e-5, err_msg=str(key))
        torch.testing.assert_close(p, p0, rtol=1e-5, atol=1e-6, msg=str(key))


@pytest.mark.parametrize("image,f28", [(28, True), (28, False), (128, False)])
def test_conv_bucket_launches_interleave_with_backward(nccl_world, native_ext, image, f28):
    """Eager step with three or more buckets: the first (decoder-end) bucket's
    all-reduce is issued before the backward GEMMs of the earlier layers, and
    the wait comes after the last backward launch. The fused 28x28 step
    (f28) issues the decoder bucket between its decoder and encoder
    weight-gradient launches."""
    from multidisttorch_amd.parallel.ddp import make_arena_reducer

    dev = torch.device("cuda", 0)
    B = 128 if image == 28 else 32
    X, idx = _data(image, 2, B, dev)
    tr = _trainer(image, B, dev, graphs=False)
    tr.ddp_overlap = True  # the overlap schedule (the auto rule picks one stream for the 28x28 RCCL step)
    if image == 28:
        assert tr.f28
        tr.f28 = f28
    bounds = tr.bucket_bounds(0.25 if image == 28 else 2.0)
    assert len(bounds) - 1 >= 3, bounds
    log = []
    tr.attach_reducer(_RedLog(make_arena_reducer(nccl_world, tr.grads, bounds), log))
    tr.bind_train_data(X, idx)
    tr.set_cursor(0, 2)
    tr.C = _CallLog(tr.C, log)
    tr.train_steps(1)
    torch.cuda.synchronize()
    nbk = len(bounds) - 1
    first = log.index(f"bucket{nbk - 1}")  # the last arena bucket holds the decoder: ready first
    wait = log.index("wait_all")
    bwd = [i for i, n in enumerate(log) if n in ("wgrad", "igemm", "thin_conv", "launch_jobs", "launch_jobs_multi")]
    assert any(first < i < wait for i in bwd), log
    assert all(f"bucket{k}" in log[:wait] for k in range(nbk)), log
    assert log.index("adam_cast") > wait, log
    if image == 28 and f28:
        jm = [i for i, n in enumerate(log) if n == "launch_jobs_multi"]
        assert len(jm) == 2 and jm[0] < first < jm[1], log  # decoder wgrads | decoder bucket | encoder wgrads


@pytest.mark.parametrize("image,f28,pair", [(28, True, True), (28, True, False), (28, False, False),
                                             (128, False, False)])
def test_conv_step_graph_issues_real_collectives(nccl_world, native_ext, image, f28, pair):
    """A one-rank group's all-reduce is an identity, so the reducer skips it
    unless told otherwise. Here it runs with PreMulSum scale 2 (a real
    ncclAllReduce on every bucket, captured into the replayed step graphs)
    while Adam's grad_scale is 0.5: the result equals the reducer-free run
    only if every collective actually executed inside the graph (a skipped
    one would leave the gradients at half)."""
    from multidisttorch_amd.parallel.ddp import make_arena_reducer

    dev = torch.device("cuda", 0)
    B = 128 if image == 28 else 32
    nb, steps = 4, 8
    X, idx = _data(image, nb, B, dev)
    runs = {}
    for mode, overlap in (("single", None), ("scaled", True), ("scaled", False)):
        tr = _trainer(image, B, dev, True)
        tr.ddp_overlap = overlap
        tr.f28_pair = pair  # the paired headline kernel under a real collective too
        if image == 28:
            tr.f28 = f28
        if mode == "scaled":
            red = make_arena_reducer(nccl_world, tr.grads, tr.bucket_bounds(0.25 if image == 28 else 2.0), scale=2.0)
            tr.attach_reducer(red)
            tr.set_hparams(grad_scale=0.5)
        tr.bind_train_data(X, idx)
        tr.set_cursor(0, nb)
        tr.train_steps(steps)
        torch.cuda.synchronize()
        runs[(mode, overlap)] = (tr.params.clone(), tr.loss_history()[:steps].copy())
        if mode == "scaled":
            assert red.launched_count() == 5 * red.num_buckets() and red.num_buckets() >= 2
            assert red.is_inline() == (image == 28 and f28 and not overlap)  # one-stream schedule: no events
    for ov in (True, False):
        np.testing.assert_allclose(runs[("scaled", ov)][1], runs[("single", None)][1], rtol=1e-5)
        torch.testing.assert_close(runs[("scaled", ov)][0], runs[("single", None)][0], rtol=1e-5, atol=1e-6)


@pytest.mark.parametrize("model", ["conv28", "mlp"])
def test_prepare_locks_graphs_for_timed_steps(native_ext, model):
    """bench.py contract: after prepare() the timed train_steps(20) with
    warmup=5, graph_steps=10 replays only pre-captured graphs."""
    from multidisttorch_amd.models.mlp_trainer import MlpVaeTrainer

    dev = torch.device("cuda", 0)
    X, idx = _data(28, 8, 128, dev)
    if model == "mlp":
        tr = MlpVaeTrainer(batch_size=128, device=dev, backend="hip", seed=1, use_graphs=True, graph_steps=10)
    else:
        tr = _trainer(28, 128, dev, True)
        tr.graph_steps = 10
    tr.bind_train_data(X, idx)
    tr.set_cursor(0, 8)
    tr.prepare([128])
    tr.strict_graphs = True
    keys = set(tr._graphs)
    assert keys == {(10, 128), (1, 128)}
    tr.train_steps(5)
    tr.train_steps(20)
    torch.cuda.synchronize()
    assert set(tr._graphs) == keys and tr.read_state()["step"] == 25
    with pytest.raises(RuntimeError, match="prepare"):
        tr.train_steps(1, M=64)


@pytest.mark.parametrize("s,image,graphs,mb,kind,mode,tail", [
    (2, 28, 1, "none", "p2p", "prod", 0), (4, 28, 1, "0.25", "p2p", "prod", 0),
    (2, 128, 1, "2", "p2p", "prod", 0), (4, 128, 0, "none", "p2p", "prod", 0),
    (2, 28, 1, "none", "p2p2", "prod", 0), (4, 128, 1, "2", "p2p2", "prod", 0),
    (2, 28, 0, "none", "xgmi", "split", 0), (4, 28, 0, "none", "xgmi", "split", 0),
    # the shipped default exactly: fused jobs with the in-kernel wait, graphs on,
    # paired kernel on, no split tail, no host barrier; CU-split ranks
    (2, 28, 1, "none", "xgmi", "cu", 0), (4, 28, 1, "none", "xgmi", "cu", 0),
    (2, 128, 1, "none", "xgmi", "cu", 0), (4, 128, 1, "none", "xgmi", "cu", 0),
    # full and tail batches alternate (different finalize-unit decompositions)
    (2, 28, 1, "none", "xgmi", "cu", 40), (2, 128, 1, "none", "xgmi", "cu", 8)])
def test_conv_p2p_multiprocess_ddp(s, image, graphs, mb, kind, mode, tail):
    from multidisttorch_amd.launch import launch

    # several processes share the GPU. "prod"/"split": the fused 28x28 step keeps
    # one workgroup per sample (MDT_F28_PAIR=0), and the "split" xgmi form runs
    # push and reduce in separate eager launches with a host barrier between
    # them. "cu": production defaults (pair on, graphs, in-kernel wait) with every
    # rank confined to its own CU share (MDT_CU_SPLIT=1, runtime/env.py), so a
    # rank's spinning reduce never holds the CUs its peers need.
    env = {"PYTHONPATH": ROOT, "OMP_NUM_THREADS": "2"}
    if mode == "cu":
        env["MDT_CU_SPLIT"] = "1"
    else:
        env["MDT_F28_PAIR"] = "0"
    wmode = "prod" if mode == "cu" else mode
    rc, outs = launch([sys.executable, os.path.join(HERE, "conv_ddp_worker.py"), str(image), str(graphs), mb, kind,
                       wmode, str(tail)], s, emulate="torchrun", timeout=150, extra_env=env, capture=True)
    text = "\n".join(o or "" for o in outs)
    assert rc == 0, text[-4000:]
    res = [json.loads(l[7:]) for l in text.splitlines() if l.startswith("RESULT ")]
    assert len(res) == s, text[-4000:]
    for r in res:
        for ph in ("same_eps", "indep_eps"):
            assert r[ph]["status"] == 0 and r[ph]["finite"], (ph, r)
            assert all(r[ph]["same"]), (ph, r)  # replicas bitwise identical at every check
            assert r[ph]["split"] == (mode == "split"), (ph, r)
            if kind.startswith("xgmi"):  # the data-plane self-test ran and passed before training
                assert r[ph]["selftest"] and r[ph]["selftest"]["result"] == "ok", (ph, r)
            if mode == "cu":
                assert r[ph]["cu_mask"], (ph, r)  # the rank really ran on its CU share
                if image == 28:
                    assert r[ph]["pair"], (ph, r)  # the paired headline kernel, as shipped
    r0 = [r for r in res if r["rank"] == 0][0]
    sg = r0["single"]
    assert sg["max_param_diff"] <= 1e-5 * max(1.0, sg["param_scale"]), sg
    np.testing.assert_allclose(r0["same_eps"]["loss"], sg["loss"], rtol=1e-5)
    # independent eps: per-replica losses differ (different samples of z)
    losses = [tuple(r["indep_eps"]["loss"]) for r in res]
    assert len(set(losses)) == s


def test_xgmi_falls_back_when_a_peer_cannot_be_mapped():
    """hipIpcOpenMemHandle failing on one member (e.g. GPU visibility
    restricted per rank; injected with MDT_TEST_IPC_FAIL_RANK) makes EVERY
    member fall back together (here: gloo world -> the c10d reducer), and the
    trial still trains data-parallel with bitwise-equal replicas."""
    from multidisttorch_amd.launch import launch

    env = {"PYTHONPATH": ROOT, "OMP_NUM_THREADS": "2", "MDT_CU_SPLIT": "1", "MDT_TEST_IPC_FAIL_RANK": "1"}
    rc, outs = launch([sys.executable, os.path.join(HERE, "conv_ddp_worker.py"), "28", "1", "none", "xgmi", "prod",
                       "0"], 2, emulate="torchrun", timeout=150, extra_env=env, capture=True)
    text = "\n".join(o or "" for o in outs)
    assert rc == 0, text[-4000:]
    res = [json.loads(l[7:]) for l in text.splitlines() if l.startswith("RESULT ")]
    assert len(res) == 2, text[-4000:]
    for r in res:
        for ph in ("same_eps", "indep_eps"):
            assert r[ph]["reducer"] == "BucketReducer", r
            assert all(r[ph]["same"]) and r[ph]["finite"], (ph, r)
    assert "falling back to the c10d reducer" in text


def test_xgmi_selftest_failure_falls_back_on_every_member():
    """The construction-time data-plane self-test (parallel/ddp.py
    ``selftest_fused``) failing on ONE member (injected with
    MDT_TEST_XGMI_SELFTEST_FAIL_RANK=1 after a real push+reduce ran) makes
    every member drop the fused reducer together: both take the collective
    fallback (gloo world -> the c10d reducer), train, and end with bitwise-equal
    replicas."""
    from multidisttorch_amd.launch import launch

    env = {"PYTHONPATH": ROOT, "OMP_NUM_THREADS": "2", "MDT_CU_SPLIT": "1", "MDT_TEST_XGMI_SELFTEST_FAIL_RANK": "1"}
    rc, outs = launch([sys.executable, os.path.join(HERE, "conv_ddp_worker.py"), "28", "1", "none", "xgmi", "prod",
                       "0"], 2, emulate="torchrun", timeout=150, extra_env=env, capture=True)
    text = "\n".join(o or "" for o in outs)
    assert rc == 0, text[-4000:]
    res = [json.loads(l[7:]) for l in text.splitlines() if l.startswith("RESULT ")]
    assert len(res) == 2, text[-4000:]
    for r in res:
        for ph in ("same_eps", "indep_eps"):
            st = r[ph]["selftest"]
            assert st["result"] == "fallback" and st["status"] == [0], (ph, r)  # the data plane itself was fine
            assert st["local_ok"] == (r["rank"] != 1), (ph, r)
            assert r[ph]["reducer"] == "BucketReducer", r
            assert all(r[ph]["same"]) and r[ph]["finite"], (ph, r)
    assert "self-test failed" in text and "falling back to the c10d reducer" in text


def _worker_results(s, image, kind, tail=0):
    from multidisttorch_amd.launch import launch

    env = {"PYTHONPATH": ROOT, "OMP_NUM_THREADS": "2", "MDT_CU_SPLIT": "1"}
    rc, outs = launch([sys.executable, os.path.join(HERE, "conv_ddp_worker.py"), str(image), "1", "none", kind, "prod",
                       str(tail)], s, emulate="torchrun", timeout=150, extra_env=env, capture=True)
    text = "\n".join(o or "" for o in outs)
    assert rc == 0, text[-4000:]
    res = [json.loads(l[7:]) for l in text.splitlines() if l.startswith("RESULT ")]
    assert len(res) == s, text[-4000:]
    return {r["rank"]: r for r in res}


@pytest.mark.parametrize("image,tail", [(128, 0), (28, 40)])
def test_fused_two_shot_is_bitwise_one_shot(image, tail):
    """The fused jobs' two-shot form (reduce-scatter to chunk owners +
    all-gather, 2/s of the arena per link; groups >= 3) sums every chunk in
    rank order with the same scale as the one-shot form: four CU-split ranks
    end bitwise where the one-shot run ends, full and tail batches alike."""
    one = _worker_results(4, image, "xgmi1", tail)
    two = _worker_results(4, image, "xgmi2", tail)
    for r in range(4):
        for ph in ("same_eps", "indep_eps"):
            assert one[r][ph]["two_shot"] is False and two[r][ph]["two_shot"] is True
            assert one[r][ph]["status"] == 0 and two[r][ph]["status"] == 0
            assert all(two[r][ph]["same"]), (ph, two[r])
            assert two[r][ph]["phash"] == one[r][ph]["phash"], (r, ph)
