"""Direct-RCCL bucket reducer (csrc/runtime/xgmi_comm.cpp) on torch's communicator.

One MI355X per gpurun box, so the group has one rank: the collective then
reduces a single contribution, which still exercises the whole path — the
communicator borrowed from ProcessGroupNCCL, the PreMulSum(scale) op, the
high-priority comm stream with event fences, and hipGraph capture. An
explicit scale makes the pre-multiplication observable.
"""
import os
import socket

import pytest
import torch
import torch.distributed as dist

pytestmark = pytest.mark.gpu


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


def test_rccl_reducer_premulsum_and_graph(nccl_world, native_ext):
    from multidisttorch_amd.parallel.ddp import make_arena_reducer, rccl_comm_ptr, reducer_kind

    C = native_ext
    dev = torch.device("cuda", 0)
    flat = torch.randn(1 << 20, device=dev)
    assert reducer_kind(nccl_world, flat) == "rccl"
    ref = flat.clone()
    bounds = [0, 300_000, 1 << 20]
    red = C.RcclBucketReducer(rccl_comm_ptr(nccl_world, dev), 1, flat, bounds, True, 0.5)
    assert red.num_buckets() == 2 and abs(red.scale() - 0.5) < 1e-7
    red.launch(1)
    red.launch(0)
    red.wait_all()
    torch.cuda.synchronize()
    torch.testing.assert_close(flat, ref * 0.5)
    # readiness mode
    red.set_param_map([0, 0, 1])
    for p in range(3):
        red.mark_ready(p)
    assert red.pending() == 2
    red.wait_all()
    red.reset_iteration()
    torch.cuda.synchronize()
    torch.testing.assert_close(flat, ref * 0.25)
    # capture launch+wait in a graph: each replay scales by 0.5 again
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=s):
        red.launch_all()
        red.wait_all()
    torch.cuda.synchronize()
    before = flat.clone()
    for _ in range(3):
        g.replay()
    torch.cuda.synchronize()
    torch.testing.assert_close(flat, before * 0.125)
    # the factory picks the RCCL path and averages (1/s = 1 on one rank)
    red2 = make_arena_reducer(nccl_world, flat, bounds)
    cur = flat.clone()
    red2.launch_all()
    red2.wait_all()
    torch.cuda.synchronize()
    torch.testing.assert_close(flat, cur)
    assert C.rccl_version() >= 22600


def test_mlp_trainer_with_rccl_reducer(nccl_world, native_ext):
    """Fused MLP step with bucket launches between the backward kernels."""
    import numpy as np

    from multidisttorch_amd.models.mlp_trainer import MlpVaeTrainer
    from multidisttorch_amd.parallel.ddp import make_arena_reducer

    dev = torch.device("cuda", 0)
    X = torch.rand(1024, 784, device=dev)
    idx = torch.arange(1024, device=dev, dtype=torch.int32)
    hist = []
    for use_red in (False, True):
        tr = MlpVaeTrainer(batch_size=128, device=dev, backend="hip", seed=5, use_graphs=True, graph_steps=4)
        if use_red:
            tr.attach_reducer(make_arena_reducer(nccl_world, tr.grads, [0, tr.split, tr.numel]))
        tr.bind_train_data(X, idx)
        tr.set_cursor(0, 8)
        tr.train_steps(12)
        torch.cuda.synchronize()
        hist.append(tr.loss_history()[:12].copy())
    # one rank: the all-reduce is an identity, only the Adam path differs
    # (separate flat Adam instead of the fused epilogue) -> same losses
    np.testing.assert_allclose(hist[0], hist[1], rtol=1e-5)


def test_trial_groups_split_from_device_bound_world(nccl_world, native_ext):
    """Eager device-bound world -> trial communicators via ncclCommSplit; the
    direct-RCCL reducer then runs on the split communicator."""
    from multidisttorch_amd.parallel import ddp
    from multidisttorch_amd.parallel.ddp import make_arena_reducer
    from multidisttorch_amd.parallel.groups import setup_ddp_groups
    from multidisttorch_amd.runtime.bootstrap import world_is_device_bound

    assert world_is_device_bound()
    (pg,) = setup_ddp_groups(1, verbose=False)
    assert dist.get_rank(pg) == 0
    assert pg.bound_device_id is not None
    flat = torch.randn(4096, device="cuda")
    ref = flat.clone()
    warm = ddp.COMM_WARMUPS[0]
    red = make_arena_reducer(pg, flat, [0, 1024, 4096])
    # the split communicator exists already: no warm-up all-reduce was needed
    assert ddp.COMM_WARMUPS[0] == warm
    red.launch_all()
    red.wait_all()
    torch.cuda.synchronize()
    torch.testing.assert_close(flat, ref)


def test_autotune_comm_times_rccl_and_p2p(nccl_world, native_ext, tmp_path):
    """The measured autotuner searches (reducer kind x bucket layout) on a GPU
    group; on one rank both reducers are identities, so training is unchanged."""
    import numpy as np

    from multidisttorch_amd.models.mlp_trainer import MlpVaeTrainer
    from multidisttorch_amd.parallel.autotune import autotune_comm
    from multidisttorch_amd.parallel.ddp import make_arena_reducer

    dev = torch.device("cuda", 0)
    X = torch.rand(1024, 784, device=dev)
    idx = torch.arange(1024, device=dev, dtype=torch.int32)
    make = lambda: MlpVaeTrainer(batch_size=128, device=dev, backend="hip", seed=3, use_graphs=True, graph_steps=4)
    bounds, kind, timings = autotune_comm(make, nccl_world, X, idx, candidates=(None, 0), steps=4, warmup=2,
                                          key="gpu-test", cache=str(tmp_path / "b.json"))
    assert kind in ("rccl", "p2p1", "xgmi1")
    assert all(any(k.startswith(c + ":") for k in timings) for c in ("rccl", "p2p1", "xgmi1"))
    hist = []
    for k in ("rccl", "p2p", "xgmi"):
        tr = make()
        tr.attach_reducer(make_arena_reducer(nccl_world, tr.grads, bounds, kind=k))
        tr.bind_train_data(X, idx)
        tr.set_cursor(0, 8)
        tr.train_steps(8)
        torch.cuda.synchronize()
        hist.append(tr.loss_history()[:8].copy())
    np.testing.assert_array_equal(hist[0], hist[1])
    np.testing.assert_array_equal(hist[0], hist[2])
