"""Launcher discovery parity (reference utils.py:9-26, :40-56, :59-90, :108-119)."""
import pytest

from multidisttorch_amd.runtime import env as E


def test_precedence_ompi_over_slurm_over_torchrun():
    e = {"OMPI_COMM_WORLD_SIZE": "6", "OMPI_COMM_WORLD_RANK": "5", "SLURM_NPROCS": "4",
         "SLURM_PROCID": "3", "WORLD_SIZE": "2", "RANK": "1"}
    assert E.init_comm_size_and_rank(e) == (6, 5)
    e.pop("OMPI_COMM_WORLD_SIZE")
    assert E.init_comm_size_and_rank(e) == (4, 3)
    e.pop("SLURM_NPROCS")
    assert E.init_comm_size_and_rank(e) == (2, 1)  # extension: torchrun honoured (Q1)
    assert E.init_comm_size_and_rank({}) == (1, 0)


def test_partial_env_falls_through():
    # reference requires BOTH size and rank of a launcher
    assert E.init_comm_size_and_rank({"OMPI_COMM_WORLD_SIZE": "4"}) == (1, 0)
    assert E.init_comm_size_and_rank({"SLURM_PROCID": "2"}) == (1, 0)


def test_local_rank():
    assert E.local_rank_from_env({"OMPI_COMM_WORLD_LOCAL_RANK": "3"}) == 3
    assert E.local_rank_from_env({"SLURM_LOCALID": "2"}) == 2
    assert E.local_rank_from_env({"LOCAL_RANK": "1"}) == 1
    assert E.local_rank_from_env({}, world_rank=13, ndev=8) == 5


@pytest.mark.parametrize("s,expect", [
    ("or-condo-g04", ["or-condo-g04"]),
    ("or-condo-g[05,07-08,13]", ["or-condo-g05", "or-condo-g07", "or-condo-g08", "or-condo-g13"]),
    ("or-condo-g[05,07-08,13],or-condo-h[01,12]",
     ["or-condo-g05", "or-condo-g07", "or-condo-g08", "or-condo-g13", "or-condo-h01", "or-condo-h12"]),
    ("frontier[00001-00003]", ["frontier00001", "frontier00002", "frontier00003"]),
    ("a1,b2", ["a1", "b2"]),
    ("node[8-11]", ["node8", "node9", "node10", "node11"]),
    ("localhost", ["localhost"]),
])
def test_parse_slurm_nodelist(s, expect):
    assert E.parse_slurm_nodelist(s) == expect


def test_find_ifname_loopback():
    assert E.find_ifname("127.0.0.1") in ("lo", "lo0")
    assert E.find_ifname("203.0.113.77") is None


def test_master_discovery():
    assert E.discover_master({}) == ("127.0.0.1", "8889")
    assert E.discover_master({"MASTER_ADDR": "h", "MASTER_PORT": "1"}) == ("h", "1")
    assert E.discover_master({"LSB_HOSTS": "batch1 h1 h1 h2"})[0] == "h1"
    assert E.discover_master({"LSB_MCPU_HOSTS": "batch1 1 h7 42"})[0] == "h7"
    assert E.discover_master({"SLURM_NODELIST": "or-condo-g[05,07]"})[0] == "or-condo-g05"


def test_discover_launcher_name():
    assert E.discover({"SLURM_NPROCS": "2", "SLURM_PROCID": "1"}).launcher == "slurm"
    assert E.discover({}).launcher == "single"


def test_eager_device_bound_world_default(monkeypatch):
    """One GPU per local rank -> eager device-bound RCCL world by default
    (trial groups then come from ncclCommSplit); shared or unknown -> lazy."""
    from multidisttorch_amd.runtime import env as E
    from multidisttorch_amd.runtime.bootstrap import eager_comm_requested

    monkeypatch.delenv("MDT_EAGER_COMM", raising=False)
    info = E.discover({"WORLD_SIZE": "8", "RANK": "3", "LOCAL_RANK": "3", "LOCAL_WORLD_SIZE": "8"}, ndev=8)
    assert info.local_size == 8 and eager_comm_requested(info, 8)
    assert not eager_comm_requested(info, 1)  # 8 ranks sharing one visible GPU
    info2 = E.discover({"SLURM_NPROCS": "4", "SLURM_PROCID": "1"}, ndev=8)
    assert info2.local_size is None and not eager_comm_requested(info2, 8)
    assert E.discover({"OMPI_COMM_WORLD_SIZE": "2", "OMPI_COMM_WORLD_RANK": "0",
                       "OMPI_COMM_WORLD_LOCAL_SIZE": "2"}).local_size == 2
    monkeypatch.setenv("MDT_EAGER_COMM", "0")
    assert not eager_comm_requested(info, 8)
    monkeypatch.setenv("MDT_EAGER_COMM", "1")
    assert eager_comm_requested(info2, 8)


def test_slurm_tasks_per_node_forms():
    """SLURM's compressed per-node task lists (srun exports no LOCAL_WORLD_SIZE)."""
    from multidisttorch_amd.runtime import env as E

    assert E.parse_slurm_tasks_per_node("8(x2)") == [8, 8]
    assert E.parse_slurm_tasks_per_node("4,2") == [4, 2]
    assert E.parse_slurm_tasks_per_node("2(x3),1") == [2, 2, 2, 1]
    for bad in ("", "x", "0", "2(x0)"):
        with pytest.raises(ValueError):
            E.parse_slurm_tasks_per_node(bad)
    base = {"SLURM_NPROCS": "10", "SLURM_PROCID": "9", "SLURM_LOCALID": "1"}
    assert E.local_size_from_env(dict(base, SLURM_TASKS_PER_NODE="8(x2)")) == 8
    assert E.local_size_from_env(dict(base, SLURM_TASKS_PER_NODE="8,2", SLURM_NODEID="1")) == 2
    assert E.local_size_from_env(dict(base, SLURM_TASKS_PER_NODE="8,2")) is None  # which node? unknown
    # the step's own list wins over the allocation's
    assert E.local_size_from_env(dict(base, SLURM_TASKS_PER_NODE="8(x2)", SLURM_STEP_TASKS_PER_NODE="4(x2)")) == 4
    assert E.local_size_from_env(dict(base, SLURM_NTASKS_PER_NODE="2", SLURM_TASKS_PER_NODE="8(x2)")) == 2


def test_eager_split_chosen_under_emulated_srun(monkeypatch):
    """A plain ``srun -N2 --ntasks-per-node 8`` environment (no LOCAL_WORLD_SIZE,
    only SLURM's lists) on 8-GPU nodes selects the eager device-bound world."""
    from multidisttorch_amd.runtime import env as E
    from multidisttorch_amd.runtime.bootstrap import eager_comm_requested

    monkeypatch.delenv("MDT_EAGER_COMM", raising=False)
    srun = {"SLURM_NPROCS": "16", "SLURM_PROCID": "11", "SLURM_LOCALID": "3", "SLURM_NODEID": "1",
            "SLURM_NODELIST": "node[01-02]", "SLURM_TASKS_PER_NODE": "8(x2)", "SLURM_STEP_TASKS_PER_NODE": "8(x2)"}
    info = E.discover(srun, ndev=8)
    assert info.launcher == "slurm" and info.local_rank == 3 and info.local_size == 8
    assert eager_comm_requested(info, 8)
    # 16 tasks crammed on one 8-GPU node: lazy path (and setup_ddp refuses RCCL)
    info2 = E.discover(dict(srun, SLURM_TASKS_PER_NODE="16", SLURM_STEP_TASKS_PER_NODE="16", SLURM_NODEID="0"), ndev=8)
    assert info2.local_size == 16 and not eager_comm_requested(info2, 8)


def test_bind_refuses_more_rccl_ranks_than_gpus(monkeypatch):
    """_bind_local_device fails loudly instead of wrapping local ranks onto
    shared GPUs when the backend is RCCL (it would die later with 'Duplicate
    GPU detected'); gloo may share (with a warning)."""
    import torch

    from multidisttorch_amd.runtime import bootstrap as B
    from multidisttorch_amd.runtime import env as E

    monkeypatch.setattr(torch.cuda, "is_available", lambda: True)
    monkeypatch.setattr(torch.cuda, "device_count", lambda: 8)
    monkeypatch.setattr(torch.cuda, "set_device", lambda i: None)
    info = E.discover({"WORLD_SIZE": "9", "RANK": "8", "LOCAL_RANK": "8", "LOCAL_WORLD_SIZE": "9"}, ndev=8)
    with pytest.raises(RuntimeError, match="one process per GPU"):
        B._bind_local_device(info, "nccl")
    assert B._bind_local_device(info, "gloo") == torch.device("cuda", 0)
    ok = E.discover({"WORLD_SIZE": "8", "RANK": "7", "LOCAL_RANK": "7", "LOCAL_WORLD_SIZE": "8"}, ndev=8)
    assert B._bind_local_device(ok, "nccl") == torch.device("cuda", 7)
    # launcher-isolated: one visible GPU per process, any local size
    monkeypatch.setattr(torch.cuda, "device_count", lambda: 1)
    iso = E.discover({"WORLD_SIZE": "8", "RANK": "5", "LOCAL_RANK": "5", "LOCAL_WORLD_SIZE": "8"}, ndev=1)
    assert B._bind_local_device(iso, "nccl") == torch.device("cuda", 0)


def test_cu_split_mask_and_slurm_nodeid_guard(monkeypatch):
    from multidisttorch_amd.runtime.env import apply_cu_split, cu_split_mask, local_size_from_env

    assert cu_split_mask(0, 2) == "0:0-127" and cu_split_mask(1, 2) == "0:128-255"
    assert cu_split_mask(3, 4) == "0:192-255"
    with pytest.raises(ValueError):
        cu_split_mask(2, 2)
    env = {"MDT_CU_SPLIT": "1", "LOCAL_RANK": "1", "LOCAL_WORLD_SIZE": "4", "RANK": "1", "WORLD_SIZE": "4"}
    monkeypatch.setenv("HSA_CU_MASK", "unset")  # recorded, so the undo removes what apply_cu_split writes
    assert apply_cu_split(env) == "0:64-127"
    assert apply_cu_split({"LOCAL_RANK": "1", "LOCAL_WORLD_SIZE": "4"}) is None  # off by default
    # a malformed SLURM_NODEID no longer raises: the same-count rule applies
    assert local_size_from_env({"SLURM_TASKS_PER_NODE": "4(x2)", "SLURM_NODEID": "x"}) == 4
    assert local_size_from_env({"SLURM_TASKS_PER_NODE": "4,2", "SLURM_NODEID": "bad"}) is None
