"""Host-side DDP policy of round 4 (parallel/ddp.py, models/conv_vae.py):
when the first-ready bucket is issued early, which reducer kind a group gets,
and the conv trainer's resolution of MDT_DDP_OVERLAP."""
import pytest

from multidisttorch_amd.parallel.ddp import overlap_pays


def test_overlap_pays_thresholds():
    # 28x28 decoder bucket: 133,248 f32 gradients = 0.53 MB -> 3.5 us on one 153 GB/s link
    dec28 = 4 * 133248
    assert not overlap_pays(dec28, 6.0)       # fused jobs: the split costs 6 us
    assert not overlap_pays(dec28, 31.0)      # RCCL on its own stream: 31 us
    # a 16 MB bucket (~110 us on one link) hides behind both
    assert overlap_pays(16 << 20, 6.0) and overlap_pays(16 << 20, 31.0)
    # faster links shrink the transfer
    assert overlap_pays(2 << 20, 6.0, link_gbps=153.0) and not overlap_pays(2 << 20, 6.0, link_gbps=1000.0)


def test_conv_trainer_overlap_resolution(monkeypatch):
    from multidisttorch_amd.models.conv_vae import ConvVaeTrainer

    monkeypatch.delenv("MDT_DDP_OVERLAP", raising=False)
    tr = ConvVaeTrainer(batch_size=8, image=28, backend="torch", seed=0)
    assert tr.ddp_overlap is None  # auto
    assert tr._overlap28(fused=True) is False and tr._overlap28(fused=False) is False
    monkeypatch.setenv("MDT_DDP_OVERLAP", "1")
    tr = ConvVaeTrainer(batch_size=8, image=28, backend="torch", seed=0)
    assert tr._overlap28(fused=True) is True
    monkeypatch.setenv("MDT_DDP_OVERLAP", "0")
    tr = ConvVaeTrainer(batch_size=8, image=28, backend="torch", seed=0)
    assert tr._overlap28(fused=False) is False


def test_reducer_kind_env_override(monkeypatch):
    import torch

    from multidisttorch_amd.parallel import ddp

    monkeypatch.setenv("MDT_REDUCER", "p2p2")
    assert ddp.reducer_kind(None, torch.zeros(4)) == "p2p2"


def test_health_error_is_none_on_the_cpu_backend():
    from multidisttorch_amd.models.conv_vae import ConvVaeTrainer

    tr = ConvVaeTrainer(batch_size=4, image=28, backend="torch", seed=0)
    assert tr.health_error() is None


def test_runner_fails_a_trial_on_reported_corruption():
    from multidisttorch_amd.hpo.runner import _check_health
    from multidisttorch_amd.runtime.faults import TrialCorrupted

    class Fake:
        def health_error(self):
            return "fused 28x28 step: a paired-workgroup exchange timed out (f28_err=1)"

    with pytest.raises(TrialCorrupted, match="exchange timed out"):
        _check_health(Fake())
    _check_health(object())  # trainers without the check pass


def test_mlp_trainer_overlap_resolution(monkeypatch):
    """MLP trainer: auto keeps both buckets inline (the 1.26 MB fc4 bucket
    moves in ~8 us over one link, less than a side-stream split costs); an
    explicit MDT_DDP_OVERLAP wins; one bucket never splits."""
    from multidisttorch_amd.models.mlp_trainer import MlpVaeTrainer

    class FakeReducer:
        def __init__(self, n):
            self.n = n

        def num_buckets(self):
            return self.n

    monkeypatch.delenv("MDT_DDP_OVERLAP", raising=False)
    tr = MlpVaeTrainer(batch_size=8, backend="torch", seed=0)
    assert tr.ddp_overlap is None and tr._overlap() is False  # no reducer
    tr.reducer = FakeReducer(2)
    assert tr._overlap() is False
    tr.ddp_overlap = True
    assert tr._overlap() is True
    tr.reducer = FakeReducer(1)
    assert tr._overlap() is False
    monkeypatch.setenv("MDT_DDP_OVERLAP", "1")
    assert MlpVaeTrainer(batch_size=8, backend="torch", seed=0).ddp_overlap is True


def test_default_reducer_follows_trainer_capability(monkeypatch):
    """Intra-node multi-rank RCCL groups: the fused xGMI jobs for trainers that
    host them (conv), RCCL inline for the MLP trainer (1.16x vs 1.39x for the
    standalone push kernel, profiles/r4_ddp_fused/ddp_structure_mlp.json)."""
    from multidisttorch_amd.parallel import ddp

    class FlatCuda:
        is_cuda = True

    monkeypatch.delenv("MDT_REDUCER", raising=False)
    monkeypatch.setattr(ddp.native, "available", lambda: True)
    monkeypatch.setattr(ddp.dist, "get_backend", lambda pg=None: "nccl")
    monkeypatch.setattr(ddp.dist, "get_world_size", lambda pg=None: 2)
    monkeypatch.setattr(ddp, "group_on_one_node", lambda pg: True)
    assert ddp.reducer_kind(object(), FlatCuda()) == "xgmi"
    assert ddp.reducer_kind(object(), FlatCuda(), comm_jobs=True) == "xgmi"
    assert ddp.reducer_kind(object(), FlatCuda(), comm_jobs=False) == "rccl"
    monkeypatch.setattr(ddp, "group_on_one_node", lambda pg: False)
    assert ddp.reducer_kind(object(), FlatCuda(), comm_jobs=True) == "rccl"


def test_trainer_comm_job_capability():
    from multidisttorch_amd.models.conv_vae import ConvVaeTrainer
    from multidisttorch_amd.models.mlp_trainer import MlpVaeTrainer

    assert ConvVaeTrainer(batch_size=4, image=28, backend="torch", seed=0).comm_jobs is False  # no HIP launches
    assert getattr(MlpVaeTrainer(batch_size=4, backend="torch", seed=0), "comm_jobs", False) is False


def test_production_paths_never_split_the_comm_tail():
    """The push/reduce split with a host barrier between them
    (``comm_split_tail``) is a test-only rehearsal form: no production module,
    the bench or the entry point may turn it on; the trainer defaults it off."""
    import ast
    import os

    from multidisttorch_amd.models.conv_vae import ConvVaeTrainer

    root = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    files = [os.path.join(root, "bench.py"), os.path.join(root, "vae-hpo.py")]
    for d, _, fs in os.walk(os.path.join(root, "multidisttorch_amd")):
        files += [os.path.join(d, f) for f in fs if f.endswith(".py")]
    offenders = []
    for path in files:
        tree = ast.parse(open(path).read())
        for node in ast.walk(tree):
            targets = node.targets if isinstance(node, ast.Assign) else (
                [node.target] if isinstance(node, (ast.AugAssign, ast.AnnAssign)) else [])
            for t in targets:
                if isinstance(t, ast.Attribute) and t.attr in ("comm_split_tail", "comm_phase_hook"):
                    v = node.value
                    if not (isinstance(v, ast.Constant) and v.value in (False, None)):
                        offenders.append(f"{path}:{node.lineno}")
            if isinstance(node, ast.Call) and getattr(node.func, "id", "") == "setattr":
                a = node.args
                if len(a) >= 2 and isinstance(a[1], ast.Constant) and a[1].value == "comm_split_tail":
                    offenders.append(f"{path}:{node.lineno}")
    assert not offenders, offenders
    tr = ConvVaeTrainer(batch_size=4, image=28, backend="torch", seed=0)
    assert tr.comm_split_tail is False and tr.comm_phase_hook is None
