"""MlpVaeTrainer on the torch (CPU) backend + checkpoint round trip."""
import os

import numpy as np
import torch

from multidisttorch_amd.ckpt import checkpoint as ckpt
from multidisttorch_amd.hpo.trial import TrialSpec
from multidisttorch_amd.models.mlp_trainer import MlpVaeTrainer


def _trainer(seed=0, **kw):
    tr = MlpVaeTrainer(batch_size=32, D=64, H=32, Z=4, backend="torch", seed=seed, **kw)
    X = torch.rand(320, 64, generator=torch.Generator().manual_seed(4))
    tr.bind_train_data(X, torch.arange(320, dtype=torch.int32))
    tr.set_cursor(0, 10)
    return tr, X


def test_training_reduces_loss_and_state_advances():
    tr, X = _trainer()
    tr.train_steps(40)
    st = tr.read_state()
    assert st["step"] == 40 and st["cursor"] == 0
    h = tr.loss_history()[:40]
    assert np.all(np.isfinite(h)) and h[-5:].mean() < h[:5].mean()


def test_tail_batch_and_eval_decode():
    tr, X = _trainer()
    tr.set_cursor(0, 2)
    tr.train_steps(1, 32)
    tr.train_steps(1, 7)
    assert tr.step_count == 2
    total, first = tr.evaluate(X, torch.arange(70, dtype=torch.int32))
    assert first.shape == (32, 64) and np.isfinite(total)
    assert tr.read_state(eval=True)["epoch_count"] == 3
    out = tr.decode(torch.randn(5, 4))
    assert out.shape == (5, 64) and float(out.min()) >= 0 and float(out.max()) <= 1


def test_hparams_seed_determinism():
    a, _ = _trainer(seed=3)
    b, _ = _trainer(seed=3)
    a.train_steps(3)
    b.train_steps(3)
    assert torch.equal(a.params, b.params)
    c, _ = _trainer(seed=4)
    assert not torch.equal(a.params, c.params)


def test_checkpoint_roundtrip(tmp_path):
    tr, X = _trainer(seed=1)
    tr.train_steps(5)
    spec = TrialSpec(group_id=2, epochs=3, lr=1e-3, beta=1.0, seed=1)
    path = ckpt.save_trial(str(tmp_path), tr, spec, epoch=1)
    assert os.path.basename(path) == "epoch-1.pt"
    # loads with the safe loader
    raw = torch.load(path, weights_only=True)
    assert raw["progress"] == {"epoch": 1, "step": 5}
    tr2, _ = _trainer(seed=99)
    prog = ckpt.load_latest(str(tmp_path), 2, tr2)
    assert prog["epoch"] == 1 and tr2.step_count == 5
    assert torch.equal(tr2.params, tr.params) and torch.equal(tr2.exp_avg_sq, tr.exp_avg_sq)
    # resumed training continues identically (same seed / Philox counters)
    tr2.seed = tr.seed
    tr.set_cursor(0, 10)
    tr2.set_cursor(0, 10)
    tr.train_steps(3)
    tr2.train_steps(3)
    torch.testing.assert_close(tr.params, tr2.params, rtol=0, atol=0)
    assert ckpt.load_latest(str(tmp_path), 7, tr2) is None


def test_state_dict_loads_into_reference_module():
    from multidisttorch_amd.models.mlp_vae import VAE

    tr, _ = _trainer()
    m = VAE(64, 32, 4)
    m.load_state_dict(tr.state_dict())


def _conv_trainer(seed=0, image=28):
    from multidisttorch_amd.models.conv_vae import ConvVaeTrainer

    tr = ConvVaeTrainer(batch_size=16, image=image, z=32 if image == 28 else 64, backend="torch", seed=seed)
    X = torch.rand(64, image * image, generator=torch.Generator().manual_seed(5))
    tr.bind_train_data(X, torch.arange(64, dtype=torch.int32))
    tr.set_cursor(0, 4)
    return tr


def test_conv_checkpoint_roundtrip(tmp_path):
    """Conv-VAE checkpoints (int(trainer.H) crashed for conv): the
    arch record replaces the MLP-only dims, loads with weights_only=True and
    refuses a trainer of another architecture."""
    import pytest

    tr = _conv_trainer(seed=1)
    tr.train_steps(3)
    spec = TrialSpec(group_id=0, epochs=2, lr=1e-3, beta=1.0, seed=1)
    path = ckpt.save_trial(str(tmp_path), tr, spec, epoch=1)
    raw = torch.load(path, weights_only=True)
    assert raw["arch"]["kind"] == "conv" and raw["arch"]["image"] == 28 and raw["progress"]["step"] == 3
    tr2 = _conv_trainer(seed=9)
    prog = ckpt.load_latest(str(tmp_path), 0, tr2)
    assert prog["epoch"] == 1 and tr2.step_count == 3
    assert torch.equal(tr2.params, tr.params) and torch.equal(tr2.exp_avg, tr.exp_avg)
    tr2.seed = tr.seed
    tr.set_cursor(0, 4)
    tr2.set_cursor(0, 4)
    tr.train_steps(2)
    tr2.train_steps(2)
    torch.testing.assert_close(tr.params, tr2.params, rtol=0, atol=0)
    mlp, _ = _trainer()
    with pytest.raises(ValueError, match="conv model"):
        ckpt.load_latest(str(tmp_path), 0, mlp)


def test_loss_ring_read_before_wrap():
    """Epochs longer than the 4096-entry loss ring are read per chunk
    (ADVICE r1): the logged losses are those of their own steps."""
    from multidisttorch_amd.hpo import runner

    tr = MlpVaeTrainer(batch_size=1, D=8, H=4, Z=2, backend="torch", seed=0)
    n = 4096 + 300
    X = torch.rand(n, 8, generator=torch.Generator().manual_seed(1))
    tr.bind_train_data(X, torch.arange(n, dtype=torch.int32))
    opts = runner.RunOptions(batch_size=1, log_interval=1000)
    step0, early = runner._launch_epoch(tr, 1, n, opts)
    assert step0 == 0 and sorted(early) == [0, 1000, 2000, 3000, 4000]
    # entry 0 was overwritten by step 4096 in the ring; the early read kept step 0's loss
    assert early[0] != float(tr.loss_history()[0])
