"""Conv-VAE spec / layout / torch backend on CPU."""
import math

import numpy as np
import torch

from multidisttorch_amd.models.conv_vae import ConvVaeTrainer, TorchConvVAE, conv_layout, conv_vae_spec


def test_spec_shapes():
    s = conv_vae_spec(28, 1, 32)
    assert [l.name for l in s] == ["enc1", "enc2", "enc_head", "dec_fc", "dec1", "dec2"]
    assert s[2].cin == 64 * 7 * 7 and s[2].cout == 64 and s[-1].out_hw == 28
    s128 = conv_vae_spec(128, 1, 64)
    assert s128[4].cin == 256 * 8 * 8 and s128[-1].out_hw == 128
    lay, n = conv_layout(s128)
    assert all(o % 64 == 0 for _, o, _ in lay)


def test_arena_roundtrip_and_forward_shape():
    spec = conv_vae_spec(28, 1, 32)
    m = TorchConvVAE(spec, 28, 1, 32)
    a = m.to_arena()
    m2 = TorchConvVAE(spec, 28, 1, 32)
    m2.from_arena(a)
    for (k1, v1), (k2, v2) in zip(m.state_dict().items(), m2.state_dict().items()):
        assert torch.equal(v1, v2)
    x = torch.rand(3, 784)
    t, mu, lv = m(x, torch.zeros(3, 32))
    assert t.shape == (3, 1, 28, 28) and mu.shape == (3, 32)


def test_torch_backend_trains():
    tr = ConvVaeTrainer(batch_size=32, image=28, backend="torch", seed=0)
    g = torch.Generator().manual_seed(0)
    yy, xx = torch.meshgrid(torch.linspace(-1, 1, 28), torch.linspace(-1, 1, 28), indexing="ij")
    c = torch.rand(256, 2, generator=g) - 0.5
    X = torch.exp(-((xx[None] - c[:, 0, None, None]) ** 2 + (yy[None] - c[:, 1, None, None]) ** 2) / 0.1).reshape(256, 784)
    tr.bind_train_data(X.float().contiguous(), torch.arange(256, dtype=torch.int32))
    tr.set_cursor(0, 8)
    tr.train_steps(16)
    h = tr.loss_history()[:16]
    assert np.all(np.isfinite(h)) and h[-3:].mean() < h[:3].mean()
    total, first = tr.evaluate(X.float(), torch.arange(40, dtype=torch.int32))
    assert first.shape == (32, 784) and np.isfinite(total)
    assert tr.decode(torch.randn(4, 32)).shape == (4, 784)


def test_conv_bucket_bounds_fall_on_layer_starts():
    from multidisttorch_amd.models.conv_vae import ConvVaeTrainer

    tr = ConvVaeTrainer(batch_size=4, image=128, z=64, backend="torch", seed=0)
    starts = {b for _, b, _ in tr.layer_ranges()}
    assert tr.bucket_bounds(None) == [0, tr.split, tr.numel]
    assert tr.bucket_bounds(0) == [0, tr.numel]
    for mb in (0.5, 2, 8):
        b = tr.bucket_bounds(mb)
        assert b[0] == 0 and b[-1] == tr.numel and b == sorted(b)
        assert all(x in starts for x in b[:-1])
    assert len(tr.bucket_bounds(0.5)) > len(tr.bucket_bounds(8)) >= 2


def test_merged_tail_finalizes_every_28x28_layer_once():
    # MDT_F28_FIN_MERGE's job table (ConvVaeTrainer._merged_pack28) has one
    # finalize job per layer of the 28x28 model, released by that layer's
    # weight-gradient job: the order list must name each layer exactly once
    names = [l.name for l in conv_vae_spec(28)]
    order = ConvVaeTrainer._FIN_ORDER28
    assert sorted(order) == sorted(names) and len(order) == len(set(order))
