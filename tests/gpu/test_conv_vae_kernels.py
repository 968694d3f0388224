"""Conv-VAE bf16 MFMA kernels vs the fp32 torch reference network (GPU).

These tests exercise the LAYER-BY-LAYER path (conv_igemm / conv_jobs /
conv_thin kernels), which 128x128 images use and 28x28 images fall back to
with MDT_CONV_F28=0; the fused 28x28 step has its own tests
(test_conv28_fused.py)."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.fixture(autouse=True)
def _layer_path(monkeypatch):
    monkeypatch.setenv("MDT_CONV_F28", "0")


def _wt_layers(tr):
    """Transposed weight copies of every layer that has a backward-data GEMM
    (the first layer's copy is never read, so the training step skips it)."""
    return {l.name: tr._wt(l).clone() for l in tr.spec[1:]}


def _rel(a, b):
    a, b = a.detach().double(), b.detach().double()
    return float((a - b).norm() / (b.norm() + 1e-12))


@pytest.mark.parametrize("M", [64, 37])
def test_conv_vae_fwd_bwd_matches_torch(M, native_ext):
    from multidisttorch_amd.models.conv_vae import ConvVaeTrainer, TorchConvVAE

    dev = torch.device("cuda")
    tr = ConvVaeTrainer(batch_size=64, image=28, device=dev, backend="hip", seed=1, use_graphs=False)
    X = torch.rand(256, 784, device=dev)
    idx = torch.randperm(256, device=dev).to(torch.int32)
    tr.bind_train_data(X, idx)
    tr.set_cursor(0, 4)
    st = tr.state
    C = tr.C
    C.step_begin(st.train_state, st.hparams)
    C.gather_rows(X, tr._data[1], st.train_state, tr.B, M, tr.xb)
    tr._forward_hip(M, st.train_state, 0, want_recon=True)
    tr._backward_hip(M)
    tr._finalize_grads(M, False)
    torch.cuda.synchronize()
    # reference: same weights, same eps, fp32 autograd
    ref = TorchConvVAE(tr.spec, 28, 1, tr.Z).to(dev)
    ref.from_arena(tr.named_parameters())
    x = tr.xb[:M].clone()
    torch.testing.assert_close(x, X[idx[:M].long()])
    eps = tr.eps[:M].clone()
    loss, t, mu, lv = ref.loss(x, eps)
    loss.backward()
    assert _rel(tr.mulv[:M], torch.cat([mu, lv], 1)) < 2e-2
    # the last layer is fused with the BCE: compare the reconstruction
    recon = tr.recon[: M * 784].view(M, 28, 28, 1).permute(0, 3, 1, 2)
    assert _rel(recon, torch.sigmoid(t)) < 1e-2
    g_ref = ref.grads_to_arena()
    g = tr.named_grads()
    # bf16 activations/gradients through six chained GEMM layers: check the
    # direction tightly (cosine) and the magnitude at bf16-chain tolerance
    errs = {}
    for name in g_ref:
        a, b = g[name].double().flatten(), g_ref[name].double().flatten()
        cos = float(a @ b / (a.norm() * b.norm() + 1e-30))
        errs[name] = (round(_rel(a, b), 4), round(cos, 5))
    print("conv grad rel-err / cosine:", errs)
    for name, (err, cos) in errs.items():
        assert err < 0.12 and cos > 0.993, (name, err, cos)


def test_conv_vae_training_and_graphs(native_ext):
    from multidisttorch_amd.models.conv_vae import ConvVaeTrainer

    dev = torch.device("cuda")
    from multidisttorch_amd.data.datasets import synthetic_images

    X = synthetic_images(2048, device=dev)
    idx = torch.arange(2048, device=dev, dtype=torch.int32)
    res = []
    for graphs in (False, True):
        tr = ConvVaeTrainer(batch_size=128, image=28, device=dev, backend="hip", seed=3, use_graphs=graphs,
                            graph_steps=4)
        tr.bind_train_data(X, idx)
        tr.set_cursor(0, 16)
        tr.train_steps(40)
        torch.cuda.synchronize()
        h = tr.loss_history()[:40]
        assert np.all(np.isfinite(h)) and h[-5:].mean() < 0.7 * h[:5].mean(), h
        res.append(h)
    # every reduction (m-split weight-gradient slabs, bias column sums) has a
    # fixed order, so graph replay and eager launches agree bitwise
    np.testing.assert_array_equal(res[0], res[1])
    total, first = tr.evaluate(X, torch.arange(300, device=dev, dtype=torch.int32))
    assert np.isfinite(total) and first.shape == (128, 784)
    out = tr.decode(torch.randn(10, tr.Z, device=dev))
    assert out.shape == (10, 784)


def test_conv_vae_128_step(native_ext):
    from multidisttorch_amd.models.conv_vae import ConvVaeTrainer

    dev = torch.device("cuda")
    X = torch.rand(256, 128 * 128, device=dev)
    tr = ConvVaeTrainer(batch_size=32, image=128, device=dev, backend="hip", seed=0, use_graphs=False)
    tr.bind_train_data(X, torch.arange(256, device=dev, dtype=torch.int32))
    tr.set_cursor(0, 8)
    tr.train_steps(3)
    torch.cuda.synchronize()
    h = tr.loss_history()[:3]
    assert np.all(np.isfinite(h))


def test_conv_vae_transposed_weights_are_parity_ordered(native_ext):
    from multidisttorch_amd.models.conv_vae import ConvVaeTrainer, _w_shape
    from multidisttorch_amd.ops.conv_layout import parity_transpose

    dev = torch.device("cuda")
    tr = ConvVaeTrainer(batch_size=16, image=28, device=dev, backend="hip", seed=1, use_graphs=False)
    for l in tr.spec:
        w = tr._w(l).view(_w_shape(l))
        torch.testing.assert_close(tr._wt(l), parity_transpose(w, l.s), rtol=0, atol=0)


@pytest.mark.parametrize("image,batch", [(28, 128), (128, 16)])
def test_two_stream_backward_is_bitwise_sequential(image, batch, native_ext):
    """The two-stream backward (weight gradients, finalize+Adam and transposes
    on a side stream, captured as parallel graph branches) runs the same
    kernels with the same reduction order: losses and weights match the
    single-stream path bit for bit, eager and graph-replayed."""
    from multidisttorch_amd.models.conv_vae import ConvVaeTrainer

    dev = torch.device("cuda")
    D = image * image
    X = torch.rand(8 * batch, D, device=dev)
    idx = torch.arange(8 * batch, device=dev, dtype=torch.int32)
    out = []
    for overlap, graphs in ((False, False), (True, False), (True, True)):
        tr = ConvVaeTrainer(batch_size=batch, image=image, device=dev, backend="hip", seed=5,
                            use_graphs=graphs, graph_steps=3)
        tr.overlap = overlap
        tr.bind_train_data(X, idx)
        tr.set_cursor(0, 8)
        tr.train_steps(7)
        torch.cuda.synchronize()
        out.append((tr.loss_history()[:7].copy(), tr.params.clone(), _wt_layers(tr)))
    for h, p, wt in out[1:]:
        np.testing.assert_array_equal(h, out[0][0])
        assert torch.equal(p, out[0][1])
        bad = [n for n in wt if not torch.equal(wt[n], out[0][2][n])]
        assert not bad, bad


@pytest.mark.parametrize("image,batch", [(28, 128), (28, 64), (128, 32)])
def test_fused_job_launches_are_bitwise_unfused(image, batch, native_ext):
    """Horizontally fused backward launches (conv_jobs.hip: weight gradient ||
    backward-data || bias column sums || loss in one kernel) run the same
    device bodies as the stand-alone kernels: identical losses, weights and
    transposed weights, eager and graph-replayed; and the fused kernels are
    actually used for these model shapes."""
    from multidisttorch_amd.models.conv_vae import ConvVaeTrainer

    dev = torch.device("cuda")
    D = image * image
    X = torch.rand(6 * batch, D, device=dev)
    idx = torch.arange(6 * batch, device=dev, dtype=torch.int32)
    out = []
    for fuse, graphs in ((False, False), (True, False), (True, True)):
        tr = ConvVaeTrainer(batch_size=batch, image=image, device=dev, backend="hip", seed=9,
                            use_graphs=graphs, graph_steps=2)
        tr.fuse_jobs = fuse
        tr.bind_train_data(X, idx)
        tr.set_cursor(0, 6)
        tr.train_steps(5)
        torch.cuda.synchronize()
        if fuse:
            assert tr._fused_launches >= len(tr.spec) - 1, tr._fused_launches
        else:
            assert tr._fused_launches == 0
        out.append((tr.loss_history()[:5].copy(), tr.params.clone(), _wt_layers(tr), tr.read_state()))
    for h, p, wt, st in out[1:]:
        np.testing.assert_array_equal(h, out[0][0])
        assert torch.equal(p, out[0][1])
        bad = [n for n in wt if not torch.equal(wt[n], out[0][2][n])]
        assert not bad, bad
        assert st["cursor"] == out[0][3]["cursor"] and st["step"] == out[0][3]["step"]


def test_encoder_head_prologue_matches_combine_launch(native_ext, monkeypatch):
    """28x28: enc2 runs split-K and its combine (+bias, ReLU) is folded into the
    encoder head's A staging (APro). Same training as with the separate combine
    launch (MDT_CONV_APRO=0), up to summation order; enc2's activations written
    by the head kernel equal the combined ones."""
    from multidisttorch_amd.data.datasets import synthetic_images
    from multidisttorch_amd.models.conv_vae import ConvVaeTrainer

    dev = torch.device("cuda")
    X = synthetic_images(1024, device=dev)
    idx = torch.arange(1024, device=dev, dtype=torch.int32)
    res, acts = [], []
    for flag in ("0", "1"):
        monkeypatch.setenv("MDT_CONV_APRO", flag)
        tr = ConvVaeTrainer(batch_size=128, image=28, device=dev, backend="hip", seed=11, use_graphs=False)
        tr.bind_train_data(X, idx)
        tr.set_cursor(0, 8)
        p = tr._plan(128)
        assert (p["ws_a"] is not None) == (flag == "1")
        tr.train_steps(6)
        torch.cuda.synchronize()
        res.append(tr.loss_history()[:6].copy())
        acts.append(tr.acts["enc2"].float().clone())
    np.testing.assert_allclose(res[0], res[1], rtol=2e-3)
    d = (acts[0] - acts[1]).abs().max().item()
    assert d <= 0.02 * acts[0].abs().max().item(), d


@pytest.mark.parametrize("image,batch", [(28, 128), (128, 32)])
def test_one_launch_optimizer_tail_is_bitwise_two_launch(image, batch, native_ext):
    """conv_jobs.hip::tail_k: the last first-layer weight-gradient block (device
    ticket) finalizes the first layer while the other blocks finalize the rest,
    and the transposed copies move into the next step's first launch. Same
    losses, master weights, Adam moments and transposed weights as the
    two-launch tail (MDT_CONV_TAIL1=0 path), eager and graph-replayed; the
    ticket is back at zero after every launch."""
    from multidisttorch_amd.models.conv_vae import ConvVaeTrainer

    dev = torch.device("cuda")
    D = image * image
    X = torch.rand(6 * batch, D, device=dev)
    idx = torch.arange(6 * batch, device=dev, dtype=torch.int32)
    out = []
    for tail1, graphs in ((False, False), (True, False), (True, True)):
        tr = ConvVaeTrainer(batch_size=batch, image=image, device=dev, backend="hip", seed=11,
                            use_graphs=graphs, graph_steps=2)
        tr.tail1 = tail1
        tr.spread_fin = False
        assert tr._tail1_active() == tail1
        tr.bind_train_data(X, idx)
        tr.set_cursor(0, 6)
        tr.train_steps(5)
        torch.cuda.synchronize()
        assert tr._ticket.tolist() == [0, 0, 0]
        out.append((tr.loss_history()[:5].copy(), tr.params.clone(), tr.exp_avg.clone(), tr.exp_avg_sq.clone(),
                    _wt_layers(tr)))
    for h, p, m, v, wt in out[1:]:
        np.testing.assert_array_equal(h, out[0][0])
        assert torch.equal(p, out[0][1]) and torch.equal(m, out[0][2]) and torch.equal(v, out[0][3])
        bad = [n for n in wt if not torch.equal(wt[n], out[0][4][n])]
        assert not bad, bad


@pytest.mark.parametrize("image,batch", [(28, 128), (128, 32)])
def test_deferred_transposes_are_bitwise_two_launch(image, batch, native_ext):
    """MDT_CONV_DEFER_WT: the tail's second launch finalizes only the first
    layer and the transposed copies are written by the next step's first launch
    (=1) or by the first decoder GEMM's launch (=2), and at the end of
    train_steps. Same losses, master weights, Adam moments
    and transposed weights as the default tail, eager and graph-replayed."""
    from multidisttorch_amd.models.conv_vae import ConvVaeTrainer

    dev = torch.device("cuda")
    D = image * image
    X = torch.rand(6 * batch, D, device=dev)
    idx = torch.arange(6 * batch, device=dev, dtype=torch.int32)
    out = []
    for defer, in_dec, graphs in ((False, False, False), (True, False, False), (True, False, True),
                                  (True, True, False), (True, True, True)):
        tr = ConvVaeTrainer(batch_size=batch, image=image, device=dev, backend="hip", seed=11,
                            use_graphs=graphs, graph_steps=2)
        tr.tail1 = False
        tr.defer_wt = defer
        tr.wt_in_dec = in_dec
        tr.spread_fin = False
        assert tr._wt_deferred() == defer
        tr.bind_train_data(X, idx)
        tr.set_cursor(0, 6)
        tr.train_steps(5)
        torch.cuda.synchronize()
        out.append((tr.loss_history()[:5].copy(), tr.params.clone(), tr.exp_avg.clone(), tr.exp_avg_sq.clone(),
                    _wt_layers(tr)))
    for h, p, m, v, wt in out[1:]:
        np.testing.assert_array_equal(h, out[0][0])
        assert torch.equal(p, out[0][1]) and torch.equal(m, out[0][2]) and torch.equal(v, out[0][3])
        bad = [n for n in wt if not torch.equal(wt[n], out[0][4][n])]
        assert not bad, bad


@pytest.mark.parametrize("image,batch", [(28, 128), (128, 32)])
def test_spread_finalize_is_bitwise_tail_finalize(image, batch, native_ext):
    """Finalize+Adam of layer j as the third job of the backward launch after
    layer j's gradients completed (MDT_CONV_SPREAD_FIN, default) gives the same
    losses, weights, moments and transposed weights as finalizing every layer
    in the optimizer tail, eager and graph-replayed, with and without the
    one-launch tail."""
    from multidisttorch_amd.models.conv_vae import ConvVaeTrainer

    dev = torch.device("cuda")
    D = image * image
    X = torch.rand(6 * batch, D, device=dev)
    idx = torch.arange(6 * batch, device=dev, dtype=torch.int32)
    out = []
    for spread, tail1, graphs in ((False, False, False), (True, False, False), (True, False, True),
                                  (True, True, True)):
        tr = ConvVaeTrainer(batch_size=batch, image=image, device=dev, backend="hip", seed=13,
                            use_graphs=graphs, graph_steps=2)
        tr.spread_fin, tr.tail1 = spread, tail1
        tr.bind_train_data(X, idx)
        tr.set_cursor(0, 6)
        tr.train_steps(5)
        torch.cuda.synchronize()
        out.append((tr.loss_history()[:5].copy(), tr.params.clone(), tr.exp_avg.clone(), tr.exp_avg_sq.clone(),
                    _wt_layers(tr)))
    for h, p, m, v, wt in out[1:]:
        np.testing.assert_array_equal(h, out[0][0])
        assert torch.equal(p, out[0][1]) and torch.equal(m, out[0][2]) and torch.equal(v, out[0][3])
        bad = [n for n in wt if not torch.equal(wt[n], out[0][4][n])]
        assert not bad, bad
