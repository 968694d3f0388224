"""Fused 28x28 conv-VAE step (csrc/kernels/conv28_fused.hip) on one MI355X.

The numerical oracle is a float64 torch re-implementation of the SAME
computation with bf16 rounding applied at exactly the points where the
kernels store bf16 (activations a1/a2/d0/d1, z, the masked gradients
gd1/gd0/ga2/ga1, d[mu|lv] for the head weight gradient, the f32 input and
dlogits as the wgrad kernels' bf16 operands) and the bf16 weight copies the
GEMMs read. What remains between kernel and oracle is f32 accumulation order,
so every gradient tensor is asserted to 1e-2 relative error (measured <= 4e-3) (the layer-path
test accepts 0.12 against a plain fp32 reference). Then: eager == graph
replay bitwise, tail batches, the fused Adam against torch.optim.Adam, and
training parity with the layer-by-layer path.
"""
import math

import numpy as np
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu


def _bf(t):
    return t.to(torch.bfloat16).to(torch.float64)


def _rel(a, b):
    a, b = a.detach().double().flatten(), b.detach().double().flatten()
    return float((a - b).norm() / (b.norm() + 1e-30))


def _trainer(B=128, seed=1, **kw):
    from multidisttorch_amd.models.conv_vae import ConvVaeTrainer

    tr = ConvVaeTrainer(batch_size=B, image=28, device=torch.device("cuda"), backend="hip", seed=seed, **kw)
    assert tr.f28
    return tr


def _emulated_reference(tr, x32, eps, beta=1.0):
    """float64 forward + backward of the conv-VAE with the fused step's bf16
    rounding points. Returns (loss, {arena name: gradient})."""
    P = {k: v.detach().double() for k, v in tr.named_parameters().items()}
    W1 = P["enc1.weight"].permute(0, 3, 1, 2)            # [32,1,4,4] f32 master
    W2 = _bf(P["enc2.weight"]).permute(0, 3, 1, 2)       # [64,32,4,4] bf16 copy
    Wh = _bf(P["enc_head.weight"]).reshape(64, 3136)
    Wd = _bf(P["dec_fc.weight"]).reshape(3136, 32)
    W3 = _bf(P["dec1.weight"]).permute(0, 3, 1, 2)       # convT [in 64, out 32, 4, 4]
    W4 = P["dec2.weight"].permute(0, 3, 1, 2)            # convT [32, 1, 4, 4] f32 master
    b = {k.split(".")[0]: v for k, v in P.items() if k.endswith(".bias")}
    M = x32.shape[0]
    x = x32.double().view(M, 1, 28, 28)
    nhwc = lambda t: t.permute(0, 2, 3, 1).reshape(M, -1)
    nchw = lambda t, c, hw: t.view(M, hw, hw, c).permute(0, 3, 1, 2)

    def vjp(fn, inp, wt, gout):
        inp = inp.detach().requires_grad_()
        wt = wt.detach().requires_grad_()
        out = fn(inp, wt)
        return torch.autograd.grad(out, (inp, wt), gout)

    conv = lambda i, w: F.conv2d(i, w, stride=2, padding=1)
    tconv = lambda i, w: F.conv_transpose2d(i, w, stride=2, padding=1)
    # ---- forward
    a1 = _bf(F.relu(conv(x, W1) + b["enc1"].view(1, -1, 1, 1)))
    a2 = _bf(F.relu(conv(a1, W2) + b["enc2"].view(1, -1, 1, 1)))
    a2f = nhwc(a2)
    h = a2f @ Wh.t() + b["enc_head"]
    mu, lv = h[:, :32], h[:, 32:]
    e = eps.double()
    sd = torch.exp(0.5 * lv)
    z = _bf(mu + e * sd)
    d0f = _bf(F.relu(z @ Wd.t() + b["dec_fc"]))
    d0 = nchw(d0f, 64, 7)
    d1 = _bf(F.relu(tconv(d0, W3) + b["dec1"].view(1, -1, 1, 1)))
    t = tconv(d1, W4) + b["dec2"].view(1, -1, 1, 1)
    sp = torch.clamp(t, min=0) + torch.log1p(torch.exp(-t.abs()))
    bce = (x * torch.clamp(sp - t, max=100.0) + (1 - x) * torch.clamp(sp, max=100.0)).sum()
    kld = -0.5 * torch.sum(1 + lv - mu.pow(2) - lv.exp())
    loss = bce + beta * kld
    # ---- backward (kernel order and rounding)
    g = {}
    dlog = torch.sigmoid(t) - x
    gi, _ = vjp(tconv, d1, W4, dlog)
    _, g["dec2.weight"] = vjp(tconv, d1, W4, _bf(dlog))
    g["dec2.bias"] = dlog.sum().view(1)
    gd1f = gi * (d1 > 0)
    gd1 = _bf(gd1f)
    g["dec1.bias"] = gd1f.sum((0, 2, 3))
    gi, g["dec1.weight"] = vjp(tconv, d0, W3, gd1)
    gd0f = nhwc(gi) * (d0f > 0)
    gd0 = _bf(gd0f)
    g["dec_fc.bias"] = gd0f.sum(0)
    dz = gd0 @ Wd
    g["dec_fc.weight"] = gd0.t() @ z
    dm = dz + beta * mu
    dl = 0.5 * dz * e * sd + 0.5 * beta * (sd * sd - 1)
    dmulv = torch.cat([dm, dl], 1)
    g["enc_head.bias"] = dmulv.sum(0)
    g["enc_head.weight"] = _bf(dmulv).t() @ a2f
    ga2f = (dmulv @ Wh) * (a2f > 0)
    ga2 = _bf(ga2f)
    g["enc2.bias"] = ga2f.view(M, 49, 64).sum((0, 1))
    gi, g["enc2.weight"] = vjp(conv, a1, W2, nchw(ga2, 64, 7))
    ga1f = gi * (a1 > 0)
    ga1 = _bf(ga1f)
    g["enc1.bias"] = ga1f.sum((0, 2, 3))
    _, g["enc1.weight"] = vjp(conv, _bf(x), W1, ga1)
    out = {}
    for k, v in g.items():
        if k.endswith(".weight") and v.dim() == 4:
            v = v.permute(0, 2, 3, 1)  # torch [O][I][kh][kw] (convT: [in][out]) -> arena [O][kh][kw][I]
        out[k] = v.reshape(tr.named_grads()[k].shape)
    return float(loss), out


@pytest.mark.parametrize("M,pair", [(128, True), (100, True), (128, False), (100, False)])
def test_f28_gradients_match_bf16_emulated_reference(M, pair, native_ext):
    from multidisttorch_amd.ops.philox import reparam_eps

    dev = torch.device("cuda")
    tr = _trainer(B=128, seed=2, use_graphs=False)
    tr.f28_pair = pair
    X = torch.rand(512, 784, generator=torch.Generator().manual_seed(7)).to(dev)
    idx = torch.randperm(512, generator=torch.Generator().manual_seed(8)).to(dev, torch.int32)
    tr.bind_train_data(X, idx)
    tr.set_cursor(0, 4)
    tr.f28_skip_adam = True
    p0 = tr.params.clone()
    tr.train_steps(1, M=M)
    torch.cuda.synchronize()
    assert torch.equal(tr.params, p0)  # no update: the gradients stay in `grads`
    assert tr.read_state()["step"] == 1 and tr.read_state()["cursor"] == 1
    x = X[idx[:M].long()]
    torch.testing.assert_close(tr.xb[:M], x, rtol=0, atol=0)
    eps = torch.from_numpy(reparam_eps(M, 32, tr.seed, tr.rng_stream, 0)).to(dev)
    torch.testing.assert_close(tr.eps[:M], eps, rtol=1e-5, atol=1e-5)  # Philox parity
    loss, gref = _emulated_reference(tr, x, eps)
    kloss = float(tr.loss_history()[0])
    assert abs(kloss - loss) / abs(loss) < 1e-4, (kloss, loss)
    errs = {n: _rel(tr.named_grads()[n], gref[n]) for n in gref}
    print("f28 grad rel-err vs bf16-emulated f64:", {k: round(v, 6) for k, v in errs.items()})
    bad = {n: e for n, e in errs.items() if not e < 1e-2}
    assert not bad, bad
    assert int(tr.f28_err.item()) == 0  # no exchange sweep timed out


def test_f28_eager_equals_graph_and_trains(native_ext):
    from multidisttorch_amd.data.datasets import synthetic_images

    dev = torch.device("cuda")
    X = synthetic_images(2048, device=dev)
    idx = torch.arange(2048, device=dev, dtype=torch.int32)
    res = []
    for graphs in (False, True):
        tr = _trainer(seed=3, use_graphs=graphs, graph_steps=4)
        tr.bind_train_data(X, idx)
        tr.set_cursor(0, 16)
        tr.train_steps(40)
        torch.cuda.synchronize()
        h = tr.loss_history()[:40]
        assert np.all(np.isfinite(h)) and h[-5:].mean() < 0.7 * h[:5].mean(), h
        res.append((h.copy(), tr.params.clone(), tr.exp_avg_sq.clone(), tr.read_state()))
    np.testing.assert_array_equal(res[0][0], res[1][0])
    assert torch.equal(res[0][1], res[1][1]) and torch.equal(res[0][2], res[1][2])
    assert res[0][3]["step"] == res[1][3]["step"] == 40 and res[0][3]["cursor"] == res[1][3]["cursor"] == 8
    # eval / decode (layer path kernels) see current transposed weights
    total, first = tr.evaluate(X, torch.arange(300, device=dev, dtype=torch.int32))
    assert np.isfinite(total) and first.shape == (128, 784)


@pytest.mark.parametrize("M", [128, 77])
def test_f28_merged_step_is_bitwise_two_launches(M, native_ext):
    """f28_step_k (forward + backward in one workgroup, masks / dlogits / dec1
    taps taken from LDS) computes exactly what the two-launch forward then
    backward computes: same losses, weights, Adam moments and every backward
    output, eager and graph-replayed."""
    from multidisttorch_amd.data.datasets import synthetic_images

    dev = torch.device("cuda")
    X = synthetic_images(1024, device=dev)
    idx = torch.arange(1024, device=dev, dtype=torch.int32)
    res = []
    # (merge, graphs, pair_delay_us): the merged one-workgroup-per-sample step,
    # and the paired launch whose partners all arrive late (every leader takes
    # the solo fallback, every partner exits): both bitwise the two launches
    for merge, graphs, delay in ((False, False, None), (True, False, None), (True, True, None), (True, False, 30),
                                 (True, True, 30)):
        tr = _trainer(seed=6, use_graphs=graphs, graph_steps=3)
        tr.f28_merge = merge
        tr.f28_pair = delay is not None
        tr.f28_pair_delay_us = delay or 0
        tr.bind_train_data(X, idx)
        tr.set_cursor(0, 8)
        tr.train_steps(6, M=M)
        torch.cuda.synchronize()
        res.append((tr.loss_history()[:6].copy(), tr.params.clone(), tr.exp_avg.clone(), tr.exp_avg_sq.clone(),
                    {k: v.clone() for k, v in tr.gacts.items()}, tr.dmulv.clone()))
        assert int(tr.f28_pairw.abs().sum()) == 0 and int(tr.f28_err.item()) == 0
    for h, p, m, v, ga, dm in res[1:]:
        np.testing.assert_array_equal(h, res[0][0])
        assert torch.equal(p, res[0][1]) and torch.equal(m, res[0][2]) and torch.equal(v, res[0][3])
        assert all(torch.equal(ga[k], res[0][4][k]) for k in ga) and torch.equal(dm, res[0][5])


def test_f28_adam_matches_torch_optim(native_ext):
    """The finalize + fused Adam of the fused step against torch.optim.Adam
    fed with the kernel's own gradients, over 3 steps (lr, betas, eps, bias
    corrections, bf16 re-cast of the weight copies)."""
    dev = torch.device("cuda")
    X = torch.rand(512, 784, generator=torch.Generator().manual_seed(1)).to(dev)
    idx = torch.arange(512, device=dev, dtype=torch.int32)
    a = _trainer(seed=5, use_graphs=False, lr=3e-3, betas=(0.8, 0.95), eps=1e-6)
    b = _trainer(seed=5, use_graphs=False, lr=3e-3, betas=(0.8, 0.95), eps=1e-6)
    for tr in (a, b):
        tr.bind_train_data(X, idx)
        tr.set_cursor(0, 4)
    b.f28_skip_adam = True
    ref = torch.nn.Parameter(a.params.detach().clone())
    opt = torch.optim.Adam([ref], lr=3e-3, betas=(0.8, 0.95), eps=1e-6)
    for step in range(3):
        p_prev = a.params.detach().clone()
        b.params.copy_(p_prev)      # b's gradient at a's current weights: bitwise a's own gradient
        b.refresh_weights()
        b.set_step(step)
        b.set_cursor(step, 4)
        b.train_steps(1)
        a.train_steps(1)            # fused finalize + Adam
        torch.cuda.synchronize()
        with torch.no_grad():
            ref.copy_(p_prev)
        ref.grad = b.grads.detach().clone()
        opt.step()
        torch.testing.assert_close(a.params, ref.detach(), rtol=1e-5, atol=1e-7)
        # moments: rounding-level agreement relative to the gradient scale (the
        # kernel's fmaf lerp vs torch's lerp_ differ in the last ulp of g)
        gmax = float(ref.grad.abs().max())
        torch.testing.assert_close(a.exp_avg, opt.state[ref]["exp_avg"], rtol=1e-5, atol=1e-6 * gmax)
        torch.testing.assert_close(a.exp_avg_sq, opt.state[ref]["exp_avg_sq"], rtol=1e-5, atol=1e-6 * gmax * gmax)
        assert torch.equal(a.w16, a.params.to(torch.bfloat16))  # bf16 re-cast of the updated masters


def test_f28_matches_layer_path_training(native_ext, monkeypatch):
    """Same trial trained by the fused step and by the layer-by-layer step:
    the per-step losses track each other (different bf16 rounding points and
    f32 summation orders, nothing else)."""
    from multidisttorch_amd.data.datasets import synthetic_images

    dev = torch.device("cuda")
    X = synthetic_images(1024, device=dev)
    idx = torch.arange(1024, device=dev, dtype=torch.int32)
    hist = []
    for f28 in ("1", "0"):
        monkeypatch.setenv("MDT_CONV_F28", f28)
        from multidisttorch_amd.models.conv_vae import ConvVaeTrainer

        tr = ConvVaeTrainer(batch_size=128, image=28, device=dev, backend="hip", seed=4, use_graphs=True,
                            graph_steps=5)
        assert tr.f28 == (f28 == "1")
        tr.bind_train_data(X, idx)
        tr.set_cursor(0, 8)
        tr.train_steps(20)
        torch.cuda.synchronize()
        hist.append(tr.loss_history()[:20].copy())
    np.testing.assert_allclose(hist[0], hist[1], rtol=3e-2)
    assert hist[0][-1] < 0.8 * hist[0][0]


@pytest.mark.parametrize("M", [128, 77])
def test_f28_pair_all_paired_and_clean(M, native_ext):
    """Two workgroups per sample: on an idle MI355X every sample pairs (no
    solo fallback), no exchange times out, the pairing words and exchange
    granules are all zero again after the launch (replays need no memset),
    and the losses track the one-workgroup step to f32-summation-order level."""
    from multidisttorch_amd.data.datasets import synthetic_images

    dev = torch.device("cuda")
    X = synthetic_images(1024, device=dev)
    idx = torch.arange(1024, device=dev, dtype=torch.int32)
    res = []
    for pair in (True, False):
        tr = _trainer(seed=9, use_graphs=False)
        tr.f28_pair = pair
        tr.f28_stamps = (torch.zeros(2 * 128 * 16, dtype=torch.int64, device=dev),
                         torch.zeros(2 * 128 * 16, dtype=torch.int64, device=dev))
        tr.bind_train_data(X, idx)
        tr.set_cursor(0, 8)
        tr.train_steps(6, M=M)
        torch.cuda.synchronize()
        if pair:
            modes = tr.f28_stamps[0].view(256, 16)[:2 * M, 15].cpu() & 15
            assert int((modes == 1).sum()) == M and int((modes == 2).sum()) == M, modes
            assert int(tr.f28_err.item()) == 0
            assert int(tr.f28_pairw.abs().sum()) == 0 and int(tr.f28_xg.abs().sum()) == 0
        res.append((tr.loss_history()[:6].copy(), tr.params.clone()))
    # the per-step losses agree to f32-summation-order level (parameters are not
    # compared elementwise: Adam turns a rounding-level sign change of a near-zero
    # gradient into a full lr-sized step; the gradients themselves are checked
    # against the f64 oracle above, pair and solo alike)
    np.testing.assert_allclose(res[0][0], res[1][0], rtol=2e-3)


def test_f28_pair_two_trials_packed(native_ext):
    """Two paired trials launched on two streams at once (4B workgroups for
    256 CUs): whatever mix of paired and solo samples the dispatch produces,
    no exchange times out, the words are clean and both trials train."""
    from multidisttorch_amd.data.datasets import synthetic_images

    dev = torch.device("cuda")
    X = synthetic_images(2048, device=dev)
    idx = torch.arange(2048, device=dev, dtype=torch.int32)
    trs = [_trainer(seed=10 + i, use_graphs=True, graph_steps=5) for i in range(2)]
    for tr in trs:
        tr.bind_train_data(X, idx)
        tr.set_cursor(0, 16)
        tr.prepare([128])
    streams = [torch.cuda.Stream() for _ in trs]
    for _ in range(8):
        for tr, s in zip(trs, streams):
            with torch.cuda.stream(s):
                tr.train_steps(5)
    torch.cuda.synchronize()
    for tr in trs:
        h = tr.loss_history()[:40]
        assert np.all(np.isfinite(h)) and h[-5:].mean() < 0.8 * h[:5].mean(), h
        assert int(tr.f28_err.item()) == 0
        assert int(tr.f28_pairw.abs().sum()) == 0 and int(tr.f28_xg.abs().sum()) == 0


@pytest.mark.parametrize("pair", [False, True])
def test_f28_run_to_run_bitwise(pair, native_ext):
    """The same trial trained twice (fresh trainers, eager, 8 steps, with an
    unrelated stream of kernels running beside the second one to perturb
    dispatch timing) must give bitwise the same losses and parameters."""
    dev = torch.device("cuda")
    X = torch.rand(4 * 128, 784, generator=torch.Generator().manual_seed(3)).to(dev)
    idx = torch.arange(4 * 128, device=dev, dtype=torch.int32)
    res = []
    for noisy in (False, True, False):
        tr = _trainer(seed=4, use_graphs=False, lr=2e-3)
        tr.f28_pair = pair
        tr.bind_train_data(X, idx)
        tr.set_cursor(0, 4)
        side = torch.cuda.Stream()
        junk = torch.rand(4096, 4096, device=dev)
        for _ in range(8):
            if noisy:
                with torch.cuda.stream(side):
                    junk = junk @ junk
                    junk = junk / junk.norm()
            tr.train_steps(1)
        torch.cuda.synchronize()
        res.append((tr.loss_history()[:8].copy(), tr.params.clone()))
    for h, p in res[1:]:
        np.testing.assert_array_equal(h, res[0][0])
        assert torch.equal(p, res[0][1])


def test_f28_exchange_timeout_is_reported(native_ext):
    """A paired half that stalls past the exchange bound (test-only stall of
    sample 0's role-1 workgroup): its partner's sweep times out, sets f28_err,
    and the trainer's health check reports the corruption instead of staying
    silent (the step trained on zero-filled partial sums)."""
    dev = torch.device("cuda")
    X = torch.rand(2 * 128, 784, generator=torch.Generator().manual_seed(5)).to(dev)
    idx = torch.arange(2 * 128, device=dev, dtype=torch.int32)
    tr = _trainer(seed=2, use_graphs=False)
    assert tr.health_error() is None
    tr.f28_pair_delay_us = -400000  # 0.4 s > the 0.25 s sweep bound
    tr.bind_train_data(X, idx)
    tr.set_cursor(0, 2)
    tr.train_steps(1)
    torch.cuda.synchronize()
    assert int(tr.f28_err.item()) & 1
    msg = tr.health_error()
    assert msg and "exchange timed out" in msg, msg


def test_f28_exchange_timeout_fails_bench_and_trial(tmp_path):
    """The same fault through the two production entry points: bench.py's
    record is marked invalid and vae-hpo.py reports the trial as failed."""
    import json
    import os
    import re
    import subprocess
    import sys

    root = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    env = dict(os.environ, MASTER_ADDR="127.0.0.1", MASTER_PORT="29631", MDT_F28_TEST_STALL_US="400000")
    r = subprocess.run([sys.executable, os.path.join(root, "bench.py"), "--steps", "2", "--warmup", "1",
                        "--graph-steps", "2"], capture_output=True, text=True, timeout=300, cwd=root, env=env)
    assert r.returncode == 0, r.stderr[-3000:]
    out = json.loads([l for l in r.stdout.splitlines() if l.startswith("{")][-1])
    assert out["config"]["valid"] is False and out["config"]["health"], out["config"]
    env["MASTER_PORT"] = "29632"
    r = subprocess.run([sys.executable, os.path.join(root, "vae-hpo.py"), "--ngroups", "1", "--epochs", "1",
                        "--model", "conv", "--train-samples", "512", "--test-samples", "256", "--no-results"],
                       capture_output=True, text=True, timeout=300, cwd=str(tmp_path), env=env)
    text = r.stdout + r.stderr
    assert r.returncode == 0, text[-4000:]
    assert "FAILED: TrialCorrupted" in text, text[-4000:]
    agg = json.loads(re.search(r"MDT_AGGREGATE (.*)", text).group(1))
    assert agg["failed_trials"] == [0], agg


def test_f28_pair_and_solo_are_bitwise_equal(native_ext):
    """The one-workgroup fallback sums every K-split partial (head forward,
    dec_fc backward, head backward row groups, enc2 bias rows) in the paired
    step's order, so which form a sample takes -- a matter of dispatch timing
    under contention -- never changes the bits."""
    dev = torch.device("cuda")
    X = torch.rand(4 * 128, 784, generator=torch.Generator().manual_seed(8)).to(dev)
    idx = torch.arange(4 * 128, device=dev, dtype=torch.int32)
    res = {}
    for pair in (True, False):
        tr = _trainer(seed=11, use_graphs=False)
        tr.f28_pair = pair
        tr.f28_skip_adam = True
        tr.bind_train_data(X, idx)
        tr.set_cursor(0, 4)
        tr.train_steps(1)
        torch.cuda.synchronize()
        B = 128
        fb, fp = tr.f28_bias, tr.f28_part
        snap = {"grads": tr.grads.clone(), "dmulv": tr.dmulv.clone(), "mulv": tr.mulv.clone(),
                "dlog32": tr.dlog32.clone(),
                "bias.dbd": fb[:B * 3136].clone(), "bias.db3": fb[B * 3136:B * 3168].clone(),
                "bias.db2": fb[B * 3168:B * 3296].clone(), "bias.db1": fb[B * 3296:].clone(),
                "part.bce": fp[:B].clone(), "part.kld": fp[B:2 * B].clone(), "part.db4": fp[2 * B:].clone()}
        snap.update({"gact." + k: v.clone() for k, v in tr.gacts.items()})
        snap.update({"act." + k: v.clone() for k, v in tr.acts.items()})
        tr.f28_skip_adam = False
        tr.train_steps(5)
        torch.cuda.synchronize()
        snap["loss"] = torch.from_numpy(tr.loss_history()[:6].copy())
        snap["params"] = tr.params.clone()
        res[pair] = snap
    diff = {k: (res[True][k].float() - res[False][k].float()).abs().max().item() for k in res[True]
            if not torch.equal(res[True][k], res[False][k])}
    assert not diff, diff


@pytest.mark.parametrize("pair", [False, True])
def test_f28_no_uninitialised_lds_reads(pair, native_ext):
    """Every LDS word the fused step reads is written in the same launch:
    poisoning every CU's LDS (NaN / a large finite pattern) before each step
    leaves the results bitwise unchanged."""
    dev = torch.device("cuda")
    X = torch.rand(4 * 128, 784, generator=torch.Generator().manual_seed(4)).to(dev)
    idx = torch.arange(4 * 128, device=dev, dtype=torch.int32)
    res = []
    for pattern in (None, 0x7FC00000, 0x4B000000):  # clean, quiet NaN, 8388608.0
        tr = _trainer(seed=12, use_graphs=False)
        tr.f28_pair = pair
        tr.bind_train_data(X, idx)
        tr.set_cursor(0, 4)
        for _ in range(4):
            if pattern is not None:
                tr.C.probe_lds_poison(pattern, 2048)
            tr.train_steps(1)
        torch.cuda.synchronize()
        res.append((tr.loss_history()[:4].copy(), tr.params.clone()))
    for h, p in res[1:]:
        np.testing.assert_array_equal(h, res[0][0])
        assert torch.equal(p, res[0][1])


def test_f28_near_path_is_exercised_and_bitwise(native_ext):
    """Same-XCD pairs hand off through workgroup-scope granule stores
    (conv28_pair.h `near`, profiles/r4_near_scope): the phase stamps' slot 15
    must show such pairs, and the paired result must still be bitwise the
    solo one, which has no hand-offs at all."""
    dev = torch.device("cuda")
    X = torch.rand(4 * 128, 784, generator=torch.Generator().manual_seed(6)).to(dev)
    idx = torch.arange(4 * 128, device=dev, dtype=torch.int32)
    res = {}
    for pair in (True, False):
        tr = _trainer(seed=5, use_graphs=False)
        tr.f28_pair = pair
        stamps = torch.zeros(2 * 128 * 16, dtype=torch.int64, device=dev)
        tr.f28_stamps = (stamps, None)
        tr.bind_train_data(X, idx)
        tr.set_cursor(0, 4)
        near = 0
        for _ in range(4):
            tr.train_steps(1)
            if pair:
                s = stamps.view(256, 16)[:, 15].cpu()
                near += int(((s >> 4) & 1).sum())
        torch.cuda.synchronize()
        res[pair] = (tr.loss_history()[:4].copy(), tr.params.clone(), near)
    assert res[True][2] > 0, "no same-XCD pair took the near hand-off"
    np.testing.assert_array_equal(res[True][0], res[False][0])
    assert torch.equal(res[True][1], res[False][1])


def test_f28_next_batch_prefetch_is_bitwise_and_tagged(native_ext):
    """The finalize of step k gathers step k+1's rows into f28_xn with
    xtag = step (the step kernel's P0 then skips the cursor -> index -> row
    chain): training with and without the prefetch is bitwise equal across
    graphs, tail batches and host cursor moves, and after a step the tags
    name the current step and xn holds exactly the next batch's rows."""
    dev = torch.device("cuda")
    B, nb, tail = 128, 3, 40
    g = torch.Generator().manual_seed(21)
    X = torch.rand(nb * B + tail, 784, generator=g).to(dev)
    idx = torch.randperm(nb * B + tail, generator=g).to(torch.int32).to(dev)
    res = {}
    for pre in (False, True):
        tr = _trainer(B=B, seed=5, use_graphs=True, graph_steps=2)
        tr.f28_prefetch = pre
        tr.bind_train_data(X, idx)
        tr.set_cursor(0, nb + 1)
        tr.train_steps(nb)
        tr.train_steps(1, M=tail)
        tr.set_cursor(1, nb + 1)  # host moves the cursor: the gathered rows are stale
        tr.train_steps(2)
        torch.cuda.synchronize()
        st = tr.read_state()
        if pre:
            assert (tr.f28_xtag == st["step"]).all()
            cur = st["cursor"]
            rows = tr._data[1][cur * B:(cur + 1) * B].long()
            assert torch.equal(tr.f28_xn.view(B, 784), X[rows])
        else:
            assert (tr.f28_xtag == -1).all()
        res[pre] = (tr.loss_history()[:nb + 3].copy(), tr.params.clone())
    np.testing.assert_array_equal(res[True][0], res[False][0])
    assert torch.equal(res[True][1], res[False][1])


_MERGED_CHILD = r"""
import sys, torch
from multidisttorch_amd.models.conv_vae import ConvVaeTrainer
B, nb = 128, 3
g = torch.Generator().manual_seed(33)
X = torch.rand(nb * B, 784, generator=g).cuda()
idx = torch.randperm(nb * B, generator=g).to(torch.int32).cuda()
tr = ConvVaeTrainer(batch_size=B, image=28, device=torch.device("cuda"), backend="hip", seed=9, use_graphs=True,
                    graph_steps=2)
assert tr.f28_fin_merge  # MDT_F28_FIN_MERGE=1 in the environment
tr.bind_train_data(X, idx)
tr.set_cursor(0, nb)
tr.train_steps(5)
torch.cuda.synchronize()
assert tr.health_error() is None, tr.health_error()
torch.save(tr.params.cpu(), sys.argv[1])
"""


def test_f28_merged_finalize_is_bitwise_the_two_launch_tail(native_ext, tmp_path):
    """The finalize + Adam (and the prefetch gather) run inside the
    weight-gradient launch, released per layer by in-launch counters
    (MDT_F28_FIN_MERGE=1, conv_jobs.hip JobPackN deps): parameters, losses and
    the gathered next batch are bitwise those of the separate finalize launch,
    over graphs, a tail batch, a host cursor move and a no-Adam step; the
    counters are back to zero after every launch and no wait gave up. Also
    with the launch confined to 32 CUs (HSA_CU_MASK, a child process), where
    most waiting workgroups are not resident beside their producers."""
    import os
    import subprocess
    import sys

    dev = torch.device("cuda")
    B, nb, tail = 128, 3, 40
    g = torch.Generator().manual_seed(23)
    X = torch.rand(nb * B + tail, 784, generator=g).to(dev)
    idx = torch.randperm(nb * B + tail, generator=g).to(torch.int32).to(dev)
    res = {}
    for merge in (False, True):
        tr = _trainer(B=B, seed=6, use_graphs=True, graph_steps=2)
        tr.f28_fin_merge = merge
        tr.bind_train_data(X, idx)
        tr.set_cursor(0, nb + 1)
        tr.train_steps(nb)
        tr.train_steps(1, M=tail)
        tr.set_cursor(1, nb + 1)
        tr.train_steps(2)
        tr.f28_skip_adam = True
        tr.train_steps(1)
        grads = tr.grads.clone()
        tr.f28_skip_adam = False
        tr.train_steps(2)
        torch.cuda.synchronize()
        assert tr.health_error() is None
        if merge:
            assert int(tr.f28_dep.abs().sum()) == 0  # every counter re-zeroed, no error word
        res[merge] = (tr.loss_history()[:nb + 6].copy(), tr.params.clone(), tr.exp_avg_sq.clone(), grads,
                      tr.f28_xn.clone(), tr.f28_xtag.clone())
    np.testing.assert_array_equal(res[True][0], res[False][0])
    for a, b in zip(res[True][1:], res[False][1:]):
        assert torch.equal(a, b)

    # reference for the child: same data / seed, separate finalize launch, in this process
    g = torch.Generator().manual_seed(33)
    X = torch.rand(nb * B, 784, generator=g).to(dev)
    idx = torch.randperm(nb * B, generator=g).to(torch.int32).to(dev)
    tr = _trainer(B=B, seed=9, use_graphs=True, graph_steps=2)
    tr.f28_fin_merge = False
    tr.bind_train_data(X, idx)
    tr.set_cursor(0, nb)
    tr.train_steps(5)
    torch.cuda.synchronize()
    ref = tr.params.cpu()
    out = tmp_path / "params.pt"
    env = dict(os.environ, HSA_CU_MASK="0:0-31", MDT_F28_FIN_MERGE="1")
    r = subprocess.run([sys.executable, "-c", _MERGED_CHILD, str(out)], env=env, capture_output=True, text=True,
                       timeout=240)
    assert r.returncode == 0, r.stderr[-2000:]
    assert torch.equal(torch.load(out, weights_only=True), ref)
