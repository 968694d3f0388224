"""Graph-replayed eval passes (multidisttorch_amd/models/eval_graphs.py): the
reference's per-epoch test() (/root/reference/vae-hpo.py:95-119) as one eager
batch + captured graphs of the rest. Must equal the eager pass bitwise (same
kernels, same order) for both trainers, with a tail batch, with and without
the reconstruction, on repeated passes (graph reuse) and after training steps
in between (the eval cursor / loss ring are device state)."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def _make(kind, graphs, dev):
    if kind == "mlp":
        from multidisttorch_amd.models.mlp_trainer import MlpVaeTrainer

        return MlpVaeTrainer(batch_size=128, device=dev, backend="hip", seed=6, use_graphs=graphs, graph_steps=4)
    from multidisttorch_amd.models.conv_vae import ConvVaeTrainer

    if kind == "conv28":
        return ConvVaeTrainer(batch_size=128, image=28, z=32, device=dev, backend="hip", seed=6, use_graphs=graphs,
                              graph_steps=4)
    return ConvVaeTrainer(batch_size=32, image=128, z=64, device=dev, backend="hip", seed=6, use_graphs=graphs,
                          graph_steps=4)


@pytest.mark.parametrize("kind", ["mlp", "conv28", "conv128"])
def test_graphed_eval_is_bitwise_eager(kind, native_ext):
    dev = torch.device("cuda", 0)
    D = 784 if kind != "conv128" else 128 * 128
    n_test = 300 if kind != "conv128" else 75
    g = torch.Generator().manual_seed(8)
    Xtr = torch.rand(512, D, generator=g).to(dev)
    Xte = torch.rand(n_test, D, generator=g).to(dev)
    idx_tr = torch.arange(512, dtype=torch.int32, device=dev)
    out = {}
    for graphs in (False, True):
        tr = _make(kind, graphs, dev)
        tr.bind_train_data(Xtr, idx_tr)
        tr.set_cursor(0, 512 // tr.B)
        res = []
        for rnd in range(2):
            tr.train_steps(2)
            for want in (True, False):
                idx = torch.arange(n_test, dtype=torch.int32, device=dev)
                total, first = tr.evaluate(Xte, idx, want_first_recon=want)
                torch.cuda.synchronize()
                res.append((total, None if first is None else first.cpu(),
                            tr.loss_history(eval=True)[: -(-n_test // tr.B)].copy(), tr.read_state(eval=True)))
        out[graphs] = res
        if graphs:
            assert tr._eval_graphs, "the graphed path did not run"
    for a, b in zip(out[False], out[True]):
        assert a[0] == b[0], (a[0], b[0])
        np.testing.assert_array_equal(a[2], b[2])
        assert a[3]["cursor"] == b[3]["cursor"] and a[3]["step"] == b[3]["step"]
        if a[1] is not None:
            assert torch.equal(a[1], b[1])


def test_conv28_paired_eval_is_bitwise_solo(native_ext, monkeypatch):
    """The eval forward through the step kernel's paired form (two workgroups
    per sample, backward skipped) equals the solo f28_fwd_k pass bit for bit,
    with a tail batch, and leaves the pair state clean (error word 0, a
    training step after it still pairs)."""
    dev = torch.device("cuda", 0)
    g = torch.Generator().manual_seed(11)
    Xtr = torch.rand(512, 784, generator=g).to(dev)
    Xte = torch.rand(300, 784, generator=g).to(dev)
    idx_tr = torch.arange(512, dtype=torch.int32, device=dev)
    out = {}
    for pair in ("0", "1"):
        monkeypatch.setenv("MDT_F28_EVAL_PAIR", pair)
        tr = _make("conv28", True, dev)
        assert tr._eval_pair == (pair == "1") and tr.f28_pair
        tr.bind_train_data(Xtr, idx_tr)
        tr.set_cursor(0, 4)
        tr.train_steps(2)
        res = []
        for want in (True, False):
            total, first = tr.evaluate(Xte, torch.arange(300, dtype=torch.int32, device=dev), want_first_recon=want)
            torch.cuda.synchronize()
            res.append((total, None if first is None else first.cpu(), tr.loss_history(eval=True)[:3].copy()))
        tr.train_steps(2)
        torch.cuda.synchronize()
        assert int(tr.f28_err.item()) == 0
        res.append(tr.params.cpu())
        out[pair] = res
    for a, b in zip(out["0"][:2], out["1"][:2]):
        assert a[0] == b[0], (a[0], b[0])
        np.testing.assert_array_equal(a[2], b[2])
        if a[1] is not None:
            assert torch.equal(a[1], b[1])
    assert torch.equal(out["0"][2], out["1"][2])


def test_eval_graph_cache_keeps_the_latest_eval_set_only(native_ext):
    """eval graphs are cached per eval set; a new X (e.g. a
    temporary ``.contiguous()`` copy each epoch) drops the previous set's
    graphs instead of capturing more and more of them, and the pass over the
    new set is still bitwise the eager pass."""
    dev = torch.device("cuda", 0)
    g = torch.Generator().manual_seed(12)
    Xtr = torch.rand(512, 784, generator=g).to(dev)
    idx_tr = torch.arange(512, dtype=torch.int32, device=dev)
    tr = _make("conv28", True, dev)
    ref = _make("conv28", False, dev)
    for t in (tr, ref):
        t.bind_train_data(Xtr, idx_tr)
        t.set_cursor(0, 4)
        t.train_steps(1)
    idx = torch.arange(300, dtype=torch.int32, device=dev)
    counts = []
    for k in range(4):
        Xte = torch.rand(300, 784, generator=g).to(dev)  # a fresh tensor every pass
        total, _ = tr.evaluate(Xte, idx, want_first_recon=False)
        rtotal, _ = ref.evaluate(Xte, idx, want_first_recon=False)
        torch.cuda.synchronize()
        assert total == rtotal, (k, total, rtotal)
        counts.append(len(tr._eval_graphs))
        assert all(key[2] == Xte.data_ptr() for key in tr._eval_graphs)
        del Xte
    assert max(counts) == counts[0] == 2, counts  # (full-batch graph, tail graph) of the latest set
