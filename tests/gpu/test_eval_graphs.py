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
