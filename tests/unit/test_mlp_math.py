"""CPU oracle checks of the math the HIP kernels implement (fp64)."""
import math

import numpy as np
import pytest
import torch
import torch.nn.functional as F

from multidisttorch_amd.models.mlp_vae import (VAE, arena_layout, init_params_, loss_function,
                                               reference_adam_, reference_forward, reference_step, views)
from multidisttorch_amd.ops.philox import philox4x32_10, reparam_eps


def _setup(D=64, H=32, Z=8, M=16, seed=0):
    lay, n, split = arena_layout(D, H, Z)
    p = torch.zeros(n, dtype=torch.float64)
    g = torch.zeros(n, dtype=torch.float64)
    host = torch.zeros(n)
    init_params_(host, lay, torch.Generator().manual_seed(seed))
    p.copy_(host)
    x = torch.rand(M, D, dtype=torch.float64, generator=torch.Generator().manual_seed(seed + 1))
    eps = torch.randn(M, Z, dtype=torch.float64, generator=torch.Generator().manual_seed(seed + 2))
    return lay, n, split, p, g, x, eps


def test_layout_matches_module_and_alignment():
    lay, n, split = arena_layout()
    m = VAE()
    shapes = {k: tuple(v.shape) for k, v in m.state_dict().items()}
    assert {name: s for name, _, s in lay} == shapes
    assert sum(math.prod(s) for _, _, s in lay) == 652824  # reference parameter count
    names = [name for name, _, _ in lay]
    assert names.index("fc4.weight") > names.index("fc1.weight")
    o = {name: off for name, off, _ in lay}
    assert o["fc22.weight"] == o["fc21.weight"] + 20 * 400  # W2 = [W21; W22] contiguous
    assert split == o["fc4.weight"] and split % 64 == 0


@pytest.mark.parametrize("beta", [1.0, 0.5, 4.0])
def test_explicit_backward_equals_autograd(beta):
    lay, n, split, p, g, x, eps = _setup()
    pv, gv = views(p, lay), views(g, lay)
    f = reference_step(pv, gv, x, eps, beta)
    m = VAE(64, 32, 8).double()
    m.load_state_dict({k: v.clone() for k, v in pv.items()})
    r, mu, lv = m(x, eps=eps)
    loss = loss_function(r, x, mu, lv, beta)
    loss.backward()
    assert float(f["loss"]) == pytest.approx(float(loss), rel=1e-10)
    for name, prm in m.named_parameters():
        torch.testing.assert_close(gv[name], prm.grad, rtol=1e-9, atol=1e-12)


def test_bce_logit_form_matches_torch_with_clamp():
    t = torch.tensor([-200.0, -30.0, -1.0, 0.0, 2.0, 50.0, 300.0], dtype=torch.float64)
    x = torch.tensor([0.0, 0.3, 1.0, 0.5, 0.0, 1.0, 0.2], dtype=torch.float64)
    from multidisttorch_amd.models.mlp_vae import _bce_terms

    ref = F.binary_cross_entropy(torch.sigmoid(t), x, reduction="none")
    torch.testing.assert_close(_bce_terms(t, x), ref, rtol=1e-6, atol=1e-6)


def test_adam_matches_torch_optim():
    torch.manual_seed(0)
    p0 = torch.randn(1000, dtype=torch.float64)
    ref = p0.clone().requires_grad_(True)
    opt = torch.optim.Adam([ref], lr=3e-3, weight_decay=0.01)
    p, m, v = p0.clone(), torch.zeros_like(p0), torch.zeros_like(p0)
    for step in range(1, 6):
        gr = torch.randn(1000, dtype=torch.float64)
        ref.grad = gr.clone()
        opt.step()
        reference_adam_(p, gr, m, v, step, 3e-3, 0.9, 0.999, 1e-8, 0.01)
    torch.testing.assert_close(p, ref.detach(), rtol=1e-12, atol=1e-14)


def test_adamw_matches_torch():
    torch.manual_seed(1)
    p0 = torch.randn(100, dtype=torch.float64)
    ref = p0.clone().requires_grad_(True)
    opt = torch.optim.AdamW([ref], lr=1e-2, weight_decay=0.1)
    p, m, v = p0.clone(), torch.zeros_like(p0), torch.zeros_like(p0)
    for step in range(1, 4):
        gr = torch.randn(100, dtype=torch.float64)
        ref.grad = gr.clone()
        opt.step()
        reference_adam_(p, gr, m, v, step, 1e-2, 0.9, 0.999, 1e-8, 0.1, decoupled=True)
    torch.testing.assert_close(p, ref.detach(), rtol=1e-12, atol=1e-14)


def test_philox_known_answer_and_normality():
    # Random123 known-answer vector for philox4x32-10 (counter=0, key=0)
    c = philox4x32_10(np.array([0], np.uint32), 0, 0, 0, 0, 0)
    assert [int(v[0]) for v in c] == [0x6627E8D5, 0xE169C58D, 0xBC57AC4C, 0x9B00DBD8]
    e = reparam_eps(4096, 20, seed=5, stream=0, step=3)
    assert abs(e.mean()) < 0.01 and abs(e.std() - 1) < 0.01
    assert np.array_equal(e, reparam_eps(4096, 20, seed=5, stream=0, step=3))
    assert not np.array_equal(e, reparam_eps(4096, 20, seed=5, stream=1, step=3))
    assert not np.array_equal(e, reparam_eps(4096, 20, seed=5, stream=0, step=4))
