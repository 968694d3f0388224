"""Gradient finalize + fused Adam (csrc/kernels/conv_small.h): the vectorised
units (4 elements per thread, 16-B accesses) against the scalar units and a
torch fp32 reference of the slab sum."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def _rel(a, b):
    return float((a.double() - b.double()).norm() / (b.double().norm() + 1e-30))


@pytest.mark.parametrize("ns", [1, 3, 9])
def test_grad_finalize_vec4_units_match_scalar_units(ns, native_ext):
    """Units of 1024 elements (planned for segments with <= 16 slabs) give
    bitwise the same gradient and Adam state as 256-element units, including a
    segment tail that is not a multiple of 4."""
    C = native_ext
    dev = torch.device("cuda")
    numel = 5000 + 2  # tail of 2 elements after the last full float4
    slab = torch.randn(ns * numel, device=dev)
    segs = C.make_grad_segs([[0, numel, slab.data_ptr(), ns, 0, 0, 0, 0, -1]], 0)
    state = C.TrialState(0)
    state.set_step(False, 1)  # Adam bias corrections of step 1
    P0 = torch.randn(numel, device=dev)
    M0, V0 = torch.randn(numel, device=dev) * 0.1, torch.rand(numel, device=dev) * 0.1
    by = {}
    for cnt in (256, 1024):
        units = [[0, st, min(cnt, numel - st)] for st in range(0, numel, cnt)]
        U = C.make_grad_units(units, 0)
        for do_adam in (False, True):
            G = torch.zeros(numel, device=dev)
            P, M, V = P0.clone(), M0.clone(), V0.clone()
            w16 = torch.zeros(numel, dtype=torch.bfloat16, device=dev)
            C.grad_finalize(P, G, M, V, w16, segs, U, len(units), state.train_state, state.hparams, do_adam)
            torch.cuda.synchronize()
            by[(cnt, do_adam)] = (G, P, M, V, w16)
    assert torch.equal(by[(256, False)][0], by[(1024, False)][0])
    assert _rel(by[(1024, False)][0], slab.view(ns, numel).sum(0)) < 1e-6
    for a, b in zip(by[(256, True)][1:], by[(1024, True)][1:]):
        assert torch.equal(a, b)
    assert not torch.equal(by[(1024, True)][1], P0)  # Adam actually updated the parameters
