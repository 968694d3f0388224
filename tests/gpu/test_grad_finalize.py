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


def _emulated_sum(slab, rp):
    """The finalize kernel's summation order in float32 (conv_small.h): thread
    row rl sums slabs rl, rl + rp, ... into 4 interleaved accumulators (full
    quads, the remainder into the first), then row 0 adds the rp row sums in
    order starting from 0."""
    ns = slab.shape[0]
    z = torch.zeros(slab.shape[1], dtype=torch.float32)
    g = z.clone()
    for rl in range(rp):
        ks = list(range(rl, ns, rp))
        a = [z.clone() for _ in range(4)]
        q = len(ks) // 4
        for i in range(q):
            for j in range(4):
                a[j] = a[j] + slab[ks[4 * i + j]]
        for k in range(4 * q, len(ks)):
            a[0] = a[0] + slab[ks[k]]
        g = g + ((a[0] + a[1]) + (a[2] + a[3]))
    return g


@pytest.mark.parametrize("ns,cnt", [(5, 16), (20, 128), (131, 16), (131, 256), (300, 64), (3, 1024), (16, 1024),
                                    (20, 1024)])
def test_grad_finalize_matches_emulated_order(ns, cnt, native_ext):
    """Bitwise: the batched-load path (<= 16 slabs per thread) and the loop
    path (more) both sum in the documented order -- units of `cnt` elements,
    rp = 256 / cnt partial rows per column (cnt 1024: 4 elements per thread)."""
    C = native_ext
    dev = torch.device("cuda")
    numel = 2048 + 4
    slab = torch.randn(ns, numel)
    ds = slab.to(dev).reshape(-1)
    segs = C.make_grad_segs([[0, numel, ds.data_ptr(), ns, 0, 0, 0, 0, -1]], 0)
    units = [[0, st, min(cnt, numel - st)] for st in range(0, numel, cnt)]
    state = C.TrialState(0)
    state.set_step(False, 1)
    G = torch.zeros(numel, device=dev)
    P, M, V = torch.zeros(numel, device=dev), torch.zeros(numel, device=dev), torch.zeros(numel, device=dev)
    w16 = torch.zeros(numel, dtype=torch.bfloat16, device=dev)
    C.grad_finalize(P, G, M, V, w16, segs, C.make_grad_units(units, 0), len(units), state.train_state,
                    state.hparams, False)
    torch.cuda.synchronize()
    got = G.cpu()
    for st, n in [(u[1], u[2]) for u in units]:
        rp = 1 if n > 256 else 256 // n  # a short tail unit takes the scalar path
        want = _emulated_sum(slab[:, st:st + n], rp)
        assert torch.equal(got[st:st + n], want), (st, n, rp)
