"""Numerics of the LDS-tiled implicit-GEMM conv kernels vs plain fp32 torch.

Inputs are rounded to bf16 first (the kernels' operand precision), so the
references differ from the kernels only by f32 summation order.
"""
import pytest
import torch
import torch.nn.functional as F

from multidisttorch_amd.ops.conv_layout import conv_desc, nchw, nhwc, parity_transpose, torch_weight

pytestmark = pytest.mark.gpu

DEV = "cuda"


def _bf(t):
    return t.to(torch.bfloat16)


def _rel(a, b):
    a, b = a.double(), b.double()
    return float((a - b).norm() / (b.norm() + 1e-12))


# (N, H, C, CO, k, s, p)
CONV_SHAPES = [
    (3, 16, 32, 64, 4, 2, 1),     # strided conv, vector im2col
    (2, 14, 32, 64, 4, 2, 1),     # 7x7 output, partial tiles
    (4, 8, 128, 256, 4, 2, 1),    # deep K, 128-wide tiles
    (64, 1, 4096, 128, 1, 1, 0),  # Linear (1x1 image): split-K path
    (5, 1, 64, 1000, 1, 1, 0),    # Linear, ragged columns
]


@pytest.mark.parametrize("shape", CONV_SHAPES)
def test_conv_mode_matches_conv2d(shape, native_ext):
    C = native_ext
    N, H, Ci, CO, k, s, p = shape
    torch.manual_seed(0)
    x = _bf(torch.randn(N, H, H, Ci, device=DEV))
    w = _bf(torch.randn(CO, k, k, Ci, device=DEV) / (k * (Ci ** 0.5)))
    b = torch.randn(CO, device=DEV)
    d = conv_desc(N, H, H, Ci, CO, k, s, p)
    OH = d[4]
    y32 = torch.zeros(N * OH * OH * CO, device=DEV)
    y16 = torch.zeros(N * OH * OH * CO, device=DEV, dtype=torch.bfloat16)
    ws = torch.zeros(64 * N * OH * OH * CO + 1, device=DEV)
    C.igemm(0, x, w.flatten(), d, b, True, y16, y32, ws=ws)
    ref = F.relu(F.conv2d(nchw(x.float()), torch_weight(w.float()), b, s, p))
    ref = nhwc(ref).flatten()
    assert _rel(y32, ref) < 1e-5
    assert _rel(y16.float(), ref) < 1e-2


def test_conv_mode_thin_f32_input(native_ext):
    """enc1 shape: single-channel f32 images, K = 16 (per-element gather)."""
    C = native_ext
    N, H, CO = 6, 28, 32
    x = torch.rand(N, H, H, 1, device=DEV)
    w = _bf(torch.randn(CO, 4, 4, 1, device=DEV) / 4)
    b = torch.randn(CO, device=DEV)
    d = conv_desc(N, H, H, 1, CO, 4, 2, 1)
    y32 = torch.zeros(N * 14 * 14 * CO, device=DEV)
    C.igemm(0, x, w.flatten(), d, b, False, None, y32)
    ref = nhwc(F.conv2d(nchw(_bf(x).float()), torch_weight(w.float()), b, 2, 1)).flatten()
    assert _rel(y32, ref) < 1e-5


# conv-view geometry (N, H, C, CO, k, s, p): backward-data of the conv = the
# forward of the transposed conv with Cin_t = CO, Cout_t = C
TCONV_SHAPES = [
    (3, 16, 32, 64, 4, 2, 1),
    (2, 14, 32, 64, 4, 2, 1),
    (2, 28, 1, 32, 4, 2, 1),      # last decoder layer: one output channel
    (4, 16, 128, 256, 4, 2, 1),
    (64, 1, 4096, 64, 1, 1, 0),   # Linear backward-data, split-K
]


@pytest.mark.parametrize("shape", TCONV_SHAPES)
def test_parity_mode_matches_conv_transpose(shape, native_ext):
    C = native_ext
    N, H, Ci, CO, k, s, p = shape
    torch.manual_seed(1)
    d = conv_desc(N, H, H, Ci, CO, k, s, p)
    OH = d[4]
    g = _bf(torch.randn(N, OH, OH, CO, device=DEV))
    w = _bf(torch.randn(CO, k, k, Ci, device=DEV) / (k * (CO ** 0.5)))
    mask = _bf(torch.randn(N, H, H, Ci, device=DEV))
    b = torch.randn(Ci, device=DEV)
    wt = parity_transpose(w, s)
    y32 = torch.zeros(N * H * H * Ci, device=DEV)
    ws = torch.zeros(64 * N * H * H * Ci + 1, device=DEV)
    if H == 1:  # split-K path: no epilogue mask
        C.igemm(1, g, wt, d, None, False, None, y32, ws=ws)
        ref = F.conv_transpose2d(nchw(g.float()), torch_weight(w.float()), None, s, p)
    else:
        C.igemm(1, g, wt, d, b, False, None, y32, mask)
        ref = F.conv_transpose2d(nchw(g.float()), torch_weight(w.float()), b, s, p)
        ref = ref * (nchw(mask.float()) > 0)
    ref = nhwc(ref).flatten()
    assert _rel(y32, ref) < 1e-5


def test_colsum_epilogue_and_fold(native_ext):
    """Column sums of the produced (masked) gradient = next layer's bias grad."""
    C = native_ext
    N, H, Ci, CO = 4, 16, 64, 128
    d = conv_desc(N, H, H, Ci, CO, 4, 2, 1)
    info = C.igemm_plan(1, d, False)
    rows, ncols = info[11], info[5]
    g = _bf(torch.randn(N, 8, 8, CO, device=DEV))
    w = _bf(torch.randn(CO, 4, 4, Ci, device=DEV) / 16)
    mask = _bf(torch.randn(N, H, H, Ci, device=DEV))
    y16 = torch.zeros(N * H * H * Ci, device=DEV, dtype=torch.bfloat16)
    cs = torch.full((rows * ncols,), float("nan"), device=DEV)
    C.igemm(1, g, parity_transpose(w, 2), d, None, False, y16, None, mask, cs)
    ref = F.conv_transpose2d(nchw(g.float()), torch_weight(w.float()), None, 2, 1) * (nchw(mask.float()) > 0)
    got = cs.view(rows, ncols).sum(0)
    assert _rel(got, ref.sum((0, 2, 3))) < 1e-4


WGRAD_SHAPES = [
    (4, 16, 32, 64, 4, 2, 1, False),
    (2, 14, 32, 64, 4, 2, 1, False),
    (8, 16, 64, 128, 4, 2, 1, False),
    (6, 28, 1, 32, 4, 2, 1, True),    # enc1: f32 single-channel input
    (3, 28, 1, 32, 4, 2, 1, False),   # last decoder layer (bf16, single channel)
    (64, 1, 4096, 128, 1, 1, 0, False),
    (37, 1, 32, 3136, 1, 1, 0, False),
]


@pytest.mark.parametrize("shape", WGRAD_SHAPES)
def test_wgrad_matches_autograd(shape, native_ext):
    C = native_ext
    N, H, Ci, CO, k, s, p, xf32 = shape
    torch.manual_seed(2)
    d = conv_desc(N, H, H, Ci, CO, k, s, p)
    OH = d[4]
    x = torch.rand(N, H, H, Ci, device=DEV) if xf32 else _bf(torch.randn(N, H, H, Ci, device=DEV))
    g = _bf(torch.randn(N, OH, OH, CO, device=DEV))
    info = C.wgrad_plan(d)
    ns = info[6]
    numel = CO * k * k * Ci
    out = torch.full((ns * numel,), float("nan"), device=DEV)
    C.wgrad(g, x, d, out)
    got = out.view(ns, numel).sum(0)
    xr = nchw(_bf(x).float())
    ref = torch.nn.grad.conv2d_weight(xr, (CO, Ci, k, k), nchw(g.float()), s, p)
    ref = ref.permute(0, 2, 3, 1).flatten()
    assert _rel(got, ref) < 1e-4, (ns, _rel(got, ref))


def test_grad_finalize_is_deterministic_and_fuses_adam(native_ext):
    C = native_ext
    dev = torch.device(DEV)
    numel, ns = 3000, 700
    slab = torch.randn(ns * numel, device=dev)
    segs = C.make_grad_segs([[0, numel, slab.data_ptr(), ns, 0, 0, 0, 0, -1]], 0)
    units = []
    rp = 64
    cnt = 512 // rp
    for st in range(0, numel, cnt):
        units.append([0, st, min(cnt, numel - st)])
    U = C.make_grad_units(units, 0)
    state = C.TrialState(0)
    P = torch.randn(numel, device=dev)
    z = lambda: torch.zeros(numel, device=dev)
    outs = []
    for _ in range(2):
        G = z()
        C.grad_finalize(P.clone(), G, z(), z(), torch.zeros(numel, dtype=torch.bfloat16, device=dev), segs, U,
                        len(units), state.train_state, state.hparams, False)
        outs.append(G)
    assert torch.equal(outs[0], outs[1])
    assert _rel(outs[0], slab.view(ns, numel).sum(0)) < 1e-6


@pytest.mark.parametrize("H", [28, 128])
@pytest.mark.parametrize("f32_in", [True, False])
def test_thin_conv_matches_conv2d(f32_in, H, native_ext):
    # H = 128 exercises the MFMA form (bit 1 of MDT_THIN_MFMA, default since
    # round 5) for the f32 input and bit 8 for bf16; H = 28 the VALU body
    """Single-input-channel conv (encoder conv 1 / last layer backward-data).
    H = 28 runs the VALU body, H = 128 the MFMA form (thin_conv_mfma_body:
    split hi/lo bf16 weights and inputs); the f32 column sums pin both to the
    f32 conv to 1e-5."""
    C = native_ext
    N, CO = (5, 32) if H == 28 else (3, 32)
    OH = H // 2
    torch.manual_seed(3)
    x = torch.rand(N, H, H, 1, device=DEV)
    if not f32_in:
        x = _bf(x)
    w = torch.randn(CO, 4, 4, 1, device=DEV) / 4
    b = torch.randn(CO, device=DEV)
    d = conv_desc(N, H, H, 1, CO, 4, 2, 1)
    M = N * OH * OH
    y16 = torch.zeros(M * CO, device=DEV, dtype=torch.bfloat16)
    mask = _bf(torch.randn(M, CO, device=DEV))
    nb = C.thin_blocks(False, d)
    cs = torch.full((nb * CO,), float("nan"), device=DEV)
    ref = F.conv2d(nchw(x.float()).double(), torch_weight(w).double(), None, 2, 1)
    if f32_in:  # encoder conv 1: bias + ReLU
        C.thin_conv(x, w.flatten(), d, b, True, y16, None, cs)
        ref = nhwc(F.relu(ref + b.double().view(1, -1, 1, 1))).reshape(M, CO)
    else:       # backward-data of the last layer: output mask + column sums
        C.thin_conv(x, w.flatten(), d, None, False, y16, mask, cs)
        ref = nhwc(ref).reshape(M, CO) * (mask.double() > 0)
    torch.cuda.synchronize()
    assert _rel(cs.view(nb, CO).double().sum(0), ref.sum(0)) < 1e-5
    assert _rel(y16.float().view(M, CO), ref.float()) < 1e-2
    # per element: within one bf16 rounding of the f64 result
    # per element: one bf16 rounding of the output plus the MFMA form's split
    # error (x and w in three bf16 terms: ~2^-24 of sum |x||w| per output)
    mag = nhwc(F.conv2d(nchw(x.float()).abs().double(), torch_weight(w).abs().double(), None, 2, 1)).reshape(M, CO)
    err = (y16.double().view(M, CO) - ref).abs()
    bad = err > ref.abs() * 2.0 ** -8 + mag * 2.0 ** -20 + 1e-7
    if bool(bad.any()):
        i = int((err / (ref.abs() + 1e-6)).argmax())
        print(f"thin_conv H={H} f32_in={f32_in}: {int(bad.sum())}/{bad.numel()} beyond one bf16 rounding; worst "
              f"flat {i} (pixel {i // CO}, co {i % CO}): kernel {float(y16.double().view(-1)[i])} ref "
              f"{float(ref.view(-1)[i])}")
    assert not bool(bad.any())


def test_thin_tconv_fused_bce(native_ext):
    """Last decoder layer (32 -> 1 transposed conv) fused with logit BCE."""
    C = native_ext
    N, OH, CI = 4, 14, 32
    torch.manual_seed(4)
    d = conv_desc(N, 2 * OH, 2 * OH, 1, CI, 4, 2, 1)
    g = _bf(torch.randn(N, OH, OH, CI, device=DEV))
    w = torch.randn(CI, 4, 4, 1, device=DEV) / 8
    b = torch.randn(1, device=DEV)
    x = torch.rand(N, 2 * OH * 2 * OH, device=DEV)
    npix = x.numel()
    nb = C.thin_blocks(True, d)
    logits = torch.zeros(npix, device=DEV)
    dlog = torch.zeros(npix, device=DEV, dtype=torch.bfloat16)
    part = torch.zeros(nb, device=DEV)
    gpart = torch.zeros(nb, device=DEV)
    C.thin_tconv(g, w.flatten(), d, b, y32=logits)
    C.thin_tconv(g, w.flatten(), d, b, X=x, dlog16=dlog, part=part, gpart=gpart)
    t = F.conv_transpose2d(nchw(g.float()), torch_weight(w), b, 2, 1).reshape(N, -1)
    assert _rel(logits.view(N, -1), t) < 1e-5
    p = torch.sigmoid(t)
    bce = F.binary_cross_entropy(p.double(), x.double(), reduction="sum")
    assert abs(float(part.sum()) - float(bce)) / float(bce) < 1e-4
    assert _rel(dlog.float().view(N, -1), p - x) < 1e-2
    assert abs(float(gpart.sum()) - float((p - x).sum())) < 1e-2 * float((p - x).abs().sum())


@pytest.mark.parametrize("image", [28, 128])
def test_weight_transposes_match_parity_transpose(image, native_ext):
    """w16t (the transposed bf16 weight copies the backward-data GEMMs read)
    equals ops.conv_layout.parity_transpose of every layer's bf16 weights:
    the 16-B form of wtrans_body for channel counts divisible by 8, the 2-B
    form for the single-channel layers."""
    from multidisttorch_amd.models.conv_vae import ConvVaeTrainer, _w_shape
    from multidisttorch_amd.ops.conv_layout import parity_transpose

    tr = ConvVaeTrainer(batch_size=8, image=image, z=32 if image == 28 else 64, device=DEV, backend="hip", seed=1)
    tr.params.copy_(torch.randn(tr.params.shape, generator=torch.Generator().manual_seed(7)).to(DEV))
    tr._cast_weights()
    torch.cuda.synchronize()
    checked = 0
    for l in tr.spec:
        w = tr._w(l).view(*_w_shape(l))
        got = tr._wt(l)
        ref = parity_transpose(w, l.s)
        assert torch.equal(got, ref), l.name
        checked += 1
    assert checked == len(tr.spec)
