"""Patch-resident direct conv kernels (csrc/kernels/conv_direct.h) vs fp32 torch.

The 128x128 conv-VAE's stride-2 4x4 layers run on these kernels through the
same ``igemm`` entry point as the im2col kernels (the planner picks them by
geometry). Each case feeds bf16-exact inputs and compares the bf16/f32 outputs,
the ReLU / ReLU-backward mask epilogue and the per-workgroup column sums with
``conv2d`` / ``conv_transpose2d`` in fp32 (the kernels accumulate in f32, so
the only difference is summation order and the final bf16 rounding)."""
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu


def _parity_B(Wc):
    """Conv-view weight [CO][C][4][4] -> per-class B[cls][C][(t0, t1, co)] of the
    parity-class transposed conv (class (ca, cb) -> output parity (oa, ob) =
    ((ca+1)&1, (cb+1)&1); tap (t0, t1) reads A row a + ea - t0 with
    ea = (oa+1-ca)>>1, i.e. kernel row ky = oa + 1 - 2 ea + 2 t0)."""
    CO, C = Wc.shape[:2]
    out = []
    for cls in range(4):
        ca, cb = cls >> 1, cls & 1
        oa, ob = (ca + 1) & 1, (cb + 1) & 1
        ea, eb = (oa + 1 - ca) >> 1, (ob + 1 - cb) >> 1
        taps = []
        for t0 in range(2):
            for t1 in range(2):
                ky, kx = oa + 1 - 2 * ea + 2 * t0, ob + 1 - 2 * eb + 2 * t1
                taps.append(Wc[:, :, ky, kx].t())  # [C][CO]
        out.append(torch.stack(taps, 1).reshape(C, 4 * CO))
    return torch.stack(out, 0).contiguous()


# (mode, H, C, OH, CO) in conv view: mode 0 = conv (A = H x H x C), mode 1 =
# transposed conv (A = OH x OH x CO, output H x H x C)
CASES = [(0, 64, 32, 32, 64), (0, 32, 64, 16, 128), (1, 32, 64, 16, 128), (1, 64, 32, 32, 64),
         (0, 16, 128, 8, 256), (1, 16, 128, 8, 256)]


@pytest.mark.parametrize("case", CASES, ids=lambda c: f"mode{c[0]}_{c[1]}x{c[2]}_{c[3]}x{c[4]}")
@pytest.mark.parametrize("epi", ["bias_relu", "mask_colsum"])
def test_direct_conv_matches_torch(case, epi, native_ext):
    C_ = native_ext
    mode, H, C, OH, CO = case
    N = 3
    dev = torch.device("cuda")
    g = torch.Generator(device="cpu").manual_seed(11 + mode + H)
    Wc = (torch.randn(CO, C, 4, 4, generator=g) * 0.05).bfloat16().float().to(dev)
    d = [N, H, H, C, OH, OH, CO, 4, 4, 2, 1]
    info = C_.igemm_plan(mode, d, False, fwd=True)
    assert info[0] >= 100, f"direct kernel not selected: {info}"
    if mode == 0:
        A = torch.randn(N, C, H, H, generator=g).bfloat16().float().to(dev)
        ref = F.conv2d(A, Wc, stride=2, padding=1)          # [N][CO][OH][OH]
        B16 = Wc.permute(0, 2, 3, 1).contiguous().bfloat16()
        ncols = CO
    else:
        A = torch.randn(N, CO, OH, OH, generator=g).bfloat16().float().to(dev)
        ref = F.conv_transpose2d(A, Wc, stride=2, padding=1)  # [N][C][H][H]
        B16 = _parity_B(Wc).bfloat16()
        ncols = C
    A16 = A.permute(0, 2, 3, 1).contiguous().bfloat16()
    ref = ref.permute(0, 2, 3, 1).contiguous()  # NHWC
    y16 = torch.empty(ref.numel(), dtype=torch.bfloat16, device=dev)
    y32 = torch.empty(ref.numel(), dtype=torch.float32, device=dev)
    bias = mask = cs = None
    relu = False
    if epi == "bias_relu":
        bias = (torch.randn(ncols, generator=g) * 0.1).to(dev)
        relu = True
        ref = torch.relu(ref + bias)
    else:
        mask = (torch.rand(ref.shape, generator=g) > 0.4).bfloat16().to(dev)
        ref = ref * mask.float()
        cs = torch.full((info[11] * ncols,), float("nan"), device=dev)
    C_.igemm(mode, A16, B16, d, bias, relu, y16, y32, mask, cs, fwd=True)
    torch.cuda.synchronize()
    r = ref.flatten()
    err = float((y32 - r).abs().max() / r.abs().max())
    assert err < 1e-5, err
    torch.testing.assert_close(y16.float(), r.bfloat16().float(), rtol=1e-2, atol=1e-2 * float(r.abs().max()))
    if cs is not None:
        assert torch.isfinite(cs).all()
        tot = cs.view(info[11], ncols).double().sum(0)
        torch.testing.assert_close(tot, ref.reshape(-1, ncols).double().sum(0), rtol=1e-5,
                                   atol=1e-5 * float(ref.abs().sum(0).max()))


def test_thin_tconv_patch_matches_torch(native_ext):
    """Last 128x128 decoder layer (convT 32 -> 1, 64^2 -> 128^2) on the
    halo-patch kernel with the fused BCE: logits vs conv_transpose2d, the
    loss / dlogits-sum partials vs their definitions."""
    C_ = native_ext
    dev = torch.device("cuda")
    N = 3
    g = torch.Generator(device="cpu").manual_seed(5)
    d = [N, 128, 128, 1, 64, 64, 32, 4, 4, 2, 1]
    nb = C_.thin_blocks(True, d)
    assert nb == N * 16, nb  # one workgroup per 4 class-grid rows: the patch kernel
    G = torch.randn(N, 32, 64, 64, generator=g).bfloat16().float().to(dev)
    Wc = (torch.randn(32, 1, 4, 4, generator=g) * 0.1).to(dev)  # conv view [CO][C][kh][kw]
    bias = torch.tensor([0.05], device=dev)
    X = torch.rand(N, 128 * 128, generator=g).to(dev)
    G16 = G.permute(0, 2, 3, 1).contiguous().bfloat16()
    Wf = Wc.permute(0, 2, 3, 1).contiguous().flatten()  # [CO][4][4][1]
    y32 = torch.empty(N * 128 * 128, device=dev)
    dlog = torch.empty(N * 128 * 128, dtype=torch.bfloat16, device=dev)
    recon = torch.empty(N * 128 * 128, device=dev)
    part = torch.full((nb,), float("nan"), device=dev)
    gpart = torch.full((nb,), float("nan"), device=dev)
    C_.thin_tconv(G16, Wf, d, bias, y32=y32, X=X, dlog16=dlog, recon=recon, part=part, gpart=gpart)
    torch.cuda.synchronize()
    t = (F.conv_transpose2d(G, Wc, stride=2, padding=1) + bias).flatten()
    torch.testing.assert_close(y32, t, rtol=1e-5, atol=1e-5)
    p = torch.sigmoid(t)
    torch.testing.assert_close(recon, p, rtol=1e-5, atol=1e-6)
    torch.testing.assert_close(dlog.float(), (p - X.flatten()).bfloat16().float(), rtol=0, atol=1e-2)
    bce = F.binary_cross_entropy_with_logits(t, X.flatten(), reduction="sum")
    torch.testing.assert_close(part.double().sum(), bce.double(), rtol=1e-4, atol=1e-3)
    torch.testing.assert_close(gpart.double().sum(), (p - X.flatten()).double().sum(), rtol=1e-4, atol=1e-2)


@pytest.mark.parametrize("geom", [(64, 32, 64), (32, 64, 128)], ids=["64x32_to_64", "32x64_to_128"])
def test_direct_wgrad_matches_torch(geom, native_ext, monkeypatch):
    """Row-streamed direct weight gradient (conv_dwgrad.h): per-image partial
    rows [N][CO][4][4][C] summed in order == conv2d_weight in fp32 (the kernel
    accumulates bf16 products in f32; only the summation order differs)."""
    C_ = native_ext
    monkeypatch.setenv("MDT_DWGRAD_L2", "1")
    H, C, CO = geom
    OH = H // 2
    dev = torch.device("cuda")
    for N in (8, 5):  # XCD-grouped and plain workgroup order
        d = [N, H, H, C, OH, OH, CO, 4, 4, 2, 1]
        info = C_.wgrad_plan(d)
        assert info[0] >= 100 and info[6] == N, info
        g = torch.Generator(device="cpu").manual_seed(3 + N + H)
        X = torch.randn(N, C, H, H, generator=g).bfloat16().float().to(dev)
        G = torch.randn(N, CO, OH, OH, generator=g).bfloat16().float().to(dev)
        out = torch.full((N * CO * 16 * C,), float("nan"), device=dev)
        C_.wgrad(G.permute(0, 2, 3, 1).contiguous().bfloat16(), X.permute(0, 2, 3, 1).contiguous().bfloat16(), d,
                 out)
        torch.cuda.synchronize()
        assert torch.isfinite(out).all()
        got = out.view(N, CO * 16 * C).double().sum(0)
        ref = torch.nn.grad.conv2d_weight(X, (CO, C, 4, 4), G, stride=2, padding=1)  # [CO][C][4][4]
        ref = ref.permute(0, 2, 3, 1).reshape(-1).double()
        err = float((got - ref).abs().max() / ref.abs().max())
        assert err < 1e-5, (N, err)


@pytest.mark.parametrize("H", [128, 64], ids=["square", "h64"])
@pytest.mark.parametrize("f32_x", [True, False], ids=["f32_input", "bf16_dlogits"])
def test_thin_wgrad_mfma_matches_torch(f32_x, H, native_ext):
    """MFMA weight gradient of the single-channel 128x128 edge layers
    (conv_thin_wg.h): enc1 (X = f32 images) and the last layer's conv view
    (X = bf16 dlogits). One [32][16] partial row per 4 output rows; their sum
    equals conv2d_weight in f64 to the f32 accumulation (bf16 X exact; f32 X
    in three bf16 terms)."""
    C_ = native_ext
    dev = torch.device("cuda")
    N, W, CO = 3, 128, 32
    OH, OW = H // 2, W // 2
    d = [N, H, W, 1, OH, OW, CO, 4, 4, 2, 1]
    info = C_.wgrad_plan(d)
    assert info[0] == 110 and info[6] == N * OH // 4, info
    g = torch.Generator(device="cpu").manual_seed(11)
    X = torch.rand(N, 1, H, W, generator=g)
    if not f32_x:
        X = X - 0.5
        X = X.bfloat16().float()
    G = torch.randn(N, CO, OH, OW, generator=g).bfloat16().float()
    Xd = (X.flatten(1).contiguous() if f32_x else X.flatten(1).bfloat16().contiguous()).to(dev)
    G16 = G.permute(0, 2, 3, 1).contiguous().bfloat16().to(dev)
    ns = info[6]
    out = torch.full((ns * CO * 16,), float("nan"), device=dev)
    C_.wgrad(G16, Xd, d, out)
    torch.cuda.synchronize()
    assert torch.isfinite(out).all()
    ref = torch.nn.grad.conv2d_weight(X.double(), (CO, 1, 4, 4), G.double(), stride=2, padding=1).reshape(-1)
    mag = torch.nn.grad.conv2d_weight(X.double().abs(), (CO, 1, 4, 4), G.double().abs(), stride=2,
                                      padding=1).reshape(-1)
    tot = out.view(ns, CO * 16).double().sum(0).cpu()
    err = (tot - ref).abs()
    bound = mag * 2.0 ** -20
    assert bool((err <= bound + 1e-6).all()), float((err / (mag + 1e-9)).max())
