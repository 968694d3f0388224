"""Host-side native runtime on CPU: the conv planners of csrc/runtime/conv_ops.cpp
(tile / split-K / wgrad grid choices) for every layer of both conv-VAEs at
awkward batch sizes. Runs in the normal CPU suite and under the ASan/UBSan
build (scripts/sanitize_host.sh, MDT_NATIVE_SO=build/san/_C.so), where an
out-of-bounds table access or signed overflow in a planner aborts the test."""
import pytest

from multidisttorch_amd.ops import native

pytestmark = pytest.mark.skipif(not native.available(), reason="native extension not built")


def _descs(image, M):
    from multidisttorch_amd.models.conv_vae import ConvVaeTrainer, conv_vae_spec

    spec = conv_vae_spec(image, 1, 32 if image == 28 else 64)
    return [(l, ConvVaeTrainer._desc(l, M)) for l in spec]


@pytest.mark.parametrize("image", [28, 128])
@pytest.mark.parametrize("M", [1, 7, 64, 128, 129, 1000])
def test_conv_planners_consistent(image, M):
    C = native.require()
    for l, d in _descs(image, M):
        if l.cin == 1 or l.cout == 1:
            nb = C.thin_blocks(l.kind == "convT", d)
            assert nb > 0
            if l.kind != "convT":
                continue
        modes = [0, 1]
        for mode in modes:
            for split in (False, True):
                try:
                    q = C.igemm_plan(mode, d, split)
                except RuntimeError as e:
                    assert "unsupported geometry" in str(e)
                    continue
                classes, rows, ncols, K, ks, csrows = q[3], q[4], q[5], q[6], q[10], q[11]
                assert classes >= 1 and rows >= 1 and ncols >= 1 and K >= 1
                assert ks >= 1 and (split or ks == 1)
                assert csrows >= 1
        w = C.wgrad_plan(d)
        assert w[6] >= 1  # m-splits (partial slabs)
        assert all(v >= 0 for v in w)
    for ks in (1, 2, 8):
        assert C.combine_reparam_blocks(ks, M, 32) >= 1


@pytest.mark.parametrize("M", [1, 7, 64, 128])
def test_thin_mfma_wgrad_plan(M):
    """The single-channel 128x128 layers (enc1, and the last layer in its conv
    view) plan the MFMA weight gradient (conv_thin_wg.h, cfg 110): one partial
    row per 4 output rows, i.e. M * 64 / 4 slabs of [32][16]; the 28x28 edge
    layers keep the generic thin weight gradient."""
    import os

    C = native.require()
    if os.environ.get("MDT_THIN_MFMA", "15") not in ("14", "15"):
        pytest.skip("non-default MDT_THIN_MFMA mask")
    for image in (28, 128):
        for l, d in _descs(image, M):
            if not (l.cin == 1 or l.cout == 1):
                continue
            info = C.wgrad_plan(d)
            if image == 128:
                assert info[0] == 110 and info[6] == M * 64 // 4 and info[1] == 32 and info[2] == 16, info
            else:
                assert info[0] != 110, info
