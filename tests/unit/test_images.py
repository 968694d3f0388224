import numpy as np
import torch

from multidisttorch_amd.utils.images import make_grid, save_image, write_png


def test_grid_layout_like_torchvision():
    t = torch.rand(16, 1, 28, 28)
    g = make_grid(t, nrow=8)
    assert g.shape == (3, 2 + 2 * 30, 2 + 8 * 30)
    assert torch.equal(g[0, 2:30, 2:30], t[0, 0])


def test_png_files(tmp_path):
    save_image(torch.rand(64, 1, 28, 28), str(tmp_path / "a.png"))
    write_png(str(tmp_path / "b.png"), np.zeros((4, 5, 3), np.uint8))
    for n in ("a.png", "b.png"):
        assert (tmp_path / n).read_bytes()[:8] == b"\x89PNG\r\n\x1a\n"


def test_png_pixels_equal_torchvision_layout(tmp_path):
    """Single-channel grids are written as 8-bit RGB (the reference's
    torchvision format, mode 'RGB') with exactly the pixels of torchvision's
    grid (three equal planes), tail row included."""
    from PIL import Image

    t = torch.rand(13, 1, 20, 12)
    save_image(t, str(tmp_path / "g.png"), nrow=4)
    im = Image.open(tmp_path / "g.png")
    assert im.mode == "RGB"
    got = np.array(im)
    ref = make_grid(t, nrow=4).mul(255).add_(0.5).clamp_(0, 255).permute(1, 2, 0).to(torch.uint8).numpy()
    assert got.ndim == 3 and np.array_equal(got, ref) and np.array_equal(ref[..., 0], ref[..., 1])
    rgb = torch.rand(3, 3, 8, 8)
    save_image(rgb, str(tmp_path / "c.png"), nrow=2)
    got = np.array(Image.open(tmp_path / "c.png"))
    ref = make_grid(rgb, nrow=2).mul(255).add_(0.5).clamp_(0, 255).permute(1, 2, 0).to(torch.uint8).numpy()
    assert np.array_equal(got, ref)


def test_parallel_deflate_is_a_valid_zlib_stream(tmp_path):
    """Big grids are deflated in independent segments inside one zlib stream
    (utils/images.py::_deflate): zlib and PIL read it back exactly."""
    import zlib

    from PIL import Image

    from multidisttorch_amd.utils import images

    data = np.random.default_rng(0).integers(0, 8, 3 << 20, dtype=np.uint8).tobytes()
    assert len(data) >= images._DEFLATE_MIN_BYTES and images.PNG_DEFLATE_THREADS > 1
    assert zlib.decompress(images._deflate(data, 1)) == data
    t = torch.rand(64, 1, 128, 128)
    save_image(t, str(tmp_path / "big.png"))
    got = np.array(Image.open(tmp_path / "big.png"))
    ref = make_grid(t).mul(255).add_(0.5).clamp_(0, 255).permute(1, 2, 0).to(torch.uint8).numpy()
    assert np.array_equal(got, ref)
