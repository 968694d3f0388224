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
