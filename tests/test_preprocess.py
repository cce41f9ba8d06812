"""Input pipeline (dp_resize_pad / detrpose_amd.preprocess) vs the CPU restatement
(oracle/preprocess_cpu.py: ATen antialiased bilinear, as torchvision's tensor resize calls it;
torchvision itself is not importable here, so parity vs torchvision is unpinned).
Tolerance: uint8 levels, i.e. multiples of 1/255: at most 1 level where the float sums land
on a .5 rounding tie in a different order, and >= 99.9% of values exact."""
import pytest
import torch

from detrpose_amd.preprocess import resized_size
from oracle.preprocess_cpu import resize_pad_cpu


@pytest.mark.parametrize("h,w,exp", [(480, 640, (480, 640)), (1080, 1920, (360, 640)), (640, 427, (640, 427)),
                                     (500, 375, (640, 480)), (639, 639, (639, 639)), (100, 50, (640, 320)),
                                     (2000, 300, (640, 96))])
def test_resized_size(h, w, exp):
    """T.Resize(639, max_size=640): shorter side 639 unless the longer would pass 640."""
    assert resized_size(h, w) == exp


@pytest.mark.gpu
@pytest.mark.parametrize("h,w", [(1080, 1920), (480, 640), (375, 500), (333, 211), (900, 300), (639, 639)])
def test_resize_pad_gpu(h, w):
    from detrpose_amd.preprocess import preprocess
    g = torch.Generator().manual_seed(h * w)
    img = torch.randint(0, 256, (3, h, w), generator=g, dtype=torch.uint8)
    # smooth + sharp content: a gradient with noise and a hard edge
    img[:, : h // 2] = (torch.arange(w) * 255 // max(1, w - 1)).to(torch.uint8)
    nh, nw = resized_size(h, w)
    ref = resize_pad_cpu(img, nh, nw)
    out, sizes = preprocess([img.cuda(), img.cuda()])
    torch.cuda.synchronize()
    assert sizes.tolist() == [[w, h], [w, h]]
    for b in range(2):
        d = (out[b].cpu() - ref).abs() * 255
        assert d.max().item() <= 1.0 + 1e-3, f"max {d.max().item()} levels"
        assert (d < 1e-3).float().mean().item() >= 0.999
        assert (out[b, :, nh:, :].cpu() == 114 / 255).all() and (out[b, :, :, nw:].cpu() == 114 / 255).all()


@pytest.mark.gpu
def test_resize_pad_rejects_mixed_devices():
    """Every image (not just the first) and `out` must sit on the first image's GPU."""
    from detrpose_amd.preprocess import preprocess
    img = torch.zeros(3, 40, 50, dtype=torch.uint8)
    with pytest.raises(ValueError, match="image 1"):
        preprocess([img.cuda(), img])
    with pytest.raises(ValueError, match="out is on"):
        preprocess([img.cuda()], out=torch.empty(1, 3, 640, 640))
