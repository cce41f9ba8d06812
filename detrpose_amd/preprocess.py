"""GPU input pipeline of the reference benchmark.

`tools/benchmark/dataset.py:56-61`: T.Resize(size=639, max_size=640) -> PadToSize((640, 640),
fill=114) -> ToTensor -> ConvertImageDtype(float), on images decoded to uint8 RGB (3, h, w)
tensors on the device (`dataset.py:74-75`). `preprocess(images)` runs it with one
`dp_resize_pad` launch per image straight into the (B, 3, 640, 640) f32 model input, and
returns `orig_target_sizes` (B, 2) = [w, h] as the dataset's blob does (`dataset.py:84`).
JPEG decoding stays with the caller (torchvision.io / rocJPEG are not part of this path).
"""
from __future__ import annotations

import ctypes as C

import torch

from . import _lib


def resized_size(h: int, w: int, size: int = 639, max_size: int = 640) -> tuple[int, int]:
    """T.Resize(size, max_size) output (new_h, new_w) for an int size: the shorter side to
    `size`, the longer one scaled (truncated), capped at `max_size` with the shorter side
    rescaled (torchvision's _compute_resized_output_size)."""
    short, long = (w, h) if w <= h else (h, w)
    new_short, new_long = size, int(size * long / short)
    if max_size is not None and new_long > max_size:
        new_short, new_long = int(max_size * new_short / new_long), max_size
    new_w, new_h = (new_short, new_long) if w <= h else (new_long, new_short)
    return new_h, new_w


def preprocess(images, size: int = 639, max_size: int = 640, pad_to=(640, 640), fill: float = 114.0,
               out: torch.Tensor | None = None):
    """images: sequence of uint8 (3, h, w) CUDA tensors (any sizes). Returns (batch f32
    (B, 3, pad_h, pad_w), orig_target_sizes int64 (B, 2) = [w, h])."""
    if len(images) == 0:
        raise ValueError("preprocess: no images")
    dev = images[0].device
    if dev.type != "cuda":
        raise RuntimeError("preprocess: images must be on the GPU (no CPU path)")
    ph, pw = pad_to
    if out is None:
        out = torch.empty(len(images), 3, ph, pw, device=dev, dtype=torch.float32)
    if out.shape != (len(images), 3, ph, pw) or out.dtype != torch.float32 or not out.is_contiguous():
        raise ValueError(f"preprocess: out must be contiguous f32 {(len(images), 3, ph, pw)}")
    if out.device != dev:
        raise ValueError(f"preprocess: out is on {out.device}, images on {dev}")
    lib = _lib.load()
    s = C.c_void_p(torch.cuda.current_stream(dev).cuda_stream)
    sizes = []
    for b, im in enumerate(images):
        if im.dtype != torch.uint8 or im.dim() != 3 or im.shape[0] != 3:
            raise ValueError(f"preprocess: image {b} must be uint8 (3, h, w), got {im.dtype} {tuple(im.shape)}")
        if im.device != dev:
            raise ValueError(f"preprocess: image {b} is on {im.device}, image 0 on {dev}: one GPU per call")
        im = im.contiguous()
        h, w = int(im.shape[1]), int(im.shape[2])
        nh, nw = resized_size(h, w, size, max_size)
        _lib.check(lib.dp_resize_pad(im.data_ptr(), h, w, nh, nw, out[b].data_ptr(), ph, pw, C.c_float(fill), s),
                   "dp_resize_pad")
        sizes.append((w, h))
    return out, torch.tensor(sizes, dtype=torch.int64, device=dev)
