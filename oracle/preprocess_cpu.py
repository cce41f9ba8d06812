"""ORACLE — TEST INFRASTRUCTURE ONLY: CPU restatement of the reference benchmark's input
pipeline (tools/benchmark/dataset.py:56-61) for checking detrpose_amd.preprocess.

T.Resize on a uint8 tensor off the CPU is torchvision's float path: the image as float,
F.interpolate(bilinear, align_corners=False, antialias=True) (ATen _upsample_bilinear2d_aa),
round, clamp, back to uint8; PadToSize pads right / bottom with the fill; ConvertImageDtype
divides by 255. torchvision is not importable here, so this is pinned to the ATen op that
torchvision calls, not to torchvision itself (parity vs torchvision unpinned).
"""
from __future__ import annotations

import torch
import torch.nn.functional as F


def resize_pad_cpu(img_u8: torch.Tensor, new_h: int, new_w: int, pad_h: int = 640, pad_w: int = 640,
                   fill: float = 114.0) -> torch.Tensor:
    x = img_u8.float()[None]
    if (new_h, new_w) != tuple(img_u8.shape[1:]):
        x = F.interpolate(x, size=(new_h, new_w), mode="bilinear", align_corners=False, antialias=True)
    x = x.round().clamp(0, 255)[0]
    out = torch.full((3, pad_h, pad_w), fill, dtype=torch.float32)
    out[:, :new_h, :new_w] = x
    return out / 255.0
