"""Deterministic synthetic weights and images.

There is no network, so no released checkpoint and no COCO data.
Weights are a seeded fan-in random re-initialisation, generated per state_dict key
from numpy's counter-based generator, so the same key/shape gives the same tensor on
every machine: the golden-fixture generator (tests/golden/make_golden.py), the
tests and bench.py all reproduce identical models without shipping weights.

The reference's default init is degenerate (zero-initialised last layers make all
17 keypoints of a query identical; SURVEY.md header fact 4), which is why a random
re-init is used instead.
"""
from __future__ import annotations

import zlib

import numpy as np
import torch

# Buffers whose values are defined by the architecture, not learned; the
# constructors compute them and the synthetic init leaves them alone.
#  transformer.up / reg_scale: transformer.py:1114-1116 (requires_grad=False params)
#  transformer.anchors / valid_mask: transformer.py:1136-1139
#  transformer.decoder.dim_t: transformer.py:501-503
FIXED_KEYS = ("transformer.up", "transformer.reg_scale", "transformer.anchors",
              "transformer.valid_mask", "transformer.decoder.dim_t")


def _rng(key: str, seed: int) -> np.random.Generator:
    return np.random.default_rng([int(seed), zlib.crc32(key.encode())])


def synthetic_tensor(key: str, shape, seed: int = 0) -> torch.Tensor:
    shape = tuple(int(s) for s in shape)
    r = _rng(key, seed)
    n = int(np.prod(shape)) if shape else 1
    leaf = key.rsplit(".", 1)[-1]
    if leaf == "running_var":
        v = r.uniform(0.5, 1.5, n)
    elif leaf == "running_mean":
        v = 0.05 * r.standard_normal(n)
    elif len(shape) >= 2:
        fan_in = int(np.prod(shape[1:]))
        v = r.standard_normal(n) / np.sqrt(fan_in)
    elif leaf in ("weight", "scale"):
        # 1-D weights are norm scales (BN / LN) or the LAB scale
        v = 1.0 + 0.05 * r.standard_normal(n)
    else:
        v = 0.05 * r.standard_normal(n)
    return torch.from_numpy(v.astype(np.float32).reshape(shape))


def synthetic_state_dict(shapes: dict, seed: int = 0) -> dict:
    """Generate a state_dict for every key in `shapes` except FIXED_KEYS and
    integer bookkeeping buffers (num_batches_tracked)."""
    out = {}
    for key in sorted(shapes):
        if key in FIXED_KEYS or key.endswith("num_batches_tracked"):
            continue
        out[key] = synthetic_tensor(key, shapes[key], seed)
    return out


def synthetic_images(batch: int, seed: int = 1, size: int = 640) -> torch.Tensor:
    """Uniform [0,1) fp32 images (B,3,size,size); the reference feeds un-normalised
    [0,1] images (configs/detrpose/include/dataset.py:38,61)."""
    r = np.random.default_rng([int(seed), 0xD7])
    return torch.from_numpy(r.random((batch, 3, size, size), dtype=np.float32))


def load_synthetic(module: torch.nn.Module, seed: int = 0) -> torch.nn.Module:
    """Fill `module` (reference-compatible key layout) with synthetic weights."""
    shapes = {k: tuple(v.shape) for k, v in module.state_dict().items()}
    sd = synthetic_state_dict(shapes, seed)
    missing, unexpected = module.load_state_dict(sd, strict=False)
    bad = [k for k in missing if k not in FIXED_KEYS and not k.endswith("num_batches_tracked")]
    if bad or unexpected:
        raise RuntimeError(f"synthetic load mismatch: missing={bad} unexpected={unexpected}")
    return module
