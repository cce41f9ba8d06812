"""Time dp_msda (bf16 wave kernel) in isolation at a config's decoder shape.

    python scripts/msda_bench.py [--size l] [--batch 64] [--reps 50]

Inputs: random bf16 memory, reference points uniform in [0.05, 0.95], sampling offsets
N(0, 2) pixels, attention logits N(0, 1). Prints us per call and the algorithmic GB/s
(SURVEY.md §8d bytes) and the gathered bytes rate (4 corners x L x P x C x 2 B per token).
"""
import argparse
import ctypes as C
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--size", default="l")
    ap.add_argument("--batch", type=int, default=64)
    ap.add_argument("--reps", type=int, default=50)
    a = ap.parse_args()
    from detrpose_amd import _lib
    geo = {"n": (128, [(80, 80), (40, 40)], 6, 8), "l": (256, [(80, 80), (40, 40), (20, 20)], 4, 8),
           "x": (384, [(80, 80), (40, 40), (20, 20)], 4, 8)}[a.size]
    Cc, shapes, P, nH = geo
    L = len(shapes)
    S = sum(h * w for h, w in shapes)
    B, lq = a.batch, 60 * 18
    rows = B * lq
    g = torch.Generator(device="cuda").manual_seed(0)
    val = torch.randn(B, S, Cc, device="cuda", generator=g).to(torch.bfloat16)
    ncol = nH * L * P * 3
    oa = torch.empty(rows, ncol, device="cuda")
    oa[:, :nH * L * P * 2] = torch.randn(rows, nH * L * P * 2, device="cuda", generator=g) * 2
    oa[:, nH * L * P * 2:] = torch.randn(rows, nH * L * P, device="cuda", generator=g)
    oa = oa.to(torch.bfloat16)
    ref = torch.rand(rows, 2, device="cuda", generator=g) * 0.9 + 0.05
    out = torch.empty(rows, Cc, device="cuda", dtype=torch.bfloat16)
    hw = (C.c_int32 * (2 * L))(*[v for s in shapes for v in s])
    lib = _lib.load()
    st = torch.cuda.current_stream().cuda_stream

    def call():
        _lib.check(lib.dp_msda(val.data_ptr(), B, S, hw, L, oa.data_ptr(), ref.data_ptr(), out.data_ptr(), Cc, lq, nH,
                               Cc // nH, P, _lib.DP_BF16, C.c_void_p(st)), "dp_msda")

    for _ in range(5):
        call()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(a.reps):
        call()
    e1.record()
    torch.cuda.synchronize()
    us = e0.elapsed_time(e1) * 1e3 / a.reps
    alg = 2 * (B * S * Cc + rows * ncol + rows * Cc) + 4 * rows * 2
    gath = rows * nH * L * P * 4 * (Cc // nH) * 2
    print(f"msda {a.size} b{B}: {us:.1f} us/call  algorithmic {alg / us / 1e3:.0f} GB/s  "
          f"gathered {gath / us / 1e3:.0f} GB/s  checksum {out.float().abs().sum().item():.6e}")


if __name__ == "__main__":
    main()
