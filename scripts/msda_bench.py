"""Time dp_msda (bf16 wave kernel) in isolation at a config's decoder shape.

    python scripts/msda_bench.py [--size l] [--batch 64] [--reps 50] [--libs a.so,b.so] [--rounds 3]

With --libs, the libraries are timed interleaved (rounds x reps each) and their outputs compared
with the first one's (max |diff|).

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
    ap.add_argument("--libs", default="")
    ap.add_argument("--rounds", type=int, default=1)
    ap.add_argument("--refs", default="random", choices=["random", "clustered", "sorted"],
                    help="reference points: uniform per token; 60 person centres per image with their 18 "
                         "tokens within +-0.05 (the decoder's layout); or clustered with the queries "
                         "ordered by centre y (a spatial token order)")
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
    if a.refs == "random":
        ref = torch.rand(rows, 2, device="cuda", generator=g) * 0.9 + 0.05
    else:
        ctr = torch.rand(B, 60, 1, 2, device="cuda", generator=g) * 0.8 + 0.1
        if a.refs == "sorted":
            order = ctr[:, :, 0, 1].argsort(dim=1)
            ctr = torch.gather(ctr, 1, order[:, :, None, None].expand_as(ctr))
        ref = (ctr + (torch.rand(B, 60, 18, 2, device="cuda", generator=g) - 0.5) * 0.1).reshape(rows, 2).contiguous()
    out = torch.empty(rows, Cc, device="cuda", dtype=torch.bfloat16)
    hw = (C.c_int32 * (2 * L))(*[v for s in shapes for v in s])
    libs = []
    if a.libs:
        for path in a.libs.split(","):
            lb = C.CDLL(path)
            lb.dp_msda.restype = C.c_int32
            lb.dp_msda.argtypes = _lib._SIGS["dp_msda"][1]
            libs.append((os.path.basename(os.path.dirname(path)) or path, lb))
    else:
        libs.append(("lib", _lib.load()))
    st = torch.cuda.current_stream().cuda_stream

    def call(lib):
        rc = lib.dp_msda(val.data_ptr(), B, S, hw, L, oa.data_ptr(), ref.data_ptr(), out.data_ptr(), Cc, lq, nH,
                         Cc // nH, P, _lib.DP_BF16, C.c_void_p(st))
        if rc:
            raise RuntimeError(f"dp_msda rc={rc}")

    times = {n: [] for n, _ in libs}
    outs = {}
    for rnd in range(a.rounds):
        for n, lib in libs:
            for _ in range(5):
                call(lib)
            torch.cuda.synchronize()
            if rnd == 0:
                outs[n] = out.float().clone()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(a.reps):
                call(lib)
            e1.record()
            torch.cuda.synchronize()
            times[n].append(e0.elapsed_time(e1) * 1e3 / a.reps)
    ref0 = outs[libs[0][0]]
    for n, _ in libs:
        us = min(times[n])
        alg = 2 * (B * S * Cc + rows * ncol + rows * Cc) + 4 * rows * 2
        gath = rows * nH * L * P * 4 * (Cc // nH) * 2
        print(f"[{n}] msda {a.size} b{B}: {us:.1f} us/call (rounds {', '.join(f'{t:.1f}' for t in times[n])})  "
              f"algorithmic {alg / us / 1e3:.0f} GB/s  gathered {gath / us / 1e3:.0f} GB/s  "
              f"checksum {outs[n].abs().sum().item():.6e}  maxdiff vs first {(outs[n] - ref0).abs().max().item():.3e}")


if __name__ == "__main__":
    main()
