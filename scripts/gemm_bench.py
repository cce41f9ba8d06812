"""Times dp_gemm on the training step's weight-gradient shapes (dW = dz^T col: M = cout, N =
cin*k*k, K = B*H*W) over split-K counts, HIP events on the launch stream.

    python scripts/gemm_bench.py [--reps 10]
"""
import argparse
import ctypes as C
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=10)
    a = ap.parse_args()
    from detrpose_amd import _lib
    from detrpose_amd._lib import GemmDesc
    lib = _lib.load()
    dev = torch.device("cuda")
    sp = C.c_void_p(torch.cuda.current_stream().cuda_stream)
    # (name, m, n, k)
    shapes = [("bb.s1.layer", 48, 432, 16 * 160 * 160), ("bb.s2.layer", 96, 864, 16 * 80 * 80),
              ("bb.s2.agg", 512, 1024, 16 * 80 * 80), ("enc.vgg3x3", 128, 1152, 16 * 80 * 80),
              ("enc.vgg3x3.40", 128, 1152, 16 * 40 * 40)]
    for name, m, n, k in shapes:
        dz = torch.randn(k, m, device=dev).bfloat16()
        col = torch.randn(k, n, device=dev).bfloat16()
        out = torch.zeros(m, n, device=dev)
        res = []
        for split in (0, 4, 8, 16, 32, 64, 128, 512):
            d = GemmDesc()
            d.a, d.a_bs, d.a_rs, d.a_ks = dz.data_ptr(), 0, 1, m
            d.b, d.b_bs, d.b_ks, d.b_ns = col.data_ptr(), 0, n, 1
            d.c, d.c_bs, d.c_rs = out.data_ptr(), 0, n
            d.batch, d.m, d.n, d.k = 1, m, n, k
            d.in_dtype, d.out_dtype = 1, 0
            d.bias, d.alpha, d.beta, d.act, d.gate = None, 1.0, 1.0, 0, None
            d.split_k = split
            fn = lambda: _lib.check(lib.dp_gemm(C.byref(d), sp), "gemm")   # noqa: E731
            fn()
            torch.cuda.synchronize()
            ts = []
            for _ in range(a.reps):
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                fn()
                e1.record()
                torch.cuda.synchronize()
                ts.append(e0.elapsed_time(e1))
            t = sorted(ts)[len(ts) // 2] * 1e3
            res.append(f"split {split}: {t:7.1f} us {2.0 * m * n * k / t / 1e6:6.1f} TF")
        print(f"{name:14s} m{m} n{n} k{k}: " + " | ".join(res), flush=True)
    # nn.Linear forward shapes of the decoder (rows = B * Qt * 18 at L b16): dp_gemm vs the 1x1
    # conv kernel on the same operands (weights [N][K] = the conv's packed layout when K % 64 == 0)
    from detrpose_amd._lib import ConvDesc
    rows = 16 * 96 * 18
    for K, N in ((256, 1024), (1024, 256), (256, 768), (512, 512), (256, 256)):
        x = torch.randn(rows, K, device=dev).bfloat16()
        W = torch.randn(N, K, device=dev).bfloat16()
        bias = torch.randn(N, device=dev)
        out = torch.empty(rows, N, device=dev).bfloat16()
        d = GemmDesc()
        d.a, d.a_bs, d.a_rs, d.a_ks = x.data_ptr(), 0, K, 1
        d.b, d.b_bs, d.b_ks, d.b_ns = W.data_ptr(), 0, 1, K
        d.c, d.c_bs, d.c_rs = out.data_ptr(), 0, N
        d.batch, d.m, d.n, d.k = 1, rows, N, K
        d.in_dtype, d.out_dtype = 1, 1
        d.bias, d.alpha, d.beta, d.act, d.gate, d.split_k = bias.data_ptr(), 1.0, 0.0, 1, None, 0
        cd = ConvDesc()
        cd.in_, cd.in_bstride, cd.in_pstride, cd.in_h, cd.in_w, cd.cin = x.data_ptr(), rows * K, K, 1, rows, K
        cd.weight, cd.kpad, cd.bias = W.data_ptr(), K, bias.data_ptr()
        cd.kh, cd.kw, cd.stride, cd.pad_t, cd.pad_l = 1, 1, 1, 0, 0
        cd.out, cd.out_bstride, cd.out_pstride, cd.out_h, cd.out_w, cd.cout = out.data_ptr(), rows * N, N, 1, rows, N
        cd.batch, cd.act, cd.dtype = 1, 1, 1
        ts = {}
        for tag, fn in (("gemm", lambda: _lib.check(lib.dp_gemm(C.byref(d), sp), "g")),
                        ("conv", lambda: _lib.check(lib.dp_conv2d(C.byref(cd), sp), "c"))):
            fn()
            torch.cuda.synchronize()
            tt = []
            for _ in range(a.reps):
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                fn()
                e1.record()
                torch.cuda.synchronize()
                tt.append(e0.elapsed_time(e1))
            ts[tag] = sorted(tt)[len(tt) // 2] * 1e3
        fl = 2.0 * rows * K * N
        print(f"linear rows {rows} K {K} N {N}: dp_gemm {ts['gemm']:7.1f} us ({fl / ts['gemm'] / 1e6:5.0f} TF)  "
              f"dp_conv2d {ts['conv']:7.1f} us ({fl / ts['conv'] / 1e6:5.0f} TF)", flush=True)


if __name__ == "__main__":
    main()
