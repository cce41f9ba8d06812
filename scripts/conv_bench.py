"""A/B microbenchmark of dp_conv2d builds on DETRPose-L b64 conv shapes (development tool).

    python scripts/conv_bench.py [--libs lib1.so,lib2.so] [--shapes all|gemm|conv3] [--reps 20] [--rounds 3]

Every library is loaded side by side (ctypes, RTLD_LOCAL) and timed on the same random
bf16 operands in interleaved rounds in one process (guide §5.4 rule 24); hipBLASLt
(torch.mm) is timed beside the 1x1 shapes as a library reference point. Reports the
median over rounds of the mean µs per launch, TF/s and algorithmic TB/s.
"""
import argparse
import ctypes as C
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from detrpose_amd._lib import DP_BF16, ConvDesc  # noqa: E402

# name, batch, H, W, cin, cout, k, stride, act, residual
SHAPES = {
    "gemm": [
        ("fpn1.cv1", 64, 80, 80, 512, 512, 1, 1, 2, False),
        ("s2.sq", 64, 40, 40, 2176, 512, 1, 1, 1, False),
        ("fpn1.cv4", 64, 80, 80, 768, 256, 1, 1, 2, False),
        ("s1.sq", 64, 80, 80, 704, 256, 1, 1, 1, False),
        ("s0.sq", 64, 160, 160, 336, 64, 1, 1, 1, False),
        ("s0.ex", 64, 160, 160, 64, 128, 1, 1, 1, False),
        ("s1.ex", 64, 80, 80, 256, 512, 1, 1, 1, False),
        ("s2.ex+res", 64, 40, 40, 512, 1024, 1, 1, 1, True),
        ("enc_output", 64, 1, 8400, 256, 256, 1, 1, 0, False),
        ("dec.ffn1", 64, 1, 1080, 256, 1024, 1, 1, 1, False),
        ("dec.ffn2", 64, 1, 1080, 1024, 256, 1, 1, 0, False),
        ("dec.gate", 64, 1, 1080, 512, 512, 1, 1, 0, False),
        ("dec.out256", 64, 1, 1080, 256, 256, 1, 1, 0, False),
        ("dec.pose0", 64, 1, 1020, 256, 256, 1, 1, 1, False),
        ("dec.offattn", 64, 1, 1080, 256, 288, 1, 1, 0, False),
        ("dec.pose2", 64, 1, 1020, 256, 66, 1, 1, 0, False),
    ],
    "dw": [
        ("s1.down dw3s2", 64, 160, 160, 128, 128, 3, 2, 0, False),
        ("s2.down dw3s2", 64, 80, 80, 512, 512, 3, 2, 0, False),
        ("s2.l dw5", 64, 40, 40, 192, 192, 5, 1, 0, False),
        ("s3.l dw5", 64, 20, 20, 384, 384, 5, 1, 0, False),
    ],
    "conv3": [
        ("s0.l (48ch)", 64, 160, 160, 48, 48, 3, 1, 1, False),
        ("s0.l@336", 64, 160, 160, 48, 48, 3, 1, 1, False),
        ("s1.l@704", 64, 80, 80, 96, 96, 3, 1, 1, False),
        ("s1.l (96ch)", 64, 80, 80, 96, 96, 3, 1, 1, False),
        ("fpn1.vgg (128ch)", 64, 80, 80, 128, 128, 3, 1, 2, False),
        ("fpn0.vgg (128ch)", 64, 40, 40, 128, 128, 3, 1, 2, False),
        ("stem3 s2", 64, 320, 320, 64, 32, 3, 2, 1, False),
    ],
}


def load(path):
    lib = C.CDLL(path)
    for fn in (lib.dp_conv2d, lib.dp_dwconv2d):
        fn.restype = C.c_int32
        fn.argtypes = [C.POINTER(ConvDesc), C.c_void_p]
    return lib


def make(shape, dev):
    name, B, H, W, cin, cout, k, s, act, res = shape
    dw = " dw" in name
    # "name@P": input and output are channel slices of one concat buffer with P channels per
    # pixel (the HG-block layout: read slot [0, cin), write slot [cin, cin + cout))
    ps = int(name.split("@")[1]) if "@" in name else 0
    kpad = (k * k * cin + 63) // 64 * 64
    pad = (k - 1) // 2
    oh, ow = (H + 2 * pad - k) // s + 1, (W + 2 * pad - k) // s + 1
    x = torch.randn(B * H * W * (ps or cin), device=dev).to(torch.bfloat16)
    w = (torch.randn(cout, kpad, device=dev) / (k * k * cin) ** 0.5).to(torch.bfloat16)
    if dw:   # depthwise: f32 [k][k][C] weights
        w = torch.randn(k * k * cin, device=dev) / k
    b = torch.randn(cout, device=dev) * 0.05
    y = torch.empty(B * oh * ow * cout, device=dev, dtype=torch.bfloat16)
    r = torch.randn(B * oh * ow * cout, device=dev).to(torch.bfloat16) if res else None
    d = ConvDesc()
    d.in_, d.in_bstride, d.in_pstride, d.in_h, d.in_w, d.cin = x.data_ptr(), H * W * cin, cin, H, W, cin
    d.weight, d.kpad, d.bias = w.data_ptr(), kpad, b.data_ptr()
    d.kh, d.kw, d.stride, d.pad_t, d.pad_l = k, k, s, pad, pad
    d.out, d.out_bstride, d.out_pstride, d.out_h, d.out_w, d.cout = y.data_ptr(), oh * ow * cout, cout, oh, ow, cout
    if ps:
        assert (oh, ow) == (H, W)
        d.in_bstride, d.in_pstride = H * W * ps, ps
        d.out, d.out_bstride, d.out_pstride = x.data_ptr() + 2 * cin, H * W * ps, ps
    if r is not None:
        d.res, d.res_bstride, d.res_pstride = r.data_ptr(), oh * ow * cout, cout
    d.batch, d.act, d.dtype = B, act, DP_BF16
    M = B * oh * ow
    flops = 2.0 * M * cout * k * k * (1 if dw else cin)
    byts = 2.0 * (B * H * W * cin + (2 * k * k * cin if dw else cout * k * k * cin) + M * cout * (2 if res else 1))
    return d, (x, w, b, y, r), flops, byts, (M, cout, k * k * cin)


def time_it(fn, reps):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    fn()
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1e3 / reps


def main():
    ap = argparse.ArgumentParser()
    here = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    ap.add_argument("--libs", default=os.path.join(here, "detrpose_amd", "lib", "libdetrpose_hip.so"))
    ap.add_argument("--shapes", default="all")
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--no-blas", action="store_true")
    ap.add_argument("--check", action="store_true", help="compare every lib's output with the first lib's")
    ap.add_argument("--only", default="", help="comma-separated shape names (prefix match)")
    a = ap.parse_args()
    dev = torch.device("cuda")
    libs = [(os.path.basename(os.path.dirname(p)) or p, load(p)) for p in a.libs.split(",")]
    shapes = sum(SHAPES.values(), []) if a.shapes == "all" else SHAPES[a.shapes]
    if a.only:
        shapes = [sh for sh in shapes if any(sh[0].startswith(o) for o in a.only.split(","))]
    s = C.c_void_p(torch.cuda.current_stream().cuda_stream)
    print(f"{'shape':18s} {'M':>8s} {'N':>5s} {'K':>5s}  " + "  ".join(f"{n[:16]:>16s}" for n, _ in libs)
          + ("  hipBLASLt" if not a.no_blas else ""), flush=True)
    for sh in shapes:
        d, keep, flops, byts, (M, N, K) = make(sh, dev)
        res = {n: [] for n, _ in libs}
        res["blas"] = []
        outs = {}
        A = Wt = None
        if sh[6] == 1 and not a.no_blas:
            A = keep[0].view(M, K)
            Wt = keep[1].view(N, -1)[:, :K]
        for _ in range(a.rounds):
            for n, lib in libs:
                def f(lib=lib):
                    rc = (lib.dp_dwconv2d if " dw" in sh[0] else lib.dp_conv2d)(C.byref(d), s)
                    assert rc == 0, rc
                res[n].append(time_it(f, a.reps))
                if a.check and n not in outs:
                    outs[n] = keep[3].float().clone()
            if A is not None:
                res["blas"].append(time_it(lambda: torch.mm(A, Wt.t()), a.reps))
        cells = []
        for n, _ in libs:
            us = statistics.median(res[n])
            cells.append(f"{us:6.1f}us {flops / us / 1e6:5.0f}TF {byts / us / 1e6:4.2f}TB")
        line = f"{sh[0]:18s} {M:8d} {N:5d} {K:5d}  " + "  ".join(cells)
        if res["blas"]:
            us = statistics.median(res["blas"])
            line += f"  {us:6.1f}us {flops / us / 1e6:5.0f}TF"
        if a.check and len(outs) > 1:
            ref = outs[libs[0][0]]
            line += "  maxdiff " + ",".join(f"{(outs[n] - ref).abs().max().item():.2e}" for n, _ in libs[1:])
        print(line, flush=True)
        del keep


if __name__ == "__main__":
    main()
