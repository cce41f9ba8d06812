"""Times dp_dwconv2d forward on the inference plan's depthwise shapes (HGNetv2-L b64, bf16),
HIP events on the launch stream, with an output checksum (kernel variants must agree bit for
bit; the round-5 variant table is profiles/r5_dw5_ab.txt).

    python scripts/dw_fwd_bench.py [--reps 50]
"""
import argparse
import ctypes as C
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=50)
    ap.add_argument("--batch", type=int, default=64)
    ap.add_argument("--libs", default="", help="comma list of library builds to time side by side (A/B)")
    a = ap.parse_args()
    from detrpose_amd import _lib
    from detrpose_amd._lib import ConvDesc
    libs = [("lib", _lib.load())]
    for path in filter(None, a.libs.split(",")):
        v = C.CDLL(path)
        v.dp_dwconv2d.restype = C.c_int32
        v.dp_dwconv2d.argtypes = [C.POINTER(ConvDesc), C.c_void_p]
        libs.append((os.path.basename(os.path.dirname(path)), v))
    dev = torch.device("cuda")
    st = torch.cuda.current_stream()
    B = a.batch
    for (h, c), (tag, lib) in [(hc, l) for hc in ((40, 192), (20, 384)) for l in libs]:
        torch.manual_seed(h)
        x = torch.randn(B, h, h, c, device=dev).bfloat16()
        y = torch.empty_like(x)
        w = torch.randn(25, c, device=dev)
        bias = torch.randn(c, device=dev)
        d = ConvDesc()
        d.in_, d.in_bstride, d.in_pstride, d.in_h, d.in_w, d.cin = x.data_ptr(), h * h * c, c, h, h, c
        d.weight, d.bias, d.kh, d.kw, d.stride, d.pad_t, d.pad_l = w.data_ptr(), bias.data_ptr(), 5, 5, 1, 2, 2
        d.out, d.out_bstride, d.out_pstride, d.out_h, d.out_w, d.cout = y.data_ptr(), h * h * c, c, h, h, c
        d.batch, d.act, d.dtype = B, _lib.DP_ACT_RELU, _lib.DP_BF16
        sp = C.c_void_p(st.cuda_stream)
        run = lambda: _lib.check(lib.dp_dwconv2d(C.byref(d), sp), "dw")
        for _ in range(5):
            run()
        torch.cuda.synchronize()
        ts = []
        for _ in range(a.reps):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(st)
            run()
            e1.record(st)
            torch.cuda.synchronize()
            ts.append(e0.elapsed_time(e1) * 1e3)
        t = sorted(ts)[len(ts) // 2]
        mb = 2 * x.numel() * 2 / 1e6
        chk = int(y.view(torch.int16).to(torch.int64).sum())   # variants must agree bit for bit
        print(f"{tag:>6s} dw5 {h}x{h} c{c} b{B}: {t:7.1f} us  {mb / t:6.2f} TB/s (in + out)  out checksum {chk}",
              flush=True)


if __name__ == "__main__":
    main()
