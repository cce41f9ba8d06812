"""Time dp_stem_fused (the fused StemBlock) in isolation, side by side for several builds.

    python scripts/stem_bench.py [--libs a.so,b.so] [--batch 64] [--reps 20] [--cout 48]

Random image and weights at DETRPose-L's stem shapes; reports us per launch and the
algorithmic HBM rate (f32 image in, bf16 stem4 map out)."""
import argparse
import ctypes as C
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from detrpose_amd._lib import StemWeights  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    here = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    ap.add_argument("--libs", default=os.path.join(here, "detrpose_amd", "lib", "libdetrpose_hip.so"))
    ap.add_argument("--batch", type=int, default=64)
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--cout", type=int, default=48)
    a = ap.parse_args()
    dev = torch.device("cuda")
    B, H, W = a.batch, 640, 640
    g = torch.Generator(device="cuda").manual_seed(0)
    img = torch.rand(B, 3, H, W, device=dev, generator=g)

    def wt(co, k, kp):
        w = torch.zeros(co, kp, device=dev)
        w[:, :k] = torch.randn(co, k, device=dev, generator=g) / k ** 0.5
        return w.to(torch.bfloat16).contiguous()

    keep = dict(w1=torch.randn(32, 27, device=dev, generator=g) / 5, b1=torch.randn(32, device=dev, generator=g) * 0.1,
                w2a=wt(16, 128, 128), b2a=torch.randn(16, device=dev, generator=g) * 0.1,
                w2b=wt(32, 64, 64), b2b=torch.randn(32, device=dev, generator=g) * 0.1,
                w3=wt(32, 576, 576), b3=torch.randn(32, device=dev, generator=g) * 0.1,
                w4=wt(a.cout, 32, 64), b4=torch.randn(a.cout, device=dev, generator=g) * 0.1)
    sw = StemWeights()
    for k, v in keep.items():
        setattr(sw, k, v.data_ptr())
    sw.k2a, sw.k2b, sw.k3, sw.k4, sw.mid, sw.cout, sw.has_lab = 128, 64, 576, 64, 32, a.cout, 0
    out = torch.empty(B, 160, 160, a.cout, device=dev, dtype=torch.bfloat16)
    s = C.c_void_p(torch.cuda.current_stream().cuda_stream)
    byts = 4.0 * B * 3 * H * W + 2.0 * out.numel()
    for path in a.libs.split(","):
        lib = C.CDLL(path)
        fn = lib.dp_stem_fused
        fn.restype = C.c_int32
        fn.argtypes = [C.c_void_p, C.c_int32, C.c_int32, C.c_int32, C.POINTER(StemWeights), C.c_void_p, C.c_int64,
                       C.c_int32, C.c_void_p]

        def call():
            rc = fn(img.data_ptr(), B, H, W, C.byref(sw), out.data_ptr(), 160 * 160 * a.cout, a.cout, s)
            assert rc == 0, rc
        call()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(a.reps):
            call()
        e1.record()
        torch.cuda.synchronize()
        us = e0.elapsed_time(e1) * 1e3 / a.reps
        print(f"{os.path.basename(os.path.dirname(path)):>12s}: {us:7.1f} us  {byts / us / 1e6:5.2f} TB/s  "
              f"checksum {out.float().abs().sum().item():.6e}", flush=True)


if __name__ == "__main__":
    main()
