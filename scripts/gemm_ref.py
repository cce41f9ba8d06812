"""Time torch.mm (hipBLASLt) on the DETRPose-L b64 1x1-conv GEMM shapes, for a library
reference point next to dp_conv2d's per-op times (not part of the product path)."""
import torch

SHAPES = [("enc.fpn1.cv1", 409600, 512, 512), ("s2.b2.sq", 102400, 512, 2176), ("enc.fpn1.cv4", 409600, 256, 768),
          ("s1.b0.sq", 409600, 256, 704), ("s1.b0.ex", 409600, 512, 256), ("s2.b1.ex", 102400, 1024, 512),
          ("s3.b0.sq", 25600, 1024, 3328), ("s0.b0.sq", 1638400, 64, 336), ("dec.ffn1", 69120, 1024, 256),
          ("vgg-as-gemm", 409600, 128, 1152), ("s0.l-as-gemm", 1638400, 48, 432)]


def main():
    dev = torch.device("cuda")
    for name, M, N, K in SHAPES:
        a = torch.randn(M, K, device=dev, dtype=torch.bfloat16)
        w = torch.randn(N, K, device=dev, dtype=torch.bfloat16)
        for _ in range(3):
            torch.mm(a, w.t())
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(10):
            torch.mm(a, w.t())
        e1.record()
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1) / 10
        fl = 2.0 * M * N * K
        by = 2.0 * (M * K + N * K + M * N)
        print(f"{name:14s} M={M:8d} N={N:5d} K={K:5d}  {ms:7.3f} ms  {fl / ms / 1e9:7.0f} TF/s  {by / ms / 1e9:6.2f} TB/s")


if __name__ == "__main__":
    main()
