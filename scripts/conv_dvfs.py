"""Is the 128-channel 3x3 conv (conv_halo_kernel, L b64 encoder shape) clock-bound? Same
launch on random vs all-zero operands (MI355X_MICROARCH.md 'DVFS give-back' (1): the chip
holds a higher clock when the MFMA operands do not toggle). Interleaved rounds, one process."""
import ctypes as C
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from detrpose_amd import _lib
from detrpose_amd._lib import ConvDesc
from detrpose_amd.engine import Packer


def main():
    B, cin, H, W = 64, 128, 80, 80
    pk = Packer({}, "bf16", torch.device("cuda"))
    w = torch.randn(128, cin, 3, 3) / (cin * 9) ** 0.5
    pcs = {"random w": pk.conv(w.double(), torch.zeros(128).double(), act="silu"),
           "zero w": pk.conv(torch.zeros_like(w).double(), torch.zeros(128).double(), act="silu")}
    xs = {"random x": torch.randn(B, H, W, cin, device="cuda").bfloat16(),
          "zero x": torch.zeros(B, H, W, cin, device="cuda", dtype=torch.bfloat16)}
    out = torch.empty(B, H, W, 128, device="cuda", dtype=torch.bfloat16)
    lib = _lib.load()
    s = C.c_void_p(torch.cuda.current_stream().cuda_stream)
    flops = 2 * B * H * W * 128 * 9 * cin
    for rnd in range(3):
        for wn, pc in pcs.items():
            for xn, x in xs.items():
                d = ConvDesc()
                d.in_, d.in_bstride, d.in_pstride, d.in_h, d.in_w, d.cin = x.data_ptr(), H * W * cin, cin, H, W, cin
                d.weight, d.kpad, d.bias = pc.w.data_ptr(), pc.kpad, pc.b.data_ptr()
                d.kh, d.kw, d.stride, d.pad_t, d.pad_l = 3, 3, 1, 1, 1
                d.out, d.out_bstride, d.out_pstride, d.out_h, d.out_w, d.cout = \
                    out.data_ptr(), H * W * 128, 128, H, W, 128
                d.batch, d.act, d.dtype = B, pc.act, _lib.DP_BF16
                for _ in range(20):
                    lib.dp_conv2d(C.byref(d), s)
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for _ in range(50):
                    lib.dp_conv2d(C.byref(d), s)
                e1.record()
                torch.cuda.synchronize()
                us = e0.elapsed_time(e1) * 1e3 / 50
                print(f"round {rnd} {wn:9s} {xn:9s} {us:7.1f} us {flops / us / 1e6:6.0f} TF/s", flush=True)


if __name__ == "__main__":
    main()
