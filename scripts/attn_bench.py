"""Times the training attention core (dp_attn_fwd / dp_attn_bwd) on the training step's shapes
(DETRPose-L b16: within-instance 18 tokens, across-instance Qt queries with the DN mask, AIFI 400
tokens) with HIP events on the launch stream; median of --reps.

    python scripts/attn_bench.py [--reps 20] [--dtype bf16]
"""
import argparse
import ctypes as C
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--dtype", default="bf16")
    a = ap.parse_args()
    from detrpose_amd import _lib
    lib = _lib.load()
    code = 1 if a.dtype == "bf16" else 0
    dt = torch.bfloat16 if code else torch.float32
    dev = torch.device("cuda")
    s = torch.cuda.current_stream()
    sp = C.c_void_p(s.cuda_stream)
    B, T, Qt, C_, nh = 16, 18, 96, 256, 8
    cases = {
        # name: (rows, n_outer, n_inner, so, si, st, L, masked, C)
        "within": (B * Qt * T, B * Qt, 1, T, 0, 1, T, False, C_),
        "across": (B * Qt * T, B, T, Qt * T, 1, T, Qt, True, C_),
        "across_nomask": (B * Qt * T, B, T, Qt * T, 1, T, Qt, False, C_),
        "aifi": (B * 400, B, 1, 400, 0, 1, 400, False, C_),
    }
    for name, (rows, no, ni, so, si, st, L, masked, Cc) in cases.items():
        dh = Cc // nh
        qkv = torch.randn(rows, 3 * Cc, device=dev).to(dt)
        out = torch.empty(rows, Cc, device=dev, dtype=dt)
        dout = torch.randn(rows, Cc, device=dev).to(dt)
        dqkv = torch.empty(rows, 3 * Cc, device=dev, dtype=dt)
        P = torch.empty(no * ni * nh * L * L, device=dev)
        mask = (torch.rand(L, L, device=dev) < 0.3).to(torch.uint8) if masked else None
        e = qkv.element_size()
        base, db = qkv.data_ptr(), dqkv.data_ptr()

        def fwd():
            _lib.check(lib.dp_attn_fwd(base, 3 * Cc, base + Cc * e, base + 2 * Cc * e, 3 * Cc, out.data_ptr(), Cc,
                                       P.data_ptr(), mask.data_ptr() if masked else None, no, ni, so, si, st, L, nh,
                                       dh, code, sp), "fwd")

        def bwd():
            _lib.check(lib.dp_attn_bwd(base, 3 * Cc, base + Cc * e, base + 2 * Cc * e, 3 * Cc, P.data_ptr(),
                                       dout.data_ptr(), out.data_ptr(), Cc, db, 3 * Cc, db + Cc * e, db + 2 * Cc * e,
                                       3 * Cc, no, ni, so, si, st, L, nh, dh, code, sp), "bwd")

        res = {}
        for tag, fn in (("fwd", fwd), ("bwd", bwd)):
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
            res[tag] = sorted(ts)[len(ts) // 2]
        waves = no * ni * nh * ((L + 63) // 64)
        flops = 4.0 * no * ni * nh * L * L * dh
        print(f"{name:14s} L={L:4d} waves={waves:6d} fwd {res['fwd'] * 1e3:8.1f} us  bwd {res['bwd'] * 1e3:8.1f} us"
              f"  ({flops / res['fwd'] / 1e9:.2f} TFLOP/s fwd)", flush=True)


if __name__ == "__main__":
    main()
