"""Times dp_dwconv_bwd (input and weight gradients, separately) and dp_frozen_act_bwd on the
backbone training step's shapes (HGNetv2-L b16), HIP events on the launch stream.

    python scripts/dw_bench.py [--reps 20]
"""
import argparse
import ctypes as C
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def timed(fn, reps):
    fn()
    torch.cuda.synchronize()
    ts = []
    for _ in range(reps):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        fn()
        e1.record()
        torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1))
    return sorted(ts)[len(ts) // 2] * 1e3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=20)
    a = ap.parse_args()
    from detrpose_amd import _lib
    lib = _lib.load()
    dev = torch.device("cuda")
    sp = C.c_void_p(torch.cuda.current_stream().cuda_stream)
    B = 16
    # (h, w, c, k, stride)
    for h, w, c, k, st in ((80, 80, 128, 5, 1), (40, 40, 256, 5, 1), (20, 20, 512, 5, 1), (160, 160, 128, 3, 2),
                           (80, 80, 512, 3, 2)):
        pad = (k - 1) // 2
        oh, ow = (h + 2 * pad - k) // st + 1, (w + 2 * pad - k) // st + 1
        x = torch.randn(B, h, w, c, device=dev).bfloat16()
        dz = torch.randn(B, oh, ow, c, device=dev).bfloat16()
        taps = torch.randn(k * k, c, device=dev)
        dx = torch.zeros(B, h, w, c, device=dev).bfloat16()
        dw = torch.zeros(c, k, k, device=dev)

        def run(do_dx, do_dw):
            return lambda: _lib.check(lib.dp_dwconv_bwd(
                x.data_ptr(), h * w * c, c, dz.data_ptr(), oh * ow * c, c, taps.data_ptr(), B, h, w, c, k, st, pad,
                oh, ow, dx.data_ptr() if do_dx else None, h * w * c, c, dw.data_ptr() if do_dw else None, 1, sp), "dw")
        tx, tw = timed(run(True, False), a.reps), timed(run(False, True), a.reps)
        mb = (x.numel() * 2 * 2 + dz.numel() * 2) / 1e6
        print(f"dw_bwd {h}x{w} c{c} k{k} s{st}: dx {tx:8.1f} us  dw {tw:8.1f} us  ({mb:.1f} MB moved by dx)", flush=True)
    for rows, c in ((B * 320 * 320, 16), (B * 320 * 320, 32), (B * 80 * 80, 128), (B * 40 * 40, 1024)):
        y = torch.randn(rows, c, device=dev).bfloat16()
        dy = torch.randn(rows, c, device=dev).bfloat16()
        dz = torch.empty(rows, c, device=dev).bfloat16()
        sc = torch.rand(c, device=dev)
        la, lb = torch.ones(1, device=dev), torch.zeros(1, device=dev)
        ga, gb = torch.zeros(1, device=dev), torch.zeros(1, device=dev)
        t = timed(lambda: _lib.check(lib.dp_frozen_act_bwd(
            y.data_ptr(), c, None, 0, dy.data_ptr(), c, dz.data_ptr(), c, rows, c, 1, la.data_ptr(), lb.data_ptr(),
            sc.data_ptr(), ga.data_ptr(), gb.data_ptr(), 1, sp), "act"), a.reps)
        print(f"frozen_act_bwd rows {rows} c {c}: {t:8.1f} us  ({rows * c * 6 / t / 1e3:.0f} GB/s)", flush=True)


if __name__ == "__main__":
    main()
