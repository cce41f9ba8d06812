"""Microbenchmark of the row-block fused decoder kernels (csrc/decoder.hip) in isolation
(development tool): HIP-event time per launch at several row counts, with the
algorithmic bytes / FLOPs of each launch.

    python scripts/dec_bench.py [--c 256] [--rows 69120] [--reps 20] [--kernels ln,gate,ffn,pos,pose]
"""
import argparse
import ctypes as C
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from detrpose_amd import _lib  # noqa: E402
from detrpose_amd._lib import contiguous_rows as cr, rowmap  # noqa: E402
from detrpose_amd.fragments import frag_pack  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--c", type=int, default=256)
    ap.add_argument("--f", type=int, default=1024)
    ap.add_argument("--rows", default="69120")
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--kernels", default="ln,gate,ffn,pos,pose,mhaw,mhaa")
    ap.add_argument("--libs", default="", help="comma-separated .so builds to time side by side (default: the package's)")
    a = ap.parse_args()
    c, f = a.c, a.f
    libs = []
    for path in (a.libs.split(",") if a.libs else [None]):
        if path is None:
            libs.append(("lib", _lib.load()))
            continue
        h = C.CDLL(path)
        for name, (res_t, args) in _lib._SIGS.items():
            fn = getattr(h, name)
            fn.restype, fn.argtypes = res_t, args
        libs.append((os.path.basename(os.path.dirname(path)), h))
    dev = "cuda"
    bf = torch.bfloat16
    T, K = 18, 17
    g = torch.Generator(device="cpu").manual_seed(0)

    def rnd(*s, scale=1.0, dt=bf):
        return (torch.randn(*s, generator=g) * scale).to(dev, dt)

    W = {n: frag_pack(rnd(o, i, scale=i ** -0.5)) for n, (o, i) in
         {"wo": (c, c), "gate": (2 * c, 2 * c), "f1": (f, c), "f2": (c, f), "p0": (c, c), "p1": (c, c),
          "q2": (66, c), "qkv": (3 * c, c)}.items()}
    B = {n: rnd(o, scale=0.1, dt=torch.float32) for n, o in
         {"wo": c, "gate": 2 * c, "f1": f, "f2": c, "p0": c, "p1": c, "q2": 66, "qkv": 3 * c}.items()}
    gam, bet = rnd(c, dt=torch.float32), rnd(c, dt=torch.float32)
    dim_t = (10000 ** (2 * (torch.arange(c // 2) // 2) / (c // 2))).float().to(dev)
    s = C.c_void_p(torch.cuda.current_stream().cuda_stream)
    eps = C.c_float(1e-5)
    for rows in [int(r) for r in a.rows.split(",")]:
        rows = rows // T * T
        nq = rows // T
        krows = nq * K
        x, res = rnd(rows, c), rnd(rows, c)
        out2 = torch.empty(rows, 2 * c, dtype=bf, device=dev)
        gx = rnd(rows, 2 * c)
        pos = torch.empty(krows, c, dtype=bf, device=dev)
        ref = torch.rand(nq, T, 2, device=dev)
        corners = [torch.randn(krows, 66, device=dev) for _ in range(2)]
        kp = rowmap(c, K, T * c, c)
        nqi = 60
        bimg = nq // nqi
        for lname, lib in libs:
          calls = {
            "mhaw": (lambda: lib.dp_mha_layernorm(out2.data_ptr(), cr(c), x.data_ptr(), cr(c), nq, 1, T, 0, 1, T,
                                                  W["qkv"].data_ptr(), B["qkv"].data_ptr(), W["wo"].data_ptr(),
                                                  B["wo"].data_ptr(), gam.data_ptr(), bet.data_ptr(), eps, c, 8, None,
                                                  cr(c), 1, 0, None, 0, None, None, 0, s),
                     2 * rows * c * 2, 2 * rows * c * 4 * c),
            "mhaa": (lambda: lib.dp_mha_layernorm(out2.data_ptr(), cr(2 * c), x.data_ptr(), cr(c), bimg, T, nqi * T,
                                                  1, T, nqi, W["qkv"].data_ptr(), B["qkv"].data_ptr(),
                                                  W["wo"].data_ptr(), B["wo"].data_ptr(), gam.data_ptr(),
                                                  bet.data_ptr(), eps, c, 8, pos.data_ptr(), cr(c), T, 1, None, 0, None, None,
                                                  0, s),
                     3 * rows * c * 2, 2 * rows * c * 4 * c),
            "ln": (lambda: lib.dp_linear_layernorm(out2.data_ptr(), cr(2 * c), x.data_ptr(), cr(c), c,
                                                   W["wo"].data_ptr(), B["wo"].data_ptr(), res.data_ptr(), cr(c),
                                                   gam.data_ptr(), bet.data_ptr(), eps, rows, c, None, cr(c), 1, 0, s),
                   3 * rows * c * 2, 2 * rows * c * c),
            "gate": (lambda: lib.dp_gate_linear_layernorm(out2.data_ptr(), cr(c), gx.data_ptr(), cr(2 * c),
                                                          W["gate"].data_ptr(), B["gate"].data_ptr(), gam.data_ptr(),
                                                          bet.data_ptr(), eps, rows, c, s),
                     3 * rows * c * 2, 2 * rows * 4 * c * c),
            "ffn": (lambda: lib.dp_ffn_layernorm(x.data_ptr(), cr(c), x.data_ptr(), cr(c), W["f1"].data_ptr(),
                                                 B["f1"].data_ptr(), f, W["f2"].data_ptr(), B["f2"].data_ptr(),
                                                 gam.data_ptr(), bet.data_ptr(), eps, rows, c, s),
                    2 * rows * c * 2, 4 * rows * c * f),
            "pos": (lambda: lib.dp_query_pos(ref.data_ptr(), krows, K, dim_t.data_ptr(), W["p0"].data_ptr(),
                                             B["p0"].data_ptr(), W["p1"].data_ptr(), B["p1"].data_ptr(),
                                             pos.data_ptr(), x.data_ptr(), kp, c, s),
                    3 * krows * c * 2, 4 * krows * c * c),
            "pose": (lambda: lib.dp_pose_mlp(x.data_ptr(), kp, res.data_ptr(), kp, krows, W["p0"].data_ptr(),
                                             B["p0"].data_ptr(), W["p1"].data_ptr(), B["p1"].data_ptr(),
                                             W["q2"].data_ptr(), B["q2"].data_ptr(), 66, corners[0].data_ptr(),
                                             corners[1].data_ptr(), c, s),
                     2 * krows * c * 2 + 2 * krows * 66 * 4, 2 * krows * c * (2 * c + 66)),
        }
          for name in a.kernels.split(","):
              fn, byts, flops = calls[name]
              _lib.check(fn(), name)
              torch.cuda.synchronize()
              e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
              e0.record()
              for _ in range(a.reps):
                  fn()
              e1.record()
              torch.cuda.synchronize()
              us = e0.elapsed_time(e1) * 1e3 / a.reps
              print(f"{lname:8s} {name:5s} rows {rows:6d}: {us:8.1f} us  {byts / us / 1e3:7.1f} GB/s  {flops / us / 1e6:7.1f} TF/s",
                    flush=True)


if __name__ == "__main__":
    main()
