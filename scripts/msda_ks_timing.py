"""Phase timing of dp_msda_bwd_sorted's sort kernel from a library built with -DDP_KS_TIMING
(wall-clock stamps of every sort block at its phase boundaries, in the workspace's last region):
per level, the mean / max block time of each phase, and the blocks' start / end spread.
Shape and inputs as scripts/msda_bwd_bench.py's "spread" case.

    DETRPOSE_HIP_LIB=<timing lib> DETRPOSE_ALLOW_STALE_LIB=1 python scripts/msda_ks_timing.py
"""
import ctypes as C
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    from detrpose_amd import _lib
    from detrpose_amd.msda import _shapes_arg
    lib = _lib.load()
    dev = torch.device("cuda")
    sp = C.c_void_p(torch.cuda.current_stream().cuda_stream)
    N, Qt, T, nH, Dh, P = 16, 96, 18, 8, 32, 4
    shapes = [(80, 80), (40, 40), (20, 20)]
    L, S, Cc, lq = len(shapes), sum(h * w for h, w in shapes), nH * Dh, Qt * T
    hw, nl = _shapes_arg(shapes)
    g = torch.Generator(device=dev).manual_seed(0)
    value = torch.randn(N, S, Cc, device=dev, generator=g).bfloat16()
    go = torch.randn(N * lq, 2 * Cc, device=dev, generator=g).bfloat16()
    gv = torch.zeros(N, S, Cc, device=dev)
    goa = torch.empty(N * lq, nH * L * P * 3, device=dev)
    ref = torch.rand(N * lq, 2, device=dev, generator=g) * 0.9 + 0.05
    off = torch.randn(N * lq, nH * L * P * 2, device=dev, generator=g) * 3
    oa = torch.cat([off, torch.randn(N * lq, nH * L * P, device=dev, generator=g)], 1).contiguous()
    nb = int(lib.dp_msda_bwd_ws_bytes(N, S, hw, nl, lq, nH, P))
    ws = torch.zeros(nb, device=dev, dtype=torch.uint8)
    for _ in range(3):
        _lib.check(lib.dp_msda_bwd_sorted(value.data_ptr(), N, S, hw, nl, oa.data_ptr(), ref.data_ptr(), go.data_ptr(),
                                          2 * Cc, lq, nH, Dh, P, gv.data_ptr(), 1, goa.data_ptr(), None,
                                          ws.data_ptr(), nb, _lib.DP_BF16, sp), "sorted")
    torch.cuda.synchronize()
    nseg = N * nH
    dbg_bytes = nseg * L * 8 * 8
    # the timing region is the layout's last take() (256-byte rounded)
    st = ws[nb - (dbg_bytes + 255) // 256 * 256:][:dbg_bytes].cpu().numpy().view(np.int64).reshape(nseg, L, 8)
    t0 = st[:, :, 0].min()
    out = {}
    for l in range(L):
        s = st[:, l, :6].astype(np.float64)
        ph = np.diff(s, axis=1) * 10e-3   # 100 MHz ticks -> us
        out[f"level{l}"] = {"phases_us_mean": [round(float(v), 2) for v in ph.mean(0)],
                            "phases_us_max": [round(float(v), 2) for v in ph.max(0)],
                            "start_us": [round(float((s[:, 0] - t0).min() * 10e-3), 2),
                                         round(float((s[:, 0] - t0).max() * 10e-3), 2)],
                            "end_us_max": round(float((s[:, 5] - t0).max() * 10e-3), 2)}
    out["phases"] = ["zero+softmax+pass1 loads", "pass1 LDS atomics", "scan", "items", "pass2"]
    print(json.dumps(out))


if __name__ == "__main__":
    main()
