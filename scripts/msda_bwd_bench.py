"""Times the MSDA module backward at the training step's shape (DETRPose-L b16: 16 images x 96
queries x 18 tokens, 8 heads, dh 32, 3 levels x 4 points, bf16 value / grad_out, accumulating into
d memory as the tape does): dp_msda_bwd (f32 atomics) vs dp_msda_bwd_sorted (per-pixel counting
sort + register sums), HIP events on the launch stream, median of --reps; and the two results'
max difference. Inputs: "spread" (offsets N(0, 3) px around uniform reference points) and
"clustered" (reference points near three spots per image: long pixel lists).

    python scripts/msda_bwd_bench.py [--reps 20] [--dtype bf16]
"""
import argparse
import ctypes as C
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--dtype", default="bf16")
    ap.add_argument("--out", default="")
    a = ap.parse_args()
    from detrpose_amd import _lib
    from detrpose_amd.msda import _shapes_arg
    lib = _lib.load()
    code = _lib.DP_BF16 if a.dtype == "bf16" else _lib.DP_F32
    dt = torch.bfloat16 if a.dtype == "bf16" else torch.float32
    dev = torch.device("cuda")
    sp = C.c_void_p(torch.cuda.current_stream().cuda_stream)
    N, Qt, T, nH, Dh, P = 16, 96, 18, 8, 32, 4
    shapes = [(80, 80), (40, 40), (20, 20)]
    L, S, Cc, lq = len(shapes), sum(h * w for h, w in shapes), nH * Dh, Qt * T
    hw, nl = _shapes_arg(shapes)
    g = torch.Generator(device=dev).manual_seed(0)
    value = torch.randn(N, S, Cc, device=dev, generator=g).to(dt)
    go = torch.randn(N * lq, 2 * Cc, device=dev, generator=g).to(dt)   # the tape's dx rows (ld 2C)
    gv = torch.zeros(N, S, Cc, device=dev)
    goa = torch.empty(N * lq, nH * L * P * 3, device=dev)
    gref = torch.empty(N * lq, 2, device=dev)
    nb = int(lib.dp_msda_bwd_ws_bytes(N, S, hw, nl, lq, nH, P))
    ws = torch.empty(nb, device=dev, dtype=torch.uint8)
    res = {"shape": {"N": N, "lq": lq, "heads": nH, "dh": Dh, "levels": shapes, "points": P, "dtype": a.dtype},
           "workspace_MB": round(nb / 2**20, 1), "cases": {}}
    for case in ("spread", "clustered"):
        if case == "spread":
            ref = torch.rand(N * lq, 2, device=dev, generator=g) * 0.9 + 0.05
            off = torch.randn(N * lq, nH * L * P * 2, device=dev, generator=g) * 3
        else:
            spots = torch.rand(N, 3, 2, device=dev, generator=g) * 0.6 + 0.2
            pick = torch.randint(0, 3, (N, lq), device=dev, generator=g)
            ref = (torch.gather(spots, 1, pick[..., None].expand(N, lq, 2)).reshape(N * lq, 2)
                   + 0.01 * torch.randn(N * lq, 2, device=dev, generator=g))
            off = torch.randn(N * lq, nH * L * P * 2, device=dev, generator=g) * 1.5
        oa = torch.cat([off, torch.randn(N * lq, nH * L * P, device=dev, generator=g)], 1).contiguous()
        args = (value.data_ptr(), N, S, hw, nl, oa.data_ptr(), ref.data_ptr(), go.data_ptr(), 2 * Cc, lq, nH, Dh, P,
                gv.data_ptr(), 1, goa.data_ptr(), gref.data_ptr())

        def atomic():
            _lib.check(lib.dp_msda_bwd(*args, code, sp), "dp_msda_bwd")

        def sorted_():
            _lib.check(lib.dp_msda_bwd_sorted(*args, ws.data_ptr(), nb, code, sp), "dp_msda_bwd_sorted")

        out = {}
        for name, fn in (("atomic", atomic), ("sorted", sorted_)):
            gv.zero_()
            fn()
            torch.cuda.synchronize()
            out[name] = (gv.clone(), goa.clone(), gref.clone())
            ts = []
            for _ in range(a.reps):
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                fn()
                e1.record()
                torch.cuda.synchronize()
                ts.append(e0.elapsed_time(e1))
            ts.sort()
            res["cases"].setdefault(case, {})[name + "_ms"] = round(ts[len(ts) // 2], 4)
        diff = {k: float((x - y).abs().max() / max(1.0, float(x.abs().max())))
                for k, x, y in zip(("grad_value", "grad_offattn", "grad_ref"), out["atomic"], out["sorted"])}
        res["cases"][case]["max_rel_diff"] = diff
    line = json.dumps(res)
    print(line)
    if a.out:
        with open(a.out, "w") as f:
            f.write(line + "\n")


if __name__ == "__main__":
    main()
