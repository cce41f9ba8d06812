"""Per-op HIP-event profile of the DETRPose plan (development tool).

    python scripts/prof_plan.py [--size l] [--batch 64] [--dtype bf16] [--top 30] [--json out.json]

Prints time per kernel family and the slowest ops with their achieved TFLOP/s
(conv/linear) or GB/s (MSDA). Set DETRPOSE_HIP_LIB to A/B a different build.
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from detrpose_amd import build_model  # noqa: E402
from detrpose_amd.synthetic import load_synthetic, synthetic_images  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--size", default="l")
    ap.add_argument("--batch", type=int, default=64)
    ap.add_argument("--dtype", default="bf16")
    ap.add_argument("--top", type=int, default=30)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--json", default="")
    a = ap.parse_args()
    m, _ = build_model(a.size, dtype=a.dtype)
    load_synthetic(m, 0)
    m.deploy()
    plan = m.engine().plan(a.batch)
    plan.input.copy_(synthetic_images(a.batch, 1).cuda())
    plan.run()
    torch.cuda.synchronize()
    ms = plan.profile(reps=a.reps)
    fam = {}
    for name, fn, _ in plan.ops:
        fam[fn.__name__] = fam.get(fn.__name__, 0.0) + ms[name]
    tot = sum(ms.values())
    print(f"total {tot:.3f} ms/step  ->  {a.batch / tot * 1e3:.1f} img/s (kernel time only)")
    for k, v in sorted(fam.items(), key=lambda kv: -kv[1]):
        print(f"  {k:24s} {v:8.3f} ms  {100 * v / tot:5.1f}%")
    cf = sum(plan.op_flops[n] for n in plan.op_flops)
    ct = sum(ms[n] for n in plan.op_flops)
    print(f"conv/linear: {ct:.3f} ms, {cf / ct / 1e9:.1f} TFLOP/s")
    rows = sorted(ms.items(), key=lambda kv: -kv[1])[: a.top]
    for n, t in rows:
        extra = ""
        if n in plan.op_flops:
            extra = f"{plan.op_flops[n] / t / 1e9:8.1f} TF/s"
        elif n in plan.op_bytes:
            extra = f"{plan.op_bytes[n] / t / 1e6:8.1f} GB/s"
        print(f"  {n:26s} {t:7.3f} ms {extra}")
    if a.json:
        with open(a.json, "w") as f:
            json.dump({"op_ms": ms, "op_flops": plan.op_flops, "op_bytes": plan.op_bytes, "family": fam}, f)


if __name__ == "__main__":
    main()
