"""Per-op roofline table for the dense conv family from a bench.py --profile-ops JSON:
measured ms vs max(algorithmic bytes / 8 TB/s, flops / 2.5 PF/s).

    python scripts/op_roofline.py gpurun_out/ops.json [--size l --batch 64] [--top 40]
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("json")
    ap.add_argument("--size", default="l")
    ap.add_argument("--batch", type=int, default=64)
    ap.add_argument("--top", type=int, default=40)
    a = ap.parse_args()
    from detrpose_amd import build_model
    from detrpose_amd.engine import Engine
    from detrpose_amd.synthetic import load_synthetic
    m, _ = build_model(a.size)
    load_synthetic(m, 0)
    p = Engine(m, "bf16", device="cpu").plan(a.batch)
    fn = {n: f.__name__ for n, f, _ in p.ops}
    om = json.load(open(a.json))["op_ms"]
    rows = []
    for n in p.op_bytes:
        if fn[n] != "dp_conv2d" or n not in om:
            continue
        lb = max(p.op_bytes[n] / 8e12, p.op_flops[n] / 2.5e15) * 1e3
        rows.append((om[n] - lb, n, om[n], lb, p.op_bytes[n] / 1e9, p.op_flops[n] / 1e12))
    rows.sort(reverse=True)
    print(f"conv family: measured {sum(r[2] for r in rows):.3f} ms, roofline {sum(r[3] for r in rows):.3f} ms")
    print(f"{'op':28s} {'ms':>7s} {'lb ms':>7s} {'GB':>6s} {'TF':>6s} {'TB/s':>6s} {'TF/s':>6s}")
    for r in rows[:a.top]:
        print(f"{r[1]:28s} {r[2]:7.3f} {r[3]:7.3f} {r[4]:6.3f} {r[5]:6.3f} {r[4] / r[2]:6.2f} {r[5] / r[2] * 1e3:6.0f}")


if __name__ == "__main__":
    main()
