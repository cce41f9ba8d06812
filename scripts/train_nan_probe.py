"""Steps of the L b16 bf16 training leg (bench.py's inputs) printing whether each step's losses
and update were finite: isolates a non-finite step between the MSDA backward variant
(DETRPOSE_MSDA_BWD=sorted|atomic) and graph replay (DETRPOSE_TRAIN_GRAPHS=1|0).

    python scripts/train_nan_probe.py [--steps 8] [--accum 2]
"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=8)
    ap.add_argument("--accum", type=int, default=2)
    ap.add_argument("--size", default="l")
    a = ap.parse_args()
    from bench import synthetic_targets
    from detrpose_amd import build_model
    from detrpose_amd.synthetic import load_synthetic, synthetic_images
    from detrpose_amd.train import Trainer
    dev = torch.device("cuda")
    model, _ = build_model(a.size, dtype="bf16")
    load_synthetic(model, 0)
    tr = Trainer(model, dtype="bf16", device=dev, grad_accum_steps=a.accum)
    images = synthetic_images(16, seed=11).to(dev)
    ts = synthetic_targets(16, seed=3, dev=dev)
    tag = f"msda={os.environ.get('DETRPOSE_MSDA_BWD', 'sorted')} graphs={tr.graphs}"
    for i in range(a.steps):
        keys, vals = tr.step(images, ts)
        torch.cuda.synchronize()
        fin = bool(torch.isfinite(vals).all())
        bad = [k for k, v in zip(keys, vals.tolist()) if not (v == v and abs(v) < float("inf"))]
        print(f"{tag} step {i}: losses finite {fin} skipped {tr.eng.step_skipped()} total {float(vals.sum()):.4f} "
              f"non-finite {bad[:6]}", flush=True)


if __name__ == "__main__":
    main()
