"""Kernel trace of the training step's steady state (under rocprofv3 --kernel-trace): a Trainer
(DETRPose-L bf16, b16, the config's grad_accum_steps) runs two warm-up steps, then STEPS steps
between two marker kernels (torch.cuda._sleep); scripts/trace_steps.py cuts the trace at the
markers and reports per-step kernel counts and times (setup copies -- the state dict upload,
the first eager tape runs, the graph captures -- stay outside).

    rocprofv3 --kernel-trace --output-format csv -d DIR -o run -- python3 scripts/train_trace.py
"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

STEPS = int(os.environ.get("TRACE_STEPS", "3"))


def main():
    from bench import synthetic_targets
    from detrpose_amd import build_model
    from detrpose_amd.synthetic import load_synthetic, synthetic_images
    from detrpose_amd.train import Trainer
    dev = torch.device("cuda")
    model, _ = build_model("l", dtype="bf16")
    load_synthetic(model, 0)
    tr = Trainer(model, dtype="bf16", device=dev)
    images = synthetic_images(16, seed=11).to(dev)
    ts = synthetic_targets(16, dev=dev)
    for _ in range(2):
        tr.step(images, ts)
    torch.cuda.synchronize()
    torch.cuda._sleep(1000)   # marker
    for _ in range(STEPS):
        tr.step(images, ts)
    torch.cuda._sleep(1000)   # marker
    torch.cuda.synchronize()
    print("steps", STEPS, "grad_accum_steps", tr.grad_accum_steps)


if __name__ == "__main__":
    main()
