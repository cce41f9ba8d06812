"""Run a plan op by op (synchronising after each) and print output statistics."""
import sys, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from detrpose_amd import build_model
from detrpose_amd.synthetic import load_synthetic, synthetic_images

size = sys.argv[1] if len(sys.argv) > 1 else "n"
dtype = sys.argv[2] if len(sys.argv) > 2 else "fp32"
m, _ = build_model(size, dtype=dtype)
load_synthetic(m, 0)
m.deploy()
eng = m.engine()
plan = eng.plan(1)
plan.input.copy_(synthetic_images(1, 1).cuda())
def dbg(name, fm):
    if fm is None:
        print(f"{name:24s} (no fmap)")
        return
    v = fm.view().float()
    print(f"{name:24s} shape={tuple(v.shape)} nan={int(torch.isnan(v).sum())} min={v.min().item():.4g} max={v.max().item():.4g} mean={v.mean().item():.4g}")
plan.run(debug=dbg)
