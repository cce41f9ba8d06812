import os, json, sys, torch
sys.path.insert(0, "/root/repo")
from detrpose_amd import build_model
from detrpose_amd.synthetic import synthetic_images, synthetic_state_dict
from detrpose_amd.engine import Engine
man = json.load(open("tests/golden/manifest.json"))
model, _ = build_model("l", dtype="bf16")
model.load_state_dict(synthetic_state_dict(man["l"], seed=0), strict=False)
model.eval()
img = synthetic_images(1, seed=5).cuda()
outs = {}
for fused in (True, False):
    if fused: os.environ.pop("DETRPOSE_NO_STEM_FUSE", None)
    else: os.environ["DETRPOSE_NO_STEM_FUSE"] = "1"
    plan = Engine(model, "bf16", device="cuda").plan(1)
    plan.input.copy_(img); plan.run(); torch.cuda.synchronize()
    outs[fused] = plan.op_out["stem" if fused else "stem4"].view().float().clone()
a, b = outs[True], outs[False]
d = (a - b).abs()
print("max", d.max().item(), "frac bad", (d > 0).float().mean().item())
bad = (d > 0).any(-1)[0]   # H x W
ys, xs = torch.nonzero(bad, as_tuple=True)
print("rows with diffs", torch.unique(ys).tolist()[:50])
print("cols with diffs", torch.unique(xs).tolist()[:50])
print("chan with diffs", torch.nonzero((d > 0).any(0).any(0).any(0)).flatten().tolist())
print("sample", a[0, 50, 50, :8].tolist(), b[0, 50, 50, :8].tolist())
# variant: identity LAB (the float max-pool path)
os.environ.pop("DETRPOSE_NO_STEM_FUSE", None)
eng = Engine(model, "bf16", device="cuda")
orig = eng._stem_fused_op
def patched(plan, img_, out):
    orig(plan, img_, out)
    sw = plan.keep[-1]
    sw.has_lab = 1
eng._stem_fused_op = patched
plan = eng.plan(1)
plan.input.copy_(img); plan.run(); torch.cuda.synchronize()
c = plan.op_out["stem"].view().float()
print("LAB-identity path vs unfused: max", (c - b).abs().max().item(), " vs fused-noLAB:", (c - a).abs().max().item())
