"""Trainer.step with its tapes replayed from hipGraphs (the default at world size 1).

A graph replay launches exactly the kernels an eager run of the tape does, on the same fixed
buffers, and the training forward has no float atomics (BatchNorm statistics are summed per
row slice in a fixed order, dp_bn_stats), so on identical inputs two eager forwards and the
graph replay agree BIT FOR BIT: backbone outputs, the encoder memory, the heads' logits and
keypoints (checked tape by tape after one eager step; whole-step losses are not compared, the
backward still sums with float atomics and one rounding-level difference can flip the two-stage
top-k or a Hungarian assignment and move a loss by percents). Then a few steps running entirely
from graphs must keep training: finite losses and gradient norms, no skipped update.
fp32 DETRPose-N (its LAB backbone stays eager) and bf16 DETRPose-L (every tape replayed)."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def _targets(dev, B):
    g = torch.Generator().manual_seed(5)
    out = []
    for b in range(B):
        n = 2 + b % 3
        c = torch.rand(n, 2, generator=g) * 0.6 + 0.2
        wh = torch.rand(n, 2, generator=g) * 0.3 + 0.05
        xy = (c[:, None] + (torch.rand(n, 17, 2, generator=g) - 0.5) * wh[:, None]).clamp(0, 1)
        vis = (torch.rand(n, 17, generator=g) > 0.25).float()
        out.append({"labels": torch.zeros(n, dtype=torch.int64, device=dev),
                    "boxes": torch.cat([c - wh / 2, c + wh / 2], 1).to(dev),
                    "keypoints": torch.cat([xy.flatten(1), vis], 1).to(dev), "area": (wh.prod(1) * 0.53).to(dev)})
    return out


def _forward_outputs(tr):
    torch.cuda.synchronize()
    return {"backbone": [v.buf.x.float().clone() for v in tr.bb.outs], "memory": tr.ep.memory.float().clone(),
            "logits": tr.plan.logits[-1].float().clone(), "kps": tr.plan.kps[-1].float().clone()}


@pytest.mark.parametrize("size,dtype,B", [("n", "fp32", 2), ("l", "bf16", 4)])
def test_graph_replay_matches_eager_tapes(size, dtype, B):
    from detrpose_amd import build_model
    from detrpose_amd.synthetic import load_synthetic, synthetic_images
    from detrpose_amd.train import Trainer
    dev = torch.device("cuda", 0)
    model, _ = build_model(size, dtype=dtype)
    load_synthetic(model, seed=0)
    tr = Trainer(model, dtype=dtype, device=dev, grad_accum_steps=1, graphs=False)
    images = synthetic_images(B, seed=1).to(dev)
    ts = _targets(dev, B)
    tr.step(images, ts)                      # every tape has run once, eagerly
    bb, ep, plan = tr.bb, tr.ep, tr.plan
    bb.forward()
    ep.forward()
    plan.forward()
    eager = _forward_outputs(tr)
    bb.forward()                             # eager again: the run-to-run spread of the atomics
    ep.forward()
    plan.forward()
    eager2 = _forward_outputs(tr)
    tr.graphs = True
    tr._set_graphs(plan, bb, ep)
    bb.forward()                             # captured, then replayed
    ep.forward()
    plan.forward()
    graph = _forward_outputs(tr)
    labs = bool(bb.labs)
    assert [t._graph is not None for t in (bb.fw, ep.fw, plan.fw)] == [not labs, True, True]
    for a, b in zip(eager["backbone"], graph["backbone"]):
        assert torch.equal(a, b), "backbone forward: graph replay differs from the eager launches"
    for k in ("memory", "logits", "kps"):
        d = float((graph[k] - eager[k]).abs().max())
        d0 = float((eager2[k] - eager[k]).abs().max())
        nd = int((graph[k] != eager[k]).sum())
        scale = max(float(eager[k].abs().max()), 1e-12)
        print(f"{size} {dtype} {k}: max |graph - eager| {d:.3g} over {nd} of {eager[k].numel()} "
              f"(eager - eager {d0:.3g}, scale {scale:.3g})")
        assert d0 == 0 and d == 0, (k, d0, d)   # deterministic forward: bit-identical
    # whole steps from the graphs: training goes on
    totals = []
    for _ in range(4):
        keys, vals = tr.step(images, ts)
        torch.cuda.synchronize()
        totals.append(float(vals.sum()))
        assert torch.isfinite(vals).all() and not tr.eng.step_skipped(), (totals, tr.eng.step_skipped())
    assert all(t._graph is not None for t in (plan.bw, ep.bw)) and (bb.bw._graph is not None) == (not labs)
    print(f"{size} {dtype}: total loss over steps replayed from graphs {[round(t, 3) for t in totals]}")
