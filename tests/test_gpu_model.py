"""End-to-end parity of the HIP forward against the reference (golden fixtures).

fp32 mode: every stage within the north-star gate (1e-3 abs on logits / keypoints) and
the two-stage top-k order identical. bf16 mode (the benchmarked kernels): the selection
is order-sensitive (SURVEY.md header fact 5), so the fp32 oracle is re-run on the HIP
path's own selection and compared query by query; the headline batch-64 plan must be
batch invariant. Also the reference's eval-loop and export call patterns.
"""
import json
import os

import numpy as np
import pytest
import torch

from detrpose_amd import build_model
from detrpose_amd.synthetic import synthetic_images, synthetic_state_dict

pytestmark = pytest.mark.gpu

CASES = [("n", 2), ("l", 1), ("x", 1)]


def _model(golden_dir, size, g, dtype):
    with open(os.path.join(golden_dir, "manifest.json")) as f:
        man = json.load(f)
    model, pp = build_model(size, dtype=dtype)
    sd = synthetic_state_dict(man[size], seed=int(g["meta"][1]))
    missing, unexpected = model.load_state_dict(sd, strict=False)
    assert not unexpected
    return model.deploy(), pp.deploy()


def _sampled(g, name, t):
    return t.reshape(-1)[torch.from_numpy(g[name + "__idx"]).to(t.device)].float().cpu().numpy(), g[name + "__val"]


@pytest.mark.parametrize("size,batch", CASES)
def test_fp32_matches_reference(golden_dir, size, batch):
    g = np.load(os.path.join(golden_dir, f"detrpose_{size}_b{batch}.npz"))
    model, pp = _model(golden_dir, size, g, "fp32")
    images = synthetic_images(batch, seed=int(g["meta"][2])).cuda()
    out = model(images)
    torch.cuda.synchronize()
    plan = model.engine().plan(batch)
    # stage by stage (NHWC buffers vs the reference's NCHW samples)
    for i, fm in enumerate(plan.bufs["backbone"]):
        a, b = _sampled(g, f"backbone{i}", fm.view().permute(0, 3, 1, 2).contiguous())
        np.testing.assert_allclose(a, b, atol=2e-3, rtol=2e-3, err_msg=f"backbone{i}")
    for i, fm in enumerate(plan.bufs["encoder"]):
        a, b = _sampled(g, f"encoder{i}", fm.view().permute(0, 3, 1, 2).contiguous())
        np.testing.assert_allclose(a, b, atol=2e-3, rtol=2e-3, err_msg=f"encoder{i}")
    np.testing.assert_array_equal(plan.bufs["topk_idx"].cpu().numpy(), g["topk_idx"])
    np.testing.assert_allclose(out["pred_logits"].cpu().numpy(), g["out_pred_logits"], atol=1e-3)
    np.testing.assert_allclose(out["pred_keypoints"].cpu().numpy(), g["out_pred_keypoints"], atol=1e-3)
    ts = torch.tensor(np.tile(g["pp_target_size"], (batch, 1)), device="cuda")
    s, l, k = pp(out, ts)
    np.testing.assert_allclose(s.cpu().numpy(), g["pp_scores"], atol=1e-3)
    np.testing.assert_array_equal(l.cpu().numpy(), g["pp_labels"])
    np.testing.assert_allclose(k.cpu().numpy(), g["pp_keypoints"], atol=640 * 1e-3)


# ---------------------------------------------------------------- bf16 production path, pinned

# bf16 storage (8 mantissa bits) through ~110 conv/linear layers, 3-6 decoder layers and an
# fp32 head, vs the fp32 oracle on the SAME selection ("Parity of the bf16
# path" and "Where the bf16 error comes from"). Keypoints are normalised image coordinates
# in [0, 1]. Measured on MI355X at HEAD (profiles/r3a_pytest_gpu.txt, stem1 on bf16-rounded
# pixels): max|dkp| 0.011 / 0.013 / 0.007 and mean 1.3-1.6e-3 for N / L / X; max|dlogit|
# 0.041 / 0.014 / 0.027, mean 4-7e-3. Bounds: ~1.5x the worst max, ~2x the worst mean.
BF16_TOL_KP, BF16_TOL_KP_MEAN = 2e-2, 3.5e-3
BF16_TOL_LOGIT, BF16_TOL_LOGIT_MEAN = 5e-2, 1.6e-2
BF16_TOPK_OVERLAP = 0.65
# GPU bf16 error vs the error of the bf16-emulating oracle (test_bf16_matches_bf16_emulation), both
# against the fp32 oracle: ratio bounds on (max, mean). Measured on MI355X (profiles/r5h_pytest_bf16_emulation.txt):
# |dkp| max ratio 1.10 / 0.90 / 1.09 and mean 0.95 / 1.03 / 1.01 for N / L / X; |dlogit| max 0.99 / 1.17 / 1.25,
# mean 0.91 / 0.87 / 1.19.
BF16_EMU_RATIO = (1.5, 1.5)


def _oracle(size, model):
    from detrpose_amd.configs import get_config
    from oracle.detrpose_cpu import OracleDETRPose
    return OracleDETRPose(get_config(size), model.state_dict())


@pytest.mark.parametrize("size,batch", CASES)
def test_bf16_matches_bf16_emulation(golden_dir, size, batch):
    """The bf16 path's end-to-end error is the error bf16 storage at the kernels' rounding points
    makes, and no more: the oracle EMULATING that storage (tests/bf16_emulation.py: operands and
    stored activations rounded to bf16 where the kernels round them, f32 accumulation, the MSDA
    offsets / attention logits bf16 as dp_mha_layernorm writes them) is run on the same forced
    selection, and the GPU's distance from the fp32 oracle must be within BF16_EMU_RATIO of the
    emulation's distance from it (max and mean, keypoints and logits). The two rounding errors are
    of one size but not correlated (accumulation order differs; the GPU-to-emulation distance is as
    large as either's distance to fp32), so the check is on magnitudes, not on the GPU matching the
    emulation."""
    from bf16_emulation import bf16_emulation
    g = np.load(os.path.join(golden_dir, f"detrpose_{size}_b{batch}.npz"))
    model, _ = _model(golden_dir, size, g, "bf16")
    images = synthetic_images(batch, seed=int(g["meta"][2]))
    out = model(images.cuda())
    torch.cuda.synchronize()
    idx = model.engine().plan(batch).bufs["topk_idx"].cpu()
    ref = _oracle(size, model)(images, force_topk=idx)
    with bf16_emulation():
        emu = _oracle(size, model)(images, force_topk=idx)
    kp, lg = out["pred_keypoints"].float().cpu(), out["pred_logits"].float().cpu()
    d32, demu = (kp - ref["pred_keypoints"]).abs(), (kp - emu["pred_keypoints"]).abs()
    dref = (emu["pred_keypoints"] - ref["pred_keypoints"]).abs()
    l32, lref = (lg - ref["pred_logits"]).abs(), (emu["pred_logits"] - ref["pred_logits"]).abs()
    r = [float(d32.max() / dref.max()), float(d32.mean() / dref.mean()),
         float(l32.max() / lref.max()), float(l32.mean() / lref.mean())]
    msg = (f"{size}: |dkp| vs fp32: GPU max {d32.max():.3g} mean {d32.mean():.3g}, emulation max {dref.max():.3g} "
           f"mean {dref.mean():.3g} (GPU vs emulation max {demu.max():.3g}) | |dlogit| vs fp32: GPU max "
           f"{l32.max():.3g} mean {l32.mean():.3g}, emulation max {lref.max():.3g} mean {lref.mean():.3g} | "
           f"ratios kp {r[0]:.2f}/{r[1]:.2f} logit {r[2]:.2f}/{r[3]:.2f}")
    print(msg)
    assert r[0] <= BF16_EMU_RATIO[0] and r[2] <= BF16_EMU_RATIO[0], msg
    assert r[1] <= BF16_EMU_RATIO[1] and r[3] <= BF16_EMU_RATIO[1], msg
    assert demu.max() <= BF16_TOL_KP, msg


@pytest.mark.parametrize("size,batch", CASES)
def test_bf16_forced_selection_matches_oracle(golden_dir, size, batch):
    """The benchmarked kernels (conv_stream / conv_halo / attn_mfma, bf16) end to end: the
    fp32 oracle is run on the HIP path's own top-k selection (force_topk), so every query
    is compared slot by slot, logits and keypoints, always asserted."""
    g = np.load(os.path.join(golden_dir, f"detrpose_{size}_b{batch}.npz"))
    model, _ = _model(golden_dir, size, g, "bf16")
    images = synthetic_images(batch, seed=int(g["meta"][2]))
    out = model(images.cuda())
    torch.cuda.synchronize()
    idx = model.engine().plan(batch).bufs["topk_idx"].cpu()
    ref = _oracle(size, model)(images, force_topk=idx)
    kp = out["pred_keypoints"].float().cpu()
    lg = out["pred_logits"].float().cpu()
    assert torch.isfinite(kp).all() and torch.isfinite(lg).all()
    dk = (kp - ref["pred_keypoints"]).abs()
    dl = (lg - ref["pred_logits"]).abs()
    # the bf16 selection against the reference's own (golden fp32) top-k, image by image
    ov = [len(set(idx[b].tolist()) & set(g["topk_idx"][b].tolist())) for b in range(batch)]
    msg = (f"{size} bf16 vs fp32 oracle (forced selection): max|dkp| {dk.max():.3g} (mean {dk.mean():.3g}), "
           f"max|dlogit| {dl.max():.3g} (mean {dl.mean():.3g}), topk overlap with the reference {ov} of "
           f"{idx.shape[1]} per image")
    print(msg)
    assert dk.max() <= BF16_TOL_KP and dl.max() <= BF16_TOL_LOGIT, msg
    assert dk.mean() <= BF16_TOL_KP_MEAN and dl.mean() <= BF16_TOL_LOGIT_MEAN, msg
    # measured (r3k): N 83/120, L 58/60, X 58/60. A floor, so a regression in the fused
    # two-stage head (which queries it selects) fails here even though the forced-selection
    # oracle follows whatever the kernel picked
    assert sum(ov) >= BF16_TOPK_OVERLAP * idx.numel() and min(ov) >= 0.5 * idx.shape[1], msg


def test_bf16_b64_headline_batch_is_batch_invariant(golden_dir):
    """The headline plan (L bf16, batch 64: 256x256/256x128 8-wave tiles, persistent
    multi-tile walks, the largest buffers) gives image 0 and image 63 the same outputs as
    a batch-1 plan of that image, and every output of the batch is finite."""
    g = np.load(os.path.join(golden_dir, "detrpose_l_b1.npz"))
    model, _ = _model(golden_dir, "l", g, "bf16")
    img = synthetic_images(1, seed=int(g["meta"][2]))
    batch = synthetic_images(64, seed=1234)
    batch[0] = img[0]
    batch[63] = img[0]
    o64 = model(batch.cuda())
    i64 = model.engine().plan(64).bufs["topk_idx"].cpu()
    o1 = model(img.cuda())
    i1 = model.engine().plan(1).bufs["topk_idx"].cpu()
    torch.cuda.synchronize()
    for k in ("pred_logits", "pred_keypoints"):
        assert torch.isfinite(o64[k]).all(), k
    for r in (0, 63):
        assert torch.equal(i64[r], i1[0]), f"row {r}: top-k differs from the batch-1 plan"
        dk = (o64["pred_keypoints"][r] - o1["pred_keypoints"][0]).abs().max().item()
        dl = (o64["pred_logits"][r] - o1["pred_logits"][0]).abs().max().item()
        print(f"b64 row {r} vs b1: max|dkp| {dk:.3g} max|dlogit| {dl:.3g}")
        assert dk <= 1e-4 and dl <= 1e-4, (r, dk, dl)
    # the other 62 images are different, so their outputs are too
    assert (o64["pred_keypoints"][1] - o64["pred_keypoints"][0]).abs().max() > 1e-3


# loose per-stage bounds on the bf16 path's relative error (max|d| / max|ref|); the measured
# table is printed and kept in DESIGN.md ("Where the bf16 error comes from")
STAGE_REL_TOL = {"backbone": 0.05, "encoder": 0.08, "layer": 0.08, "corners": 0.08}


@pytest.mark.parametrize("size,batch", CASES)
def test_bf16_stage_errors(golden_dir, size, batch):
    """Attribute the bf16 path's end-to-end error: every stage's output (backbone levels,
    encoder levels = the MSDA memory, each decoder layer's token rows, each layer's
    pred_corners) against the fp32 oracle's on the SAME selection."""
    g = np.load(os.path.join(golden_dir, f"detrpose_{size}_b{batch}.npz"))
    model, _ = _model(golden_dir, size, g, "bf16")
    images = synthetic_images(batch, seed=int(g["meta"][2]))
    model(images.cuda())
    plan = model.engine().plan(batch)
    nl = len(plan.bufs["layers"])
    got = {}

    def grab(name, _out):
        for l, (layer_op, corners_op) in enumerate(plan.bufs["layer_ops"]):
            if name == layer_op:
                got[f"layer{l}"] = plan.bufs["layers"][l].float().cpu()
            if name == corners_op:
                got[f"corners{l}"] = plan.bufs["corners"][l % 2].float().cpu()

    plan.run(debug=grab)
    torch.cuda.synchronize()
    idx = plan.bufs["topk_idx"].cpu()
    ref = _oracle(size, model)(images, intermediates=True, force_topk=idx)
    rows = []

    def rel(stage, a, b):
        a, b = a.float().reshape(-1), b.float().reshape(-1)
        d = (a - b).abs()
        r = (d.max() / b.abs().max()).item()
        rows.append((stage, d.max().item(), d.mean().item(), r))
        return r

    for i, fm in enumerate(plan.bufs["backbone"]):
        assert rel(f"backbone{i}", fm.view().permute(0, 3, 1, 2).cpu(), ref["backbone"][i]) <= STAGE_REL_TOL["backbone"]
    for i, fm in enumerate(plan.bufs["encoder"]):
        assert rel(f"encoder{i}", fm.view().permute(0, 3, 1, 2).cpu(), ref["encoder"][i]) <= STAGE_REL_TOL["encoder"]
    for l in range(nl):
        assert rel(f"layer{l}", got[f"layer{l}"], ref["layers"][l]) <= STAGE_REL_TOL["layer"]
        assert rel(f"corners{l}", got[f"corners{l}"], ref["corners"][l]) <= STAGE_REL_TOL["corners"]
    print(f"\n{size} bf16 per-stage error vs fp32 oracle (forced selection): stage max|d| mean|d| max|d|/max|ref|")
    for st, mx, mn, r in rows:
        print(f"  {st:10s} {mx:.3e} {mn:.3e} {r:.3e}")


@pytest.mark.parametrize("size,gbatch,big,rows", [
    ("n", 2, 32, ((0, 1), (30, 31))),     # BASELINE configs[1]: DETRPose-N bf16 batch 32, 1 GPU
    ("x", 1, 32, ((0,), (31,))),          # configs[3]: DETRPose-X bf16 256 over 8 GPUs = 32 per rank
])
def test_bf16_baseline_batch(golden_dir, size, gbatch, big, rows):
    """A BASELINE config at its own per-GPU batch: the golden images placed at the first
    and last rows of the batch give the same top-k and outputs (<=1e-4) as a plan at the
    golden batch, match the fp32 oracle on that selection within the bf16 bounds, and
    every output of the batch is finite."""
    g = np.load(os.path.join(golden_dir, f"detrpose_{size}_b{gbatch}.npz"))
    model, _ = _model(golden_dir, size, g, "bf16")
    img = synthetic_images(gbatch, seed=int(g["meta"][2]))
    batch = synthetic_images(big, seed=4321)
    for rr in rows:
        batch[list(rr)] = img
    ob = model(batch.cuda())
    ib = model.engine().plan(big).bufs["topk_idx"].cpu()
    ob = {k: v.float().cpu() for k, v in ob.items()}
    os_ = model(img.cuda())
    i_s = model.engine().plan(gbatch).bufs["topk_idx"].cpu()
    os_ = {k: v.float().cpu() for k, v in os_.items()}
    for k in ("pred_logits", "pred_keypoints"):
        assert torch.isfinite(ob[k]).all(), k
    for rr in rows:
        rr = list(rr)
        assert torch.equal(ib[rr], i_s), f"rows {rr}: top-k differs from the batch-{gbatch} plan"
        dk = (ob["pred_keypoints"][rr] - os_["pred_keypoints"]).abs().max().item()
        dl = (ob["pred_logits"][rr] - os_["pred_logits"]).abs().max().item()
        print(f"{size} b{big} rows {rr} vs b{gbatch}: max|dkp| {dk:.3g} max|dlogit| {dl:.3g}")
        assert dk <= 1e-4 and dl <= 1e-4, (rr, dk, dl)
    ref = _oracle(size, model)(img, force_topk=i_s)
    rr = list(rows[-1])
    dk = (ob["pred_keypoints"][rr] - ref["pred_keypoints"]).abs()
    dl = (ob["pred_logits"][rr] - ref["pred_logits"]).abs()
    msg = f"{size} b{big} rows {rr} vs fp32 oracle (forced selection): max|dkp| {dk.max():.3g} max|dlogit| {dl.max():.3g}"
    print(msg)
    assert dk.max() <= BF16_TOL_KP and dl.max() <= BF16_TOL_LOGIT, msg
    # different images give different outputs (the batch is not one image repeated)
    assert (ob["pred_keypoints"][rows[0][-1] + 1] - ob["pred_keypoints"][rows[0][0]]).abs().max() > 1e-3


# ---------------------------------------------------------------- reference call patterns


def test_eval_loop_call_pattern(golden_dir):
    """src/solver/engine.py:133-137: model.eval(); outputs = model(samples, targets); then
    the NON-deploy PostProcess (postprocesses.py:32-40) -> per-image dicts with (60, 51)
    keypoints [x*w, y*h, 1]. Keypoints come out flattened (B, 60, 34) before deploy
    (transformer.py:1320-1321)."""
    from detrpose_amd import PostProcess
    size, batch = "n", 2
    g = np.load(os.path.join(golden_dir, f"detrpose_{size}_b{batch}.npz"))
    with open(os.path.join(golden_dir, "manifest.json")) as f:
        man = json.load(f)
    model, _ = build_model(size, dtype="fp32")
    model.load_state_dict(synthetic_state_dict(man[size], seed=int(g["meta"][1])), strict=False)
    model.eval()
    images = synthetic_images(batch, seed=int(g["meta"][2])).cuda()
    targets = [{"labels": torch.zeros(1, dtype=torch.int64), "keypoints": torch.rand(1, 51)} for _ in range(batch)]
    out = model(images, targets)
    assert out["pred_keypoints"].shape == (batch, 60, 34)
    np.testing.assert_allclose(out["pred_keypoints"].cpu().numpy(), g["out_pred_keypoints"].reshape(batch, 60, 34),
                               atol=1e-3)
    ts = torch.tensor(np.tile(g["pp_target_size"], (batch, 1)), device="cuda")
    res = PostProcess(60, 17)(out, ts)
    assert isinstance(res, list) and len(res) == batch
    exp = np.concatenate([g["pp_keypoints"], np.ones_like(g["pp_keypoints"][..., :1])], -1).reshape(batch, 60, 51)
    for b, r in enumerate(res):
        np.testing.assert_allclose(r["scores"].cpu().numpy(), g["pp_scores"][b], atol=1e-3)
        np.testing.assert_array_equal(r["labels"].cpu().numpy(), g["pp_labels"][b])
        np.testing.assert_allclose(r["keypoints"].cpu().numpy(), exp[b], atol=640 * 1e-3)


def test_deploy_model_boundary(golden_dir):
    """tools/deployment/export_onnx.py:46-56: Model(images, orig_target_sizes) ->
    (scores, labels, keypoints); eager and hipGraph-replay forms agree with the golden
    deploy PostProcess."""
    from detrpose_amd.export import DeployModel
    size, batch = "n", 2
    g = np.load(os.path.join(golden_dir, f"detrpose_{size}_b{batch}.npz"))
    model, pp = _model(golden_dir, size, g, "fp32")
    dm = DeployModel(model, pp)
    images = synthetic_images(batch, seed=int(g["meta"][2])).cuda()
    ts = torch.tensor(np.tile(g["pp_target_size"], (batch, 1)), device="cuda")
    for s, l, k in (dm(images, ts), dm.replay(images, ts)):
        torch.cuda.synchronize()
        np.testing.assert_allclose(s.cpu().numpy(), g["pp_scores"], atol=1e-3)
        np.testing.assert_array_equal(l.cpu().numpy(), g["pp_labels"])
        np.testing.assert_allclose(k.cpu().numpy(), g["pp_keypoints"], atol=640 * 1e-3)
    with pytest.raises(ValueError):
        model(torch.rand(1, 3, 320, 320, device="cuda"))


@pytest.mark.parametrize("size,batch", [("l", 2), ("l", 9), ("x", 1)])
def test_stem_fused_bit_identical(golden_dir, size, batch, monkeypatch):
    """dp_stem_fused (the whole StemBlock in one launch, hgnetv2.py:204-220) writes exactly
    the map of the five-launch path (stem1, stem2a + pool, stem2b, stem3, stem4): same K
    order, f32 accumulation sequence and bf16 rounding points. Also the end outputs. L b9
    has 900 tiles, more than the one-block-per-CU grid: blocks run the pipelined steady state
    (stem3/stem4 of one tile beside stem1 of the next) over several tiles."""
    from detrpose_amd.engine import Engine
    with open(os.path.join(golden_dir, "manifest.json")) as f:
        man = json.load(f)
    model, _ = build_model(size, dtype="bf16")
    model.load_state_dict(synthetic_state_dict(man[size], seed=0), strict=False)
    model.eval()
    img = synthetic_images(batch, seed=5).cuda()
    outs = {}
    for fused in (True, False):
        if fused:
            monkeypatch.delenv("DETRPOSE_NO_STEM_FUSE", raising=False)
        else:
            monkeypatch.setenv("DETRPOSE_NO_STEM_FUSE", "1")
        plan = Engine(model, "bf16", device="cuda").plan(batch)
        names = [n for n, _, _ in plan.ops]
        assert ("stem" in names) == fused and ("stem1" in names) != fused
        plan.input.copy_(img)
        plan.run()
        torch.cuda.synchronize()
        outs[fused] = (plan.op_out["stem" if fused else "stem4"].view().clone(),
                       plan.outputs["pred_logits"].clone(), plan.outputs["pred_keypoints"].clone())
    for a, b, what in zip(outs[True], outs[False], ("stem4 map", "logits", "keypoints")):
        assert torch.equal(a, b), what
