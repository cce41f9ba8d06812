"""End-to-end parity of the HIP forward against the reference (golden fixtures).

fp32 mode: every stage within the north-star gate (1e-3 abs on logits / keypoints) and
the two-stage top-k order identical. bf16 mode: the selection is order-sensitive
(SURVEY.md header fact 5), so outputs are compared per matched query.
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


@pytest.mark.parametrize("size,batch", CASES)
def test_bf16_tracks_reference(golden_dir, size, batch):
    """bf16 storage / f32 accumulation: per matched query the keypoints stay close; the
    selected query set overlaps the fp32 reference's (top-k order may flip)."""
    g = np.load(os.path.join(golden_dir, f"detrpose_{size}_b{batch}.npz"))
    model, _ = _model(golden_dir, size, g, "bf16")
    out = model(synthetic_images(batch, seed=int(g["meta"][2])).cuda())
    plan = model.engine().plan(batch)
    idx = plan.bufs["topk_idx"].cpu().numpy()
    kp = out["pred_keypoints"].float().cpu().numpy()
    assert np.isfinite(kp).all() and np.isfinite(out["pred_logits"].float().cpu().numpy()).all()
    errs = []
    for b in range(batch):
        ref_pos = {int(v): q for q, v in enumerate(g["topk_idx"][b])}
        common = [(q, ref_pos[int(v)]) for q, v in enumerate(idx[b]) if int(v) in ref_pos]
        assert len(common) >= 0.75 * len(idx[b]), f"top-k overlap {len(common)}/{len(idx[b])}"
        # queries whose slot matches: identical tgt_embed, so outputs are comparable
        same = [q for q, r in common if q == r]
        if same:
            errs.append(np.abs(kp[b, same] - g["out_pred_keypoints"][b, same]).max())
    if errs:
        assert max(errs) < 0.1, f"bf16 matched-query keypoint error {max(errs):.3g}"
