"""Pin the CPU oracle (oracle/detrpose_cpu.py) to the reference.

The fixtures were produced by running the reference itself (tests/golden/make_golden.py);
these tests show that the oracle restates it, so the oracle can check the HIP path.
"""
import json
import os

import numpy as np
import pytest
import torch

from detrpose_amd.configs import get_config
from detrpose_amd.synthetic import synthetic_images, synthetic_state_dict
from oracle.detrpose_cpu import OracleDETRPose, msda_core, postprocess, sine_pos_embed_2d, weighting_function

CASES = [("n", 2), ("l", 1), ("x", 1)]


def _load(golden_dir, size, batch):
    return np.load(os.path.join(golden_dir, f"detrpose_{size}_b{batch}.npz"))


def _sampled(g, name, t):
    return t.reshape(-1).numpy()[g[name + "__idx"]], g[name + "__val"]


@pytest.fixture(scope="module")
def manifest(golden_dir):
    with open(os.path.join(golden_dir, "manifest.json")) as f:
        return json.load(f)


@pytest.mark.parametrize("size,batch", CASES)
def test_oracle_end_to_end(golden_dir, manifest, size, batch):
    torch.set_num_threads(max(1, min(8, len(os.sched_getaffinity(0)))))
    g = _load(golden_dir, size, batch)
    sd = synthetic_state_dict(manifest[size], seed=int(g["meta"][1]))
    out = OracleDETRPose(get_config(size), sd)(synthetic_images(batch, seed=int(g["meta"][2])), intermediates=True)
    assert (out["topk_idx"].numpy() == g["topk_idx"]).all()
    for i, f in enumerate(out["backbone"]):
        a, b = _sampled(g, f"backbone{i}", f)
        np.testing.assert_allclose(a, b, atol=1e-5, rtol=1e-5)
    for i, f in enumerate(out["encoder"]):
        a, b = _sampled(g, f"encoder{i}", f)
        np.testing.assert_allclose(a, b, atol=1e-4, rtol=1e-4)
    for i, f in enumerate(out["layers"]):
        a, b = _sampled(g, f"dec_layer{i}", f)
        np.testing.assert_allclose(a, b, atol=1e-4, rtol=1e-4)
    np.testing.assert_allclose(out["pred_logits"].numpy(), g["out_pred_logits"], atol=1e-4)
    np.testing.assert_allclose(out["pred_keypoints"].numpy(), g["out_pred_keypoints"], atol=1e-4)
    ts = torch.from_numpy(np.tile(g["pp_target_size"], (batch, 1)))
    s, l, k = postprocess(out["pred_logits"], out["pred_keypoints"], ts)
    np.testing.assert_allclose(s.numpy(), g["pp_scores"], atol=1e-5)
    assert (l.numpy() == g["pp_labels"]).all()
    np.testing.assert_allclose(k.numpy(), g["pp_keypoints"], atol=640 * 1e-4)


@pytest.mark.parametrize("size", ["n", "l", "x"])
def test_oracle_msda_vectors(golden_dir, size):
    g = np.load(os.path.join(golden_dir, f"msda_{size}.npz"))
    shapes = [tuple(int(v) for v in s) for s in g["shapes"]]
    out = msda_core(torch.from_numpy(g["value"]), shapes, torch.from_numpy(g["loc"]), torch.from_numpy(g["attn"]))
    np.testing.assert_allclose(out.numpy(), g["out"], atol=2e-5, rtol=1e-5)


def test_oracle_misc(golden_dir):
    g = np.load(os.path.join(golden_dir, "misc.npz"))
    for rs in (4, 8):
        np.testing.assert_allclose(weighting_function(32, 0.5, float(rs)).numpy(), g[f"project_rs{rs}"].reshape(-1),
                                   atol=1e-6)
    for size, C in (("n", 128), ("l", 256), ("x", 384)):
        np.testing.assert_allclose(sine_pos_embed_2d(20, 20, C // 2, 20).numpy(), g[f"pos_embed_{size}"], atol=1e-6)


def test_oracle_forced_selection(golden_dir, manifest):
    """force_topk (the hook the bf16 GPU test uses) with the reference's own selection
    reproduces the reference outputs; a different selection changes them."""
    g = _load(golden_dir, "n", 2)
    sd = synthetic_state_dict(manifest["n"], seed=int(g["meta"][1]))
    orc = OracleDETRPose(get_config("n"), sd)
    img = synthetic_images(2, seed=int(g["meta"][2]))
    out = orc(img, force_topk=torch.from_numpy(g["topk_idx"]))
    np.testing.assert_allclose(out["pred_keypoints"].numpy(), g["out_pred_keypoints"], atol=1e-4)
    np.testing.assert_allclose(out["pred_logits"].numpy(), g["out_pred_logits"], atol=1e-4)
    other = torch.from_numpy(g["topk_idx"]).flip(1)
    out2 = orc(img, force_topk=other)
    assert (out2["pred_keypoints"] - out["pred_keypoints"]).abs().max() > 1e-3
