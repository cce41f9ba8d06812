"""The transformer training step on the HIP kernels (detrpose_amd/train_engine.py) against the
reference's own DN training step (tests/golden/train_dn_n_b2.npz) and the pinned training oracle
(oracle/train_cpu.py, tests/test_train_oracle.py): every head output, every loss (incl. the
dn_* losses) and the gradient of every transformer parameter, fp32 mode, N at batch 2 with the
reference's DN draws. The encoder memory is the oracle's (the step differentiates the
transformer; the encoder is an input)."""
import os

import numpy as np
import pytest
import torch

from detrpose_amd import build_model
from detrpose_amd.criterion import pack_targets
from detrpose_amd.synthetic import load_synthetic

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))


def _targets(g, dev):
    sizes = [int(v) for v in g["sizes"]]
    off = np.concatenate([[0], np.cumsum(sizes)])
    ts = []
    for b in range(len(sizes)):
        sl = slice(off[b], off[b + 1])
        ts.append({"labels": torch.as_tensor(g["tgt_labels"][sl]).to(dev),
                   "keypoints": torch.as_tensor(g["tgt_kps"][sl]).to(dev),
                   "area": torch.as_tensor(g["tgt_area"][sl]).to(dev),
                   "boxes": torch.as_tensor(g["tgt_boxes"][sl]).to(dev)})
    return sizes, ts


@pytest.fixture(scope="module")
def step(golden_dir):
    import sys
    sys.path.insert(0, HERE)
    from test_train_oracle import dn_inputs, oracle_train_step
    from detrpose_amd.train_engine import TrainEngine
    g = np.load(os.path.join(golden_dir, "train_dn_n_b2.npz"))
    res, ld, grads, feats = oracle_train_step("n", g)
    model, _ = build_model("n", dtype="fp32")
    load_synthetic(model, seed=int(g["meta"][1]))
    dev = torch.device("cuda")
    eng = TrainEngine(model, "fp32", dev)
    B = int(g["meta"][0])
    shapes = [(f.shape[2], f.shape[3]) for f in feats]
    memory = torch.cat([f.flatten(2).permute(0, 2, 1) for f in feats], 1)
    P = int(g["dn_pad_size"])
    plan = eng.plan(B, P, shapes)
    plan.set_inputs(memory.to(dev), dn_inputs(g))
    sizes, ts = _targets(g, dev)
    packed = pack_targets(ts, 17, dev)
    plan.forward()
    keys, vals = plan.criterion(packed, sizes, int(g["dn_num_group"]))
    plan.backward()
    torch.cuda.synchronize()
    return g, res, ld, grads, plan, eng, dict(zip(keys, vals.cpu().tolist()))


def test_train_forward_heads(step):
    """Every layer's logits / keypoints (matching and DN rows), pre and interm heads."""
    g, res, _, _, plan, eng, _ = step
    P, L = plan.P, eng.L
    got = {}
    for l in range(L):
        name = "out" if l == L - 1 else f"aux{l}"
        got[name] = (plan.logits[l][:, P:], plan.kps[l][:, P:].flatten(-2))
        got[f"dn{l}"] = (plan.logits[l][:, :P], plan.kps[l][:, :P].flatten(-2))
    got["pre"] = (plan.pre_logits[:, P:], plan.pre_out[:, P:].flatten(-2))
    got["dn_pre"] = (plan.pre_logits[:, :P], plan.pre_out[:, :P].flatten(-2))
    got["interm"] = (plan.interm_logits, plan.ref0[:, :, 1:].flatten(-2))
    bad = []
    for name, (lg, kp) in got.items():
        for k, t in (("pred_logits", lg), ("pred_keypoints", kp)):
            ref = g[f"{name}.{k}"]
            err = float(np.abs(t.cpu().numpy() - ref).max())
            print(f"{name}.{k}: max|d| {err:.3g}")
            if err > 1e-3:
                bad.append((name, k, err))
    assert not bad, bad


def test_train_losses_match_reference(step):
    """All 27 losses (final, aux, pre, interm, dn_0..2, dn_pre) within 1e-5 relative."""
    g, _, _, _, _, _, losses = step
    ref = dict(zip([str(k) for k in g["loss_keys"]], g["loss_vals"]))
    assert sorted(losses) == sorted(ref)
    for k in sorted(ref):
        print(f"{k}: {losses[k]:.6f} ref {ref[k]:.6f}")
    for k in ref:
        assert abs(losses[k] - ref[k]) <= 1e-5 * max(abs(ref[k]), 1.0), (k, losses[k], ref[k])


def test_train_gradients_match_reference(step):
    """Every transformer parameter's gradient within 1e-3 of its scale (max |g| of the
    reference gradient), fp32."""
    g, _, _, ograds, plan, eng, _ = step
    names = [k for k in g.files if k.startswith("grad.")]
    rows = []
    for k in names:
        ref = g[k]
        got = eng.grads["transformer." + k[len("grad."):]].cpu().numpy()
        scale = max(float(np.abs(ref).max()), 1e-12)
        rows.append((float(np.abs(got - ref).max()) / scale, k))
    rows.sort(reverse=True)
    for err, k in rows[:25]:
        print(f"{k}: {err:.3g}")
    assert rows[0][0] <= 1e-3, rows[:10]
