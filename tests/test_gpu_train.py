"""Training-mode forward (no denoising, frozen BN) and the criterion on its outputs.

The reference's own non-DN training forward stops with UnboundLocalError at
transformer.py:1353; tests/golden/make_train_golden.py captures every value it computes
before that line (decoder return, two-stage tensors) from the reference on the N golden
images (b2), BatchNorm in eval mode: tests/golden/train_forward_n_b2.npz. The HIP path in
fp32 parity mode must match every output of every layer within the north-star gate
(1e-3 abs on logits / keypoints; pred_corners, distribution logits of scale ~10, within
1e-3 of their scale). In bf16 the training plan's final outputs must equal the inference
plan's bit for bit (same kernels), and the criterion must consume the dict as the
reference's would.
"""
import json
import os

import numpy as np
import pytest
import torch

from detrpose_amd import build_model
from detrpose_amd.synthetic import synthetic_images, synthetic_state_dict

pytestmark = pytest.mark.gpu


def _model(golden_dir, size, seed, dtype):
    with open(os.path.join(golden_dir, "manifest.json")) as f:
        man = json.load(f)
    model, _ = build_model(size, dtype=dtype)
    model.load_state_dict(synthetic_state_dict(man[size], seed=seed), strict=False)
    return model


def _frozen_bn_train(model):
    model.train()
    for m in model.modules():
        if isinstance(m, torch.nn.modules.batchnorm._BatchNorm):
            m.eval()
    return model


def test_train_forward_matches_reference(golden_dir):
    g = np.load(os.path.join(golden_dir, "train_forward_n_b2.npz"))
    batch, wseed, iseed = (int(v) for v in g["meta"])
    model = _frozen_bn_train(_model(golden_dir, "n", wseed, "fp32"))
    out = model(synthetic_images(batch, seed=iseed).cuda())
    torch.cuda.synchronize()
    heads = {"out": out, "pre": out["aux_pre_outputs"], "interm": out["aux_interm_outputs"][0]}
    heads.update({f"aux{i}": a for i, a in enumerate(out["aux_outputs"])})
    n = 0
    for key in g.files:
        if key == "meta":
            continue
        name, field = key.split(".")
        got = heads[name][field].float().cpu().numpy()
        ref = g[key]
        assert got.shape == ref.shape, (key, got.shape, ref.shape)
        tol = 1e-3 * max(1.0, float(np.abs(ref).max())) if field == "pred_corners" else 1e-3
        np.testing.assert_allclose(got, ref, atol=tol, rtol=0, err_msg=key)
        n += 1
    assert n == 4 * len(out["aux_outputs"]) + 4 + 2 + 2
    assert out["aux_outputs"][0]["teacher_corners"] is out["pred_corners"]
    assert float(out["reg_scale"]) == 4.0 and out["reg_max"] == 32


def test_train_forward_refusals(golden_dir):
    model = _model(golden_dir, "n", 0, "fp32")
    img = synthetic_images(1, seed=1).cuda()
    model.train()   # encoder BatchNorm in train mode: batch statistics are not built
    with pytest.raises(NotImplementedError):
        model(img)
    _frozen_bn_train(model)
    with pytest.raises(ValueError):   # targets -> denoising queries, which need the xyxy boxes
        model(img, [{"labels": torch.zeros(1, dtype=torch.int64).cuda(), "keypoints": torch.rand(1, 51).cuda(),
                     "area": torch.rand(1).cuda()}])


def test_train_forward_bf16_and_criterion(golden_dir):
    from detrpose_amd.criterion import Criterion, HungarianMatcher
    batch = 4
    model = _model(golden_dir, "l", 0, "bf16")
    img = synthetic_images(batch, seed=1).cuda()
    ev = model.eval()(img)
    out = _frozen_bn_train(model)(img)
    assert torch.equal(out["pred_logits"], ev["pred_logits"])
    assert torch.equal(out["pred_keypoints"], ev["pred_keypoints"])
    assert len(out["aux_outputs"]) == 5
    gen = torch.Generator().manual_seed(3)
    targets = []
    for n in (3, 0, 5, 1):
        kp = torch.cat([torch.rand(n, 34, generator=gen), (torch.rand(n, 17, generator=gen) > 0.3).float()], 1)
        targets.append({"labels": torch.zeros(n, dtype=torch.int64).cuda(), "keypoints": kp.cuda(),
                        "area": (torch.rand(n, generator=gen) * 0.2 + 0.01).cuda()})
    crit = Criterion(2, HungarianMatcher(2.0, 0.25, 10.0, 4.0), {"loss_vfl": 2.0, "loss_keypoints": 10.0,
                                                                 "loss_oks": 4.0}, ["vfl", "keypoints"], 17)
    losses = crit(out, targets)
    assert len(losses) == 3 * (1 + 5 + 1 + 1)
    vals = torch.stack(list(losses.values()))
    assert torch.isfinite(vals).all() and (vals >= 0).all()


def test_train_forward_with_targets_autograd(golden_dir):
    """The reference's training loop on the drop-in API (src/solver/engine.py:34-60):
    outputs = model(samples, targets) with OKS-denoising queries, loss = sum(criterion(outputs,
    targets).values()), loss.backward() -> every transformer parameter has a .grad, equal to the
    training plan's own gradient for the same DN draws (the autograd glue hands the Criterion's
    gradients to the recorded backward unchanged)."""
    from detrpose_amd.criterion import Criterion, HungarianMatcher, pack_targets
    model = _model(golden_dir, "n", 0, "fp32").cuda()
    _frozen_bn_train(model)
    img = synthetic_images(2, seed=1).cuda()
    gen = torch.Generator().manual_seed(4)
    targets = []
    for n in (3, 2):
        c = torch.rand(n, 2, generator=gen) * 0.6 + 0.2
        wh = torch.rand(n, 2, generator=gen) * 0.3 + 0.05
        kp = torch.cat([torch.rand(n, 34, generator=gen), (torch.rand(n, 17, generator=gen) > 0.3).float()], 1)
        targets.append({"labels": torch.tensor([i % 2 for i in range(n)]).cuda(), "keypoints": kp.cuda(),
                        "boxes": torch.cat([c - wh / 2, c + wh / 2], 1).cuda(), "area": (wh.prod(1) * 0.53).cuda()})
    crit = Criterion(2, HungarianMatcher(2.0, 0.25, 10.0, 4.0), {"loss_vfl": 2.0, "loss_keypoints": 10.0,
                                                                 "loss_oks": 4.0}, ["vfl", "keypoints"], 17)
    out = model(img, targets)
    assert out["dn_meta"] == {"pad_size": 36, "num_dn_group": 6}   # 3 targets at most: 40 // 6 groups
    assert len(out["dn_aux_outputs"]) == 3 and out["dn_aux_outputs"][0]["pred_logits"].shape == (2, 36, 2)
    losses = crit(out, targets)
    assert len(losses) == 27 and any(k.endswith("_dn_pre") for k in losses)
    loss = sum(losses.values())
    assert torch.isfinite(loss)
    loss.backward()
    tr = model._trainer
    names = [n for n, p in model.named_parameters() if n.startswith("transformer.") and p.requires_grad]
    assert all(dict(model.named_parameters())[n].grad is not None for n in names)
    # the plan's own hand-off on the same draws
    plan = next(p for p in tr.eng.plans.values() if p.P == 36)
    packed = pack_targets(targets, 17, img.device)
    keys, vals = plan.criterion(packed, packed.sizes, 6)
    ref_losses = dict(zip(keys, vals.cpu().tolist()))
    for k, v in losses.items():
        assert abs(float(v) - ref_losses[k]) <= 1e-5 * max(1.0, abs(ref_losses[k])), k
    plan.backward()
    torch.cuda.synchronize()
    params = dict(model.named_parameters())
    rows = sorted(((float((params[n].grad - tr.eng.grads[n]).abs().max()) /
                    max(float(tr.eng.grads[n].abs().max()), 1e-12), n, float(tr.eng.grads[n].abs().max()),
                    float(params[n].grad.abs().max())) for n in names), reverse=True)
    print("autograd vs plan gradient: worst relative differences", rows[:6])
    assert rows[0][0] <= 1e-5


def test_train_forward_full_network_autograd(golden_dir):
    """The reference's training loop with the model in train mode (encoder BatchNorm on batch
    statistics): model(samples, targets) -> criterion -> loss.backward() gives EVERY trainable
    parameter (backbone, encoder, transformer) a .grad equal to the training tapes' own gradient
    replayed on the same forward, and the encoder's BatchNorm running statistics move."""
    from detrpose_amd.criterion import Criterion, HungarianMatcher, pack_targets
    model = _model(golden_dir, "n", 0, "fp32").cuda()
    model.train()
    rm0 = model.encoder.input_proj[0].norm.running_mean.clone()
    img = synthetic_images(2, seed=1).cuda()
    gen = torch.Generator().manual_seed(4)
    targets = []
    for n in (3, 2):
        c = torch.rand(n, 2, generator=gen) * 0.6 + 0.2
        wh = torch.rand(n, 2, generator=gen) * 0.3 + 0.05
        kp = torch.cat([torch.rand(n, 34, generator=gen), (torch.rand(n, 17, generator=gen) > 0.3).float()], 1)
        targets.append({"labels": torch.tensor([i % 2 for i in range(n)]).cuda(), "keypoints": kp.cuda(),
                        "boxes": torch.cat([c - wh / 2, c + wh / 2], 1).cuda(), "area": (wh.prod(1) * 0.53).cuda()})
    crit = Criterion(2, HungarianMatcher(2.0, 0.25, 10.0, 4.0), {"loss_vfl": 2.0, "loss_keypoints": 10.0,
                                                                 "loss_oks": 4.0}, ["vfl", "keypoints"], 17)
    out = model(img, targets)
    loss = sum(crit(out, targets).values())
    assert torch.isfinite(loss)
    loss.backward()
    tr = model._trainer
    assert tr.scope == "full"
    params = dict(model.named_parameters())
    names = [n for n, p in params.items() if p.requires_grad]
    assert all(params[n].grad is not None for n in names), [n for n in names if params[n].grad is None][:5]
    assert sum(n.startswith("backbone.") for n in names) > 100 and sum(n.startswith("encoder.") for n in names) > 50
    assert not torch.equal(rm0, model.encoder.input_proj[0].norm.running_mean)
    # replay: the plan's own criterion + the three backward tapes on the same forward
    plan = next(p for p in tr.eng.plans.values() if p.P == 36)
    packed = pack_targets(targets, 17, img.device)
    plan.criterion(packed, packed.sizes, 6)
    plan.backward()
    tr.ep.backward()
    tr.bb.backward()
    torch.cuda.synchronize()
    # relative to each gradient's scale, floored at 1e-4 of the largest (analytically-zero BN
    # biases ahead of a training-mode BatchNorm carry only atomic-order noise); the LAB scalars
    # (sums over whole maps that cancel, f32 atomics in another order) to 2.5e-2
    top = max(float(tr.eng.grads[n].abs().max()) for n in names)
    rows = sorted(((float((params[n].grad - tr.eng.grads[n]).abs().max()) /
                    max(float(tr.eng.grads[n].abs().max()), 1e-4 * top) / (50.0 if params[n].numel() == 1 else 1.0),
                    n) for n in names), reverse=True)
    print("autograd vs tapes: worst relative differences (scalars / 50)", rows[:6])
    assert rows[0][0] <= 5e-4


def test_trainer_full_steps_reduce_the_loss(golden_dir):
    """Trainer(scope='full') end to end on N bf16: backbone + encoder (BN batch statistics) +
    transformer, clip + AdamW (backbone lr 1e-5) + EMA; six steps on one batch lower the loss."""
    from detrpose_amd.train import Trainer
    g = np.load(os.path.join(golden_dir, "train_dn_n_b2.npz"))
    model, _ = build_model("n")
    from detrpose_amd.synthetic import load_synthetic
    load_synthetic(model, seed=int(g["meta"][1]))
    dev = torch.device("cuda")
    tr = Trainer(model, dtype="bf16", device=dev, lr=2e-4, backbone_lr=2e-5)
    images = synthetic_images(2, seed=1).to(dev)
    sizes = [int(v) for v in g["sizes"]]
    off = np.concatenate([[0], np.cumsum(sizes)])
    ts = [{"labels": torch.as_tensor(g["tgt_labels"][off[b]:off[b + 1]]).to(dev),
           "keypoints": torch.as_tensor(g["tgt_kps"][off[b]:off[b + 1]]).to(dev),
           "area": torch.as_tensor(g["tgt_area"][off[b]:off[b + 1]]).to(dev),
           "boxes": torch.as_tensor(g["tgt_boxes"][off[b]:off[b + 1]]).to(dev)} for b in range(len(sizes))]
    totals = []
    for _ in range(6):
        keys, vals = tr.step(images, ts)
        totals.append(float(vals.sum()))
    print("full-network bf16 total loss per step:", [round(t, 3) for t in totals])
    assert all(np.isfinite(totals)) and len(keys) == 27
    assert totals[-1] < totals[0], totals
    assert tr.eng.ema_updates == 6 and torch.isfinite(tr.eng.ema).all()
