"""Generate the training-criterion fixtures under tests/golden/ by running the REFERENCE
HungarianMatcher + Criterion (read-only at /root/reference) on CPU-constructed decoder
outputs (training parity is pinned on the criterion with such inputs; the
DN path needs .cuda()).

    PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_train_golden.py

Import recipe: make_golden._import_reference() plus two bare namespaces the criterion's
import chain needs: `src.data` (its __init__ pulls cv2) and `src.data.dataloader` (imported by
src/misc/dist_utils.py for a DataLoader class the criterion never uses; torchvision's
transforms are absent), stubbed as an empty module.

One deliberate change to the reference's behaviour: Criterion._get_go_indices orders the
(query, target) pair counts with torch.argsort(descending=True) (criterion.py:258), whose
order among EQUAL counts is unspecified (on CPU it is not stable: it differs from
torch.sort(stable=True) on ties). While the criterion runs here torch.argsort is replaced by
the stable sort, so that among tied counts the smaller target index wins: the rule
detrpose_amd (dp_match_union) and the oracle implement. Without it the chosen target of a
tied query is an artefact of the sort kernel. Everything else runs unmodified.

Output: criterion_{a,b,c}.npz with inputs (per-head logits / keypoints, targets), the
reference's per-head matchings, the final head's cost matrix, the union matching, the loss
dict and the gradients of sum(losses) and of the vfl losses w.r.t. every head's outputs.
"""
from __future__ import annotations

import os
import sys
import types

sys.dont_write_bytecode = True
HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)

import numpy as np  # noqa: E402
import torch  # noqa: E402

import make_golden  # noqa: E402

CASES = {
    # name: (B, Q, ncls, K, n_aux, target sizes, seed)
    "a": (4, 60, 2, 17, 5, [3, 0, 7, 1], 11),
    "b": (2, 20, 2, 17, 3, [25, 4], 12),     # an image with more targets than queries
    "c": (3, 30, 2, 14, 5, [5, 2, 9], 13),   # CrowdPose keypoints (14, other sigmas)
}


class _bn_contiguous_grad:
    """While active, every F.batch_norm output hands its backward a contiguous gradient.

    torch 2.10's CPU batch-norm backward in training mode returns wrong input / weight / bias
    gradients when the incoming gradient is channels-last strided while the input is NCHW
    contiguous (checked against central finite differences; DESIGN.md, "Training parity at
    DETRPose-L"). The reference's HybridEncoder hands exactly that layout to the BatchNorm in
    front of the AIFI layer (src_flatten = proj.flatten(2).permute(0, 2, 1),
    hybrid_encoder.py:476; its backward is a permuted view), so on this CPU build its own
    gradients of input_proj[use_encoder_idx] and of the backbone below it are wrong. Making the
    gradient contiguous changes no value of the reference's arithmetic, only the memory layout
    the backward kernel sees (the GPU kernels the reference trains on are not affected)."""

    def __enter__(self):
        import torch.nn.functional as F
        self.F, self.orig = F, F.batch_norm

        def bn(*a, **k):
            y = self.orig(*a, **k)
            if y.requires_grad:
                y.register_hook(lambda g: g.contiguous())
            return y

        F.batch_norm = bn
        return self

    def __exit__(self, *exc):
        self.F.batch_norm = self.orig
        return False


def _import_criterion():
    make_golden._import_reference()
    ref = make_golden.REF
    m = types.ModuleType("src.data")
    m.__path__ = [os.path.join(ref, "src", "data")]
    sys.modules["src.data"] = m
    dl = types.ModuleType("src.data.dataloader")
    dl.DataLoader = None
    sys.modules["src.data.dataloader"] = dl
    from src.models.detrpose.criterion import Criterion
    from src.models.detrpose.matcher import HungarianMatcher
    return Criterion, HungarianMatcher


def make_case(Criterion, HungarianMatcher, B, Q, ncls, K, n_aux, sizes, seed):
    g = torch.Generator().manual_seed(seed)
    r = np.random.default_rng(seed)
    targets = []
    for n in sizes:
        xy = torch.rand(n, K, 2, generator=g)
        vis = (torch.rand(n, K, generator=g) > 0.3).float()
        if n >= 3:
            vis[1] = 0.0                      # an instance with no visible keypoint
        kps = torch.cat([xy.flatten(1), vis], 1)
        targets.append({"labels": torch.as_tensor(r.integers(0, ncls, n), dtype=torch.int64),
                        "keypoints": kps, "area": torch.rand(n, generator=g) * 0.3 + 0.002,
                        "boxes": torch.zeros(n, 4)})
    heads = 1 + n_aux + 2   # final, aux, pre, interm
    lg, kp = [], []
    for h in range(heads):
        logit = torch.randn(B, Q, ncls, generator=g) * 2
        k = torch.sigmoid(torch.randn(B, Q, 2 * K, generator=g) * 2)
        # some queries near their image's targets, so matchings are not arbitrary
        for b, t in enumerate(targets):
            for i in range(len(t["labels"])):
                q = int(r.integers(0, Q))
                k[b, q] = (t["keypoints"][i, :2 * K] + 0.03 * torch.randn(2 * K, generator=g)).clamp(0, 1)
        lg.append(logit.requires_grad_(True))
        kp.append(k.requires_grad_(True))

    def head(i):
        return {"pred_logits": lg[i], "pred_keypoints": kp[i]}

    outputs = {**head(0), "pred_corners": torch.zeros(1), "ref_points": torch.zeros(1), "up": torch.tensor(0.5),
               "reg_scale": torch.tensor(4.0), "reg_max": 32,
               "aux_outputs": [head(1 + i) for i in range(n_aux)],
               "aux_pre_outputs": head(1 + n_aux), "aux_interm_outputs": [head(2 + n_aux)]}
    matcher = HungarianMatcher(cost_class=2.0, cost_keypoints=10.0, cost_oks=4.0, focal_alpha=0.25,
                               num_body_points=K)
    crit = Criterion(num_classes=ncls, matcher=matcher,
                     weight_dict={"loss_vfl": 2.0, "loss_keypoints": 10.0, "loss_oks": 4.0},
                     losses=["vfl", "keypoints"], num_body_points=K, focal_alpha=0.25)
    store = {"B": np.array(B), "Q": np.array(Q), "ncls": np.array(ncls), "K": np.array(K), "n_aux": np.array(n_aux),
             "sizes": np.array(sizes, np.int64)}
    for i in range(heads):
        store[f"logits{i}"] = lg[i].detach().numpy()
        store[f"kps{i}"] = kp[i].detach().numpy()
    T = sum(sizes)
    store["tgt_labels"] = torch.cat([t["labels"] for t in targets]).numpy() if T else np.zeros(0, np.int64)
    store["tgt_kps"] = torch.cat([t["keypoints"] for t in targets]).numpy() if T else np.zeros((0, 3 * K), np.float32)
    store["tgt_area"] = torch.cat([t["area"] for t in targets]).numpy() if T else np.zeros(0, np.float32)
    # per-head matchings of the reference matcher (matcher.py:47-112)
    match = np.full((heads, B, Q), -1, np.int64)
    with torch.no_grad():
        for i in range(heads):
            for b, (I, J) in enumerate(matcher(head(i), targets)):
                match[i, b, I.numpy()] = J.numpy()
    store["match"] = match
    # the final head's cost matrix (matcher.py:87), all targets of the batch as columns
    cap = {}
    orig_split = torch.Tensor.split

    def split_spy(self, sizes_, dim=0):
        if dim == -1 and self.dim() == 3 and "C" not in cap:
            cap["C"] = self.clone()
        return orig_split(self, sizes_, dim)

    torch.Tensor.split = split_spy
    try:
        with torch.no_grad():
            matcher(head(0), targets)
    finally:
        torch.Tensor.split = orig_split
    store["cost_final"] = cap["C"].numpy()
    # criterion with a stable argsort in _get_go_indices (module docstring)
    orig_argsort = torch.argsort

    def stable_argsort(x, dim=-1, descending=False, **kw):
        return torch.sort(x, dim=dim, descending=descending, stable=True)[1]

    go_cap = {}
    orig_go = Criterion._get_go_indices

    def go_spy(self, indices, indices_aux_list):
        res = orig_go(self, indices, indices_aux_list)
        go_cap["go"] = res
        return res

    torch.argsort = stable_argsort
    Criterion._get_go_indices = go_spy
    try:
        losses = crit(outputs, targets)
    finally:
        torch.argsort = orig_argsort
        Criterion._get_go_indices = orig_go
    go = np.full((B, Q), -1, np.int64)
    for b, (I, J) in enumerate(go_cap["go"]):
        go[b, I.numpy()] = J.numpy()
    store["go"] = go
    keys = sorted(losses)
    store["loss_keys"] = np.array(keys)
    store["loss_vals"] = np.array([float(losses[k]) for k in keys], np.float64)
    total = sum(losses.values())
    grads = torch.autograd.grad(total, lg + kp, retain_graph=True)
    for i in range(heads):
        store[f"grad_logits{i}"] = grads[i].numpy()
        store[f"grad_kps{i}"] = grads[heads + i].numpy()
    vfl = sum(v for k, v in losses.items() if k.startswith("loss_vfl"))
    gv = torch.autograd.grad(vfl, lg)
    for i in range(heads):
        store[f"grad_vfl_logits{i}"] = gv[i].numpy()
    print(f"  B={B} Q={Q} K={K} heads={heads} sizes={sizes}: {len(keys)} losses, "
          f"go pairs={int((go >= 0).sum())}, total={float(total):.6f}")
    return store


def golden_train_forward(ref, size, batch, wseed=0):
    """The reference's training-mode forward without denoising (targets=None) on the golden
    images, BatchNorm layers in eval mode (frozen BN: the path detrpose_amd builds).

    The reference itself cannot finish this call: without DN, Transformer.forward raises
    UnboundLocalError at transformer.py:1353 (`out_refs` is only bound on the DN branch,
    1339). Everything it computes before that line is captured by hooks: the decoder's
    return value (per-layer poses / logits / corners / references, pre poses / scores,
    transformer.py:1293-1316), its refpoints_sigmoid input (= enc_outputs_pose_coord) and the
    two-stage class scores gathered at the top-k (interm_class, 1248-1250). The dict that
    1348-1385 would assemble from them is rebuilt here the same way."""
    from detrpose_amd.synthetic import load_synthetic, synthetic_images
    torch.manual_seed(0)
    model, _ = make_golden.build_reference(ref, size)
    load_synthetic(model, seed=wseed)
    model.train()
    for m in model.modules():
        if isinstance(m, torch.nn.modules.batchnorm._BatchNorm):
            m.eval()
    images = synthetic_images(batch, seed=1)
    tr = model.transformer
    cap = {}
    h1 = tr.decoder.register_forward_hook(lambda mod, a, out: cap.__setitem__("dec", out))
    h2 = tr.decoder.register_forward_pre_hook(
        lambda mod, a, kw: cap.__setitem__("ref0", kw["refpoints_sigmoid"].clone()), with_kwargs=True)
    h3 = tr.enc_out_class_embed.register_forward_hook(lambda mod, a, out: cap.__setitem__("cls", out))
    err = None
    try:
        with torch.no_grad():
            model(images)
    except UnboundLocalError as e:
        err = str(e)
    finally:
        h1.remove(), h2.remove(), h3.remove()
    assert err is not None and "out_refs" in err, "the reference's non-DN training forward was expected to fail"
    poses, logits, corners, refs, pre_poses, pre_scores = cap["dec"]
    topk = torch.topk(cap["cls"].max(-1)[0], tr.num_queries, dim=1)[1]
    interm_cls = torch.gather(cap["cls"], 1, topk.unsqueeze(-1).repeat(1, 1, cap["cls"].shape[-1]))
    st = {"meta": np.array([batch, wseed, 1], np.int64)}
    nl = poses.shape[0]
    for l in range(nl):
        name = "out" if l == nl - 1 else f"aux{l}"
        st[f"{name}.pred_logits"] = logits[l].numpy()
        st[f"{name}.pred_keypoints"] = poses[l].flatten(-2).numpy()
        st[f"{name}.pred_corners"] = corners[l].numpy()
        st[f"{name}.ref_points"] = refs[l].numpy()
    st["pre.pred_logits"] = pre_scores.numpy()
    st["pre.pred_keypoints"] = pre_poses.numpy()
    st["interm.pred_logits"] = interm_cls.numpy()
    st["interm.pred_keypoints"] = cap["ref0"][:, :, 1:].flatten(-2).numpy()
    print(f"  [{size}] train forward b{batch}: {nl} layers (reference stopped at: {err})")
    return st


def dn_targets(B, K, sizes, seed):
    """Synthetic COCO-style targets: labels, xyxy boxes, (x, y) keypoints + visibility (0/1),
    area, all normalised."""
    g = torch.Generator().manual_seed(seed)
    out = []
    for b, n in enumerate(sizes):
        c = torch.rand(n, 2, generator=g) * 0.6 + 0.2
        wh = torch.rand(n, 2, generator=g) * 0.3 + 0.05
        boxes = torch.cat([c - wh / 2, c + wh / 2], 1)
        xy = (c[:, None] + (torch.rand(n, K, 2, generator=g) - 0.5) * wh[:, None]).clamp(0, 1)
        vis = (torch.rand(n, K, generator=g) > 0.25).float()
        out.append({"labels": (torch.arange(n) + b) % 2, "boxes": boxes,
                    "keypoints": torch.cat([xy.flatten(1), vis], 1), "area": wh.prod(1) * 0.53})
    return out


def golden_train_dn(ref, size, batch, sizes, wseed=0, tseed=21, dn_seed=5, enc_train=False, full_train=False,
                    accum=1):
    """The reference's full training step with OKS-denoising queries (transformer.py:1265-1385,
    dn_component.py:39-183) on CPU: training-mode forward WITH targets, the Criterion with its
    dn_* losses (criterion.py:385-435), loss.backward(). BatchNorm layers in eval mode (frozen
    BN) and the encoder outputs detached (a forward hook returns them detached), so the
    gradients are those of the transformer's parameters (BASELINE config 5's decoder half).

    Deliberate changes to the reference's run, none of which touches its arithmetic:
      - torch.Tensor.cuda is the identity while it runs (prepare_for_cdn and the criterion's
        DN indices call .cuda(): dn_component.py:115-116, 141-142, criterion.py:393-395);
      - prepare_for_cdn is wrapped to record the DN inputs it draws (noised labels, noised
        keypoints, attention mask, dn_meta), so the build can be fed the same ones;
      - torch.argsort is the stable sort inside the criterion (see the module docstring);
      - every BatchNorm output hands its backward a contiguous gradient (_bn_contiguous_grad:
        a torch CPU bug, not the reference's arithmetic);
      - each class_embed[l] gets a copy of its input (a forward pre-hook returning x.clone()).
        Its input output[:, :, 0] is a view of the decoder output that the next layer's
        in-place with_pos_embed (transformer.py:369) bumps the version of, so in fp32 autograd
        refuses the backward ("modified by an inplace operation"); the values of token 0
        are never modified, so the copy changes no value or gradient. It is what the
        reference's AMP training run does anyway (autocast's casts are copies).
    Stored: targets, DN inputs, every loss, the outputs of every head, and for every
    transformer parameter its gradient (full, f32).

    enc_train=True (the encoder half of config 5): the HybridEncoder runs in training mode as
    the reference trains it (its BatchNorm2d layers on batch statistics, sync_bn on one
    process), the backbone (FrozenBatchNorm2d, freeze_norm=True) is evaluated without
    gradient and its outputs enter the encoder as leaves, so the gradients stored are the
    encoder's and the transformer's parameters' plus d loss / d backbone-output ("dfeat.*"),
    and the encoder outputs ("enc.*") and every encoder BN's running statistics after the
    step's update ("bn.*") are stored too.

    full_train=True (the whole of config 5): as enc_train, but the backbone is trained too, as
    the reference configures it (freeze_at=-1: no stage or stem frozen; freeze_norm=True: its
    norms are FrozenBatchNorm2d), so every backbone parameter's gradient (conv weights, the
    LearnableAffineBlock scalars) is stored ("grad.backbone.*") with the backbone outputs
    ("bb.*") instead of d loss / d backbone-output.

    accum > 1 (train_one_epoch's gradient accumulation, src/solver/engine.py:28, 43-59; the L
    config inherits grad_accum_steps=2 from configs/detrpose/include/detrpose_hgnetv2.py:15):
    the batch is split into `accum` consecutive sub-batches, each runs its own forward (its own
    DN draws, BatchNorm batch statistics and running-statistics update), criterion (its own
    matching and num_boxes) and backward into the same .grad, exactly the loop of engine.py:43-59.
    Per sub-batch j the DN draws, losses, the matcher's per-head assignments, backbone / encoder
    outputs and the full d loss / d memory the transformer hands the encoder ("s{j}.dmem", f32
    (B/accum, sum HW, C)) are stored under "s{j}." (heads are not stored); the gradients are the
    accumulated sums, the running statistics those after the last sub-batch. d memory is stored
    whole because the backbone / encoder gradients are a badly conditioned function of it at L
    ("Training parity at DETRPose-L"): a checker drives its encoder / backbone backward
    with the reference's own d memory."""
    if accum > 1:
        return _golden_train_accum(ref, size, batch, sizes, wseed, tseed, dn_seed, accum)
    enc_train = enc_train or full_train
    from detrpose_amd.synthetic import load_synthetic, synthetic_images
    import src.models.detrpose.transformer as tmod
    Criterion, HungarianMatcher = _import_criterion()
    torch.manual_seed(0)
    model, _ = make_golden.build_reference(ref, size)
    load_synthetic(model, seed=wseed)
    model.train()
    for m in (model.backbone if enc_train else model).modules():
        if isinstance(m, torch.nn.modules.batchnorm._BatchNorm):
            m.eval()
    K = model.transformer.num_body_points
    images = synthetic_images(batch, seed=1)
    targets = dn_targets(batch, K, sizes, tseed)
    feats_cap, enc_cap, bb_cap = [], [], []
    if full_train:
        hk = model.backbone.register_forward_hook(lambda mod, a, out: bb_cap.extend(o.detach() for o in out))
        he = model.encoder.register_forward_hook(lambda mod, a, out: enc_cap.extend(o.detach() for o in out))
    elif enc_train:
        model.backbone.eval()

        def leaf_feats(mod, a, out):
            feats_cap.extend(o.detach().requires_grad_(True) for o in out)
            return list(feats_cap)

        hk = model.backbone.register_forward_hook(leaf_feats)
        he = model.encoder.register_forward_hook(lambda mod, a, out: enc_cap.extend(o.detach() for o in out))
    else:
        hk = model.encoder.register_forward_hook(lambda mod, a, out: [o.detach() for o in out])
    hcls = [m.register_forward_pre_hook(lambda mod, a: (a[0].clone(),) + tuple(a[1:]))
            for m in model.transformer.class_embed]
    cap = {}
    orig_cdn = tmod.prepare_for_cdn

    def cdn_spy(*a, **kw):
        r = orig_cdn(*a, **kw)
        cap["cdn"] = r
        return r

    orig_cuda = torch.Tensor.cuda
    orig_argsort = torch.argsort
    matcher = HungarianMatcher(cost_class=2.0, cost_keypoints=10.0, cost_oks=4.0, focal_alpha=0.25,
                               num_body_points=K)
    crit = Criterion(num_classes=2, matcher=matcher, weight_dict={"loss_vfl": 2.0, "loss_keypoints": 10.0,
                                                                 "loss_oks": 4.0},
                     losses=["vfl", "keypoints"], num_body_points=K, focal_alpha=0.25)
    tmod.prepare_for_cdn = cdn_spy
    torch.Tensor.cuda = lambda self, *a, **k: self
    bnfix = _bn_contiguous_grad().__enter__()
    try:
        torch.manual_seed(dn_seed)
        out = model(images, targets)
        torch.argsort = lambda x, dim=-1, descending=False, **kw: torch.sort(x, dim=dim, descending=descending,
                                                                             stable=True)[1]
        losses = crit(out, targets)
        torch.argsort = orig_argsort
        total = sum(losses.values())
        total.backward()
    finally:
        bnfix.__exit__()
        tmod.prepare_for_cdn = orig_cdn
        torch.Tensor.cuda = orig_cuda
        torch.argsort = orig_argsort
        hk.remove()
        if enc_train:
            he.remove()
        for h in hcls:
            h.remove()
    label, pose, mask, meta = cap["cdn"]
    st = {"meta": np.array([batch, wseed, 1, tseed, dn_seed], np.int64), "sizes": np.array(sizes, np.int64)}
    T = sum(sizes)
    st["tgt_labels"] = torch.cat([t["labels"] for t in targets]).numpy()
    st["tgt_boxes"] = torch.cat([t["boxes"] for t in targets]).numpy()
    st["tgt_kps"] = torch.cat([t["keypoints"] for t in targets]).numpy()
    st["tgt_area"] = torch.cat([t["area"] for t in targets]).numpy()
    # DN inputs as drawn: the label embedding rows come from label_enc, so store which
    # label each DN slot embeds (-1: padding) by matching the rows back to label_enc
    le = model.transformer.label_enc.weight.detach()
    lab = label[:, :, 0].detach()   # (B, pad, C)
    d = ((lab[:, :, None, :] - le[None, None]) ** 2).sum(-1)
    slot = d.argmin(-1)
    pad_zero = lab.abs().sum(-1) == 0
    st["dn_label"] = torch.where(pad_zero, torch.full_like(slot, -1), slot).numpy()
    assert float(d.min(-1)[0][~pad_zero].max()) == 0.0
    st["dn_pose_unsig"] = pose.detach().numpy()
    st["dn_attn_mask"] = mask.numpy()
    st["dn_pad_size"] = np.array(meta["pad_size"])
    st["dn_num_group"] = np.array(meta["num_dn_group"])
    keys = sorted(losses)
    st["loss_keys"] = np.array(keys)
    st["loss_vals"] = np.array([float(losses[k]) for k in keys], np.float64)

    def head(name, o):
        st[name + ".pred_logits"] = o["pred_logits"].detach().numpy()
        st[name + ".pred_keypoints"] = o["pred_keypoints"].detach().numpy()

    head("out", out)
    for i, o in enumerate(out["aux_outputs"]):
        head(f"aux{i}", o)
    head("pre", out["aux_pre_outputs"])
    head("interm", out["aux_interm_outputs"][0])
    for i, o in enumerate(out["dn_aux_outputs"]):
        head(f"dn{i}", o)
    head("dn_pre", out["dn_aux_pre_outputs"])
    ng = 0
    # enc_train: sampled (make_golden._sample: seeded indices + values, sum, |sum|) to keep the
    # fixture small; the backbone features are not stored (the checker recomputes them)
    put = (lambda name, t: make_golden._sample(st, name, t)) if enc_train else \
        (lambda name, t: st.__setitem__(name, t.detach().numpy()))
    for n, p in model.transformer.named_parameters():
        if p.grad is not None:
            put("grad." + n, p.grad)
            ng += 1
    if enc_train:
        for n, p in model.encoder.named_parameters():
            if p.grad is not None:
                put("grad.encoder." + n, p.grad)
                ng += 1
        for i, f in enumerate(feats_cap):
            put(f"dfeat{i}", f.grad)
        if full_train:
            for n, p in model.backbone.named_parameters():
                if p.grad is not None:
                    put("grad.backbone." + n, p.grad)
                    ng += 1
            for i, f in enumerate(bb_cap):
                put(f"bb{i}", f)
        for i, e in enumerate(enc_cap):
            put(f"enc{i}", e)
        for n, m in model.encoder.named_modules():
            if isinstance(m, torch.nn.modules.batchnorm._BatchNorm):
                st[f"bn.encoder.{n}.running_mean"] = m.running_mean.numpy()
                st[f"bn.encoder.{n}.running_var"] = m.running_var.numpy()
    print(f"  [{size}] DN train step b{batch} targets {sizes}: pad {meta['pad_size']} groups {meta['num_dn_group']}, "
          f"{len(keys)} losses, total {float(total):.6f}, {ng} parameter gradients")
    return st


def _dn_label_slots(model, label):
    """Which label_enc row each DN slot embeds (-1: padding), matched back from the rows."""
    le = model.transformer.label_enc.weight.detach()
    lab = label[:, :, 0].detach()   # (B, pad, C)
    d = ((lab[:, :, None, :] - le[None, None]) ** 2).sum(-1)
    slot = d.argmin(-1)
    pad_zero = lab.abs().sum(-1) == 0
    assert float(d.min(-1)[0][~pad_zero].max()) == 0.0
    return torch.where(pad_zero, torch.full_like(slot, -1), slot).numpy()


def _golden_train_accum(ref, size, batch, sizes, wseed, tseed, dn_seed, accum):
    """golden_train_dn(full_train=True, accum>1): the whole network trained, engine.py:43-59's
    sub-batch loop (see golden_train_dn's docstring for the deliberate changes and the keys)."""
    from detrpose_amd.synthetic import load_synthetic, synthetic_images
    import src.models.detrpose.transformer as tmod
    Criterion, HungarianMatcher = _import_criterion()
    assert batch % accum == 0
    sub = batch // accum
    torch.manual_seed(0)
    model, _ = make_golden.build_reference(ref, size)
    load_synthetic(model, seed=wseed)
    model.train()
    for m in model.backbone.modules():
        if isinstance(m, torch.nn.modules.batchnorm._BatchNorm):
            m.eval()
    K = model.transformer.num_body_points
    images = synthetic_images(batch, seed=1)
    targets = dn_targets(batch, K, sizes, tseed)
    bb_cap, enc_cap = [], []
    hk = model.backbone.register_forward_hook(lambda mod, a, out: bb_cap.extend(o.detach() for o in out))
    he = model.encoder.register_forward_hook(lambda mod, a, out: enc_cap.extend(o.detach() for o in out))
    hcls = [m.register_forward_pre_hook(lambda mod, a: (a[0].clone(),) + tuple(a[1:]))
            for m in model.transformer.class_embed]
    cdn = []
    orig_cdn = tmod.prepare_for_cdn

    def cdn_spy(*a, **kw):
        r = orig_cdn(*a, **kw)
        cdn.append(r)
        return r

    orig_cuda = torch.Tensor.cuda
    orig_argsort = torch.argsort
    matcher = HungarianMatcher(cost_class=2.0, cost_keypoints=10.0, cost_oks=4.0, focal_alpha=0.25,
                               num_body_points=K)
    crit = Criterion(num_classes=2, matcher=matcher, weight_dict={"loss_vfl": 2.0, "loss_keypoints": 10.0,
                                                                 "loss_oks": 4.0},
                     losses=["vfl", "keypoints"], num_body_points=K, focal_alpha=0.25)
    # the matcher's assignments per call (Criterion.forward's order: final, aux 0..L-2, pre,
    # interm; criterion.py:289-303), recorded so a checker can run on the same assignment
    calls = []
    orig_fwd = matcher.forward

    def match_spy(outputs, targets_):
        r = orig_fwd(outputs, targets_)
        calls.append(r)
        return r

    matcher.forward = match_spy
    # d loss / d (the transformer's input feats) of each sub-batch: the gradient the transformer
    # alone hands the encoder (a view of each feat, consumed only by the transformer, with a
    # grad hook), in the layout of its memory (B, sum HW, C)
    dmem = []

    def tr_pre(mod, args):
        feats = [f.view_as(f) for f in args[0]]
        parts = [None] * len(feats)

        def keep(i):
            def hook(gr):
                parts[i] = gr.detach().flatten(2).permute(0, 2, 1)
                if all(p_ is not None for p_ in parts):
                    dmem.append(torch.cat(parts, 1).contiguous())
            return hook

        for i, f in enumerate(feats):
            f.register_hook(keep(i))
        return (feats,) + tuple(args[1:])

    htr = model.transformer.register_forward_pre_hook(tr_pre)
    st = {"meta": np.array([batch, wseed, 1, tseed, dn_seed, accum], np.int64), "sizes": np.array(sizes, np.int64)}
    st["tgt_labels"] = torch.cat([t["labels"] for t in targets]).numpy()
    st["tgt_boxes"] = torch.cat([t["boxes"] for t in targets]).numpy()
    st["tgt_kps"] = torch.cat([t["keypoints"] for t in targets]).numpy()
    st["tgt_area"] = torch.cat([t["area"] for t in targets]).numpy()
    tmod.prepare_for_cdn = cdn_spy
    torch.Tensor.cuda = lambda self, *a, **k: self
    totals = []
    bnfix = _bn_contiguous_grad().__enter__()
    try:
        torch.manual_seed(dn_seed)
        for j in range(accum):          # engine.py:43-59
            sl = slice(j * sub, (j + 1) * sub)
            out = model(images[sl], targets[sl])
            torch.argsort = lambda x, dim=-1, descending=False, **kw: torch.sort(
                x, dim=dim, descending=descending, stable=True)[1]
            losses = crit(out, targets[sl])
            torch.argsort = orig_argsort
            total = sum(losses.values())
            total.backward()
            totals.append(float(total))
            label, pose, mask, meta = cdn[-1]
            p = f"s{j}."
            st[p + "dn_label"] = _dn_label_slots(model, label)
            st[p + "dn_pose_unsig"] = pose.detach().numpy()
            st[p + "dn_attn_mask"] = mask.numpy()
            st[p + "dn_pad_size"] = np.array(meta["pad_size"])
            st[p + "dn_num_group"] = np.array(meta["num_dn_group"])
            keys = sorted(losses)
            st[p + "loss_keys"] = np.array(keys)
            st[p + "loss_vals"] = np.array([float(losses[k]) for k in keys], np.float64)
            nq = out["pred_logits"].shape[1]
            match = np.full((len(calls), sub, nq), -1, np.int64)
            for h, r in enumerate(calls):
                for b, (I, J) in enumerate(r):
                    match[h, b, I.numpy()] = J.numpy()
            st[p + "match"] = match
            calls.clear()
            st[p + "dmem"] = dmem[-1].numpy().astype(np.float32)
    finally:
        bnfix.__exit__()
        tmod.prepare_for_cdn = orig_cdn
        torch.Tensor.cuda = orig_cuda
        torch.argsort = orig_argsort
        hk.remove()
        he.remove()
        htr.remove()
        for h in hcls:
            h.remove()
    nb, ne = len(bb_cap) // accum, len(enc_cap) // accum
    for j in range(accum):
        for i in range(nb):
            make_golden._sample(st, f"s{j}.bb{i}", bb_cap[j * nb + i])
        for i in range(ne):
            make_golden._sample(st, f"s{j}.enc{i}", enc_cap[j * ne + i])
    ng = 0
    for prefix, mod in (("", model.transformer), ("encoder.", model.encoder), ("backbone.", model.backbone)):
        for n, p in mod.named_parameters():
            if p.grad is not None:
                make_golden._sample(st, "grad." + prefix + n, p.grad)
                ng += 1
    for n, m in model.encoder.named_modules():
        if isinstance(m, torch.nn.modules.batchnorm._BatchNorm):
            st[f"bn.encoder.{n}.running_mean"] = m.running_mean.numpy()
            st[f"bn.encoder.{n}.running_var"] = m.running_var.numpy()
    print(f"  [{size}] DN train step b{batch} = {accum} x b{sub}, targets {sizes}: pads "
          f"{[int(st[f's{j}.dn_pad_size']) for j in range(accum)]}, totals {totals}, {ng} parameter gradients")
    return st


def main():
    torch.set_num_threads(max(1, len(os.sched_getaffinity(0))))
    Criterion, HungarianMatcher = _import_criterion()
    ref = make_golden._import_reference()
    if os.environ.get("ONLY_FULL_L"):
        st = golden_train_dn(ref, "l", 2, [3, 1], full_train=True, accum=2)
        np.savez_compressed(os.path.join(HERE, "train_full_l_b2a2.npz"), **st)
        print("wrote train_full_l_b2a2.npz")
        return
    if os.environ.get("ONLY_FULL"):
        st = golden_train_dn(ref, "n", 2, [3, 1], full_train=True)
        np.savez_compressed(os.path.join(HERE, "train_full_n_b2.npz"), **st)
        print("wrote train_full_n_b2.npz")
        return
    if os.environ.get("ONLY_DN_ENC"):
        st = golden_train_dn(ref, "n", 2, [3, 1], enc_train=True)
        np.savez_compressed(os.path.join(HERE, "train_dn_enc_n_b2.npz"), **st)
        print("wrote train_dn_enc_n_b2.npz")
        return
    if os.environ.get("ONLY_DN"):
        st = golden_train_dn(ref, "n", 2, [3, 1])
        np.savez_compressed(os.path.join(HERE, "train_dn_n_b2.npz"), **st)
        print("wrote train_dn_n_b2.npz")
        return
    st = golden_train_forward(ref, "n", 2)
    np.savez_compressed(os.path.join(HERE, "train_forward_n_b2.npz"), **st)
    print("wrote train_forward_n_b2.npz")
    st = golden_train_dn(ref, "n", 2, [3, 1])
    np.savez_compressed(os.path.join(HERE, "train_dn_n_b2.npz"), **st)
    print("wrote train_dn_n_b2.npz")
    for name, (B, Q, ncls, K, n_aux, sizes, seed) in CASES.items():
        st = make_case(Criterion, HungarianMatcher, B, Q, ncls, K, n_aux, sizes, seed)
        np.savez_compressed(os.path.join(HERE, f"criterion_{name}.npz"), **st)
        print("wrote", f"criterion_{name}.npz")


if __name__ == "__main__":
    main()
