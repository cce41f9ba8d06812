"""ORACLE — TEST INFRASTRUCTURE ONLY (never imported by the product path).

CPU fp32 restatement of the reference's TRAINING-mode transformer forward with OKS-denoising
queries, differentiable with torch autograd, so its gradients are the reference's:

  * two-stage selection in training mode (transformer.py:1219-1261): enc_output + LN on the
    masked memory, class head, top-k, gathered interm class scores, enc_pose_embed keypoints;
  * the denoising queries as prepare_for_cdn builds them (dn_component.py:132-153) from GIVEN
    draws (the noised labels and keypoints and the attention mask are random; the tests feed
    the draws the reference made, recorded by tests/golden/make_train_golden.py): token 0 =
    label_enc[label], tokens 1..K = pose_enc.weight, zero rows for padding slots, refs =
    sigmoid(noised inverse-sigmoid keypoints), concatenated in front of the matching queries
    (transformer.py:1278-1279);
  * every decoder layer in training mode (transformer.py:588-602, 701-728, 903-916): the
    across attention with the DN attn_mask, heads at every layer, refs detached between
    layers, pred_corners NOT detached between layers, output_pose_detach aliasing the next
    layer's in-place pos add;
  * the DN output split and the output dict (transformer.py:1331-1385).

Plus the DN losses of the criterion (criterion.py:385-435) on top of oracle/criterion_cpu.py.
Pinned to the reference by tests/golden/train_dn_n_b2.npz (tests/test_train_oracle.py).
"""
from __future__ import annotations

import math

import numpy as np
import torch
import torch.nn.functional as F

from oracle import criterion_cpu as crit
from oracle.detrpose_cpu import (anchors_and_mask, bilinear_gather, inverse_sigmoid, msda_core, sine_embedding, tap,
                                 weighting_function)

T_ = "transformer."


def _lin(x, P, p):
    return F.linear(x, P[p + ".weight"], P.get(p + ".bias"))


def _mlp(x, P, p, n):
    """utils.py:75-87."""
    for i in range(n):
        x = _lin(x, P, f"{p}.layers.{i}")
        if i < n - 1:
            x = F.relu(x)
    return x


def _ln(x, P, p):
    return F.layer_norm(x, (x.shape[-1],), P[p + ".weight"], P[p + ".bias"], 1e-5)


def _mha(x, P, p, nhead, mask=None):
    """nn.MultiheadAttention(batch_first, dropout 0) with q = k = v = x and a bool attn_mask
    (True = not allowed), F.multi_head_attention_forward's math."""
    W, b = P[p + ".in_proj_weight"], P[p + ".in_proj_bias"]
    B, L, C = x.shape
    dh = C // nhead
    q, k, v = F.linear(x, W, b).split(C, -1)
    q = q.reshape(B, L, nhead, dh).transpose(1, 2)
    k = k.reshape(B, L, nhead, dh).transpose(1, 2)
    v = v.reshape(B, L, nhead, dh).transpose(1, 2)
    s = (q / math.sqrt(dh)) @ k.transpose(-1, -2)
    if mask is not None:
        s = s.masked_fill(mask, float("-inf"))
    o = (torch.softmax(s, -1) @ v).transpose(1, 2).reshape(B, L, C)
    return F.linear(o, P[p + ".out_proj.weight"], P[p + ".out_proj.bias"])


def decoder_layer(tgt, pos, ref, memory, shapes, P, p, nhead, n_levels, n_points, mask, cut_loc=False):
    """DeformableTransformerDecoderLayer.forward (transformer.py:387-442), training mode.
    tgt (B, Q, 1+K, C) already carries the in-place pos of transformer.py:369 (the caller adds
    it, because the addition is visible to the previous layer's output_pose_detach)."""
    B, Q, T, C = tgt.shape
    x = tgt.flatten(0, 1)
    t = _ln(tgt + _mha(x, P, p + ".within_attn", nhead).reshape(B, Q, T, C), P, p + ".within_norm")
    x = t.transpose(1, 2).flatten(0, 1)   # (B*T, Q, C)
    t = _ln(x + _mha(x, P, p + ".across_attn", nhead, mask), P, p + ".across_norm").reshape(B, T, Q, C).transpose(1, 2)
    # second in-place with_pos_embed (transformer.py:422): the query AND the gate input
    t = torch.cat([t[:, :, :1], t[:, :, 1:] + pos], 2)
    query = t.flatten(1, 2)
    Lq = Q * T
    off = _lin(query, P, p + ".cross_attn.sampling_offsets").reshape(B, Lq, nhead, n_levels, n_points, 2)
    aw = _lin(query, P, p + ".cross_attn.attention_weights").reshape(B, Lq, nhead, n_levels * n_points)
    aw = torch.softmax(aw, -1).reshape(B, Lq, nhead, n_levels, n_points)
    norm = torch.tensor([[w, h] for h, w in shapes], dtype=torch.float32).reshape(1, 1, 1, n_levels, 1, 2)
    loc = ref.reshape(B, Lq, 1, 1, 1, 2) + off / norm
    if cut_loc:   # parity-analysis variant (train_transformer): no gradient through the locations
        loc = loc.detach()
    m = msda_core(memory, shapes, loc, aw).reshape(B, Q, T, C)
    g = torch.sigmoid(_lin(torch.cat([t, m], -1), P, p + ".gateway.gate"))
    g1, g2 = g.chunk(2, -1)
    t = _ln(g1 * t + g2 * m, P, p + ".gateway.norm")
    return _ln(t + _lin(F.relu(_lin(t, P, p + ".linear1")), P, p + ".linear2"), P, p + ".norm2")


def lqe(scores, kps, feat_nhwc, P, p, k=4):
    """LQE.forward (transformer.py:275-288)."""
    B, Q, K, _ = kps.shape
    s = bilinear_gather(feat_nhwc, kps.reshape(B, Q * K, 2)).reshape(B, Q, K, -1)
    top = s.topk(k, dim=-1)[0]
    stat = torch.cat([top, top.mean(-1, keepdim=True)], -1).reshape(B, Q, -1)
    return scores + _mlp(stat, P, p + ".reg_conf", 2)


def dn_queries(P, dn, B, K, C):
    """prepare_for_cdn's query tensors (dn_component.py:132-153) from given draws:
    dn["label"] (B, pad) int64 (-1 = padding slot), dn["pose_unsig"] (B, pad, 1+K, 2)."""
    lab = torch.as_tensor(dn["label"])
    pad = lab.shape[1]
    le, pe = P[T_ + "label_enc.weight"], P[T_ + "pose_enc.weight"]
    valid = (lab >= 0).to(torch.float32)[..., None, None]
    rows = torch.cat([le[lab.clamp(min=0)][:, :, None], pe[None, None].expand(B, pad, K, C)], 2)
    tgt = rows * valid
    ref = torch.sigmoid(torch.as_tensor(dn["pose_unsig"], dtype=torch.float32))
    return tgt, ref


def train_transformer(feats, P, cfg, dn=None, force_topk=None, cut_loc=False):
    """Transformer.forward in training mode (targets given => dn draws given), returning the
    reference's output dict (transformer.py:1348-1385). feats: encoder outputs (detached);
    P: name -> tensor (reference keys, parameters as autograd leaves). cut_loc: the values are
    the same, but no gradient flows through the bilinear sampling locations (MSDA's sampling
    offsets, the LQE's keypoints) — the comparison variant detrpose_amd's TrainPlan
    (cut_location_grads) mirrors, for per-parameter precision checks."""
    C, nhead, nq, K = cfg["hidden_dim"], cfg["nhead"], cfg["num_queries"], cfg["num_body_points"]
    nlayers, reg_max = cfg["num_decoder_layers"], cfg["reg_max"]
    reg_scale = float(cfg["reg_scale"])
    B = feats[0].shape[0]
    shapes = [(f.shape[2], f.shape[3]) for f in feats]
    memory = torch.cat([f.flatten(2).permute(0, 2, 1) for f in feats], 1)
    anchors, invalid = anchors_and_mask(cfg["feat_strides"], cfg["eval_spatial_size"])
    om = _ln(_lin(memory.masked_fill(invalid, 0.0), P, T_ + "enc_output"), P, T_ + "enc_output_norm")
    cls = _lin(om, P, T_ + "enc_out_class_embed")
    topk_idx = torch.topk(cls.max(-1)[0], nq, dim=1)[1] if force_topk is None else torch.as_tensor(force_topk)
    tmem = torch.gather(om, 1, topk_idx.unsqueeze(-1).expand(-1, -1, C))
    tanc = torch.gather(anchors.expand(B, -1, -1), 1, topk_idx.unsqueeze(-1).expand(-1, -1, 2))
    kp = torch.sigmoid(_mlp(tmem, P, T_ + "enc_pose_embed", 4).reshape(B, nq, K, 2) + tanc.unsqueeze(-2))
    enc_coord = torch.cat([kp.mean(2, keepdim=True), kp], 2)
    ref = enc_coord.detach()
    interm_class = torch.gather(cls, 1, topk_idx.unsqueeze(-1).expand(-1, -1, cls.shape[-1]))
    tgt_kp = P[T_ + "keypoint_embedding.weight"][None, None] + P[T_ + "tgt_embed.weight"][None, :, None]
    tgt_inst = P[T_ + "instance_embedding.weight"][None, None].expand(1, nq, 1, C)
    tgt = torch.cat([tgt_inst, tgt_kp], 2).expand(B, -1, -1, -1)
    pad = 0
    mask = None
    if dn is not None:
        dtgt, dref = dn_queries(P, dn, B, K, C)
        pad = dtgt.shape[1]
        tgt = torch.cat([dtgt, tgt], 1)
        ref = torch.cat([dref, ref], 1)
        mask = torch.as_tensor(dn["attn_mask"])
    Qt = tgt.shape[1]
    project = weighting_function(reg_max, 0.5, reg_scale).to(memory.dtype)   # float64 checker runs too
    dim_t = P[T_ + "decoder.dim_t"]
    feat0 = feats[0].permute(0, 2, 3, 1)
    out = tgt
    prev_pose_detach = None
    prev_corners = None
    poses, logits, corners_l = [], [], []
    for l in range(nlayers):
        ref_kp = ref[:, :, 1:]
        pos = _mlp(sine_embedding(ref_kp, dim_t), P, T_ + "decoder.half_pose_ref_point_head", 2)
        # in-place with_pos_embed on the layer input (transformer.py:369)
        x0 = torch.cat([out[:, :, :1], out[:, :, 1:] + pos], 2)
        if prev_pose_detach is not None:
            prev_pose_detach = x0[:, :, 1:].detach()   # the aliased view sees the pos add
        out = decoder_layer(x0, pos, ref, memory, shapes, P, f"{T_}decoder.layers.{l}", nhead,
                            cfg["num_feature_levels"], cfg["dec_n_points"], mask, cut_loc)
        pose, inst = out[:, :, 1:], out[:, :, 0]
        if l == 0:
            pre_poses = torch.sigmoid(_mlp(pose, P, T_ + "pre_pose_embed", 3) + inverse_sigmoid(ref_kp))
            pre_scores = _lin(inst, P, f"{T_}class_embed.0")
            ref_init = pre_poses.detach()
        hin = pose if prev_pose_detach is None else pose + prev_pose_detach
        corners = _mlp(hin, P, f"{T_}pose_embed.{l}", 3)
        if prev_corners is not None:
            corners = corners + prev_corners
        prob = torch.softmax(corners.reshape(-1, reg_max + 1), 1)
        d = F.linear(prob, project[None]).reshape(B, Qt, K, 2)
        kps = ref_init + d / abs(reg_scale)
        score = _lin(inst, P, f"{T_}class_embed.{l}")
        logit = lqe(score, kps.detach() if cut_loc else kps, feat0, P, f"{T_}lqe_embed.{l}")
        poses.append(kps)
        logits.append(logit)
        corners_l.append(corners)
        prev_corners = corners
        ref = torch.cat([kps.mean(2, keepdim=True), kps], 2).detach()
        prev_pose_detach = pose.detach()   # replaced by the next layer's aliased view above

    def split(t):
        return t[:, :pad], t[:, pad:]

    res = {"interm": {"pred_logits": interm_class, "pred_keypoints": enc_coord[:, :, 1:].flatten(-2)},
           "topk_idx": topk_idx}
    heads, dn_heads = [], []
    for l in range(nlayers):
        dl, ml = split(logits[l])
        dk, mk = split(poses[l].flatten(-2))
        heads.append({"pred_logits": ml, "pred_keypoints": mk})
        dn_heads.append({"pred_logits": dl, "pred_keypoints": dk})
    dpl, mpl = split(pre_scores)
    dpk, mpk = split(pre_poses.flatten(-2))
    res.update(final=heads[-1], aux=heads[:-1], pre={"pred_logits": mpl, "pred_keypoints": mpk})
    if dn is not None:
        res.update(dn=dn_heads, dn_pre={"pred_logits": dpl, "pred_keypoints": dpk},
                   dn_meta={"pad_size": pad, "num_dn_group": int(dn["num_group"])})
    return res


def dn_match(sizes, pad_size, num_group):
    """criterion.py:385-399: DN query g*single_pad + t <-> target t (positives only)."""
    single = pad_size // num_group
    m = np.full((len(sizes), pad_size), -1, np.int64)
    for b, n in enumerate(sizes):
        for g in range(num_group):
            for t in range(n):
                m[b, g * single + t] = t
    return m


def losses(res, sizes, tgt_labels, tgt_kps, tgt_area, K, ncls, weights=(2.0, 10.0, 4.0), force_match=None):
    """Criterion.forward (criterion.py:285-435) incl. the dn_* losses; force_match: the (H, B, Q)
    per-head matchings to use (criterion_cpu.criterion)."""
    heads = [(res["final"]["pred_logits"], res["final"]["pred_keypoints"])]
    heads += [(h["pred_logits"], h["pred_keypoints"]) for h in res["aux"]]
    heads += [(res["pre"]["pred_logits"], res["pre"]["pred_keypoints"]),
              (res["interm"]["pred_logits"], res["interm"]["pred_keypoints"])]
    out, matches, go = crit.criterion(heads, sizes, tgt_labels, tgt_kps, tgt_area, K, ncls, len(res["aux"]), weights,
                                      force_match)
    if "dn" in res:
        meta = res["dn_meta"]
        m = dn_match(sizes, meta["pad_size"], meta["num_dn_group"])
        nb = max(float(sum(sizes)), 1.0) * meta["num_dn_group"]
        dn = [(h["pred_logits"], h["pred_keypoints"], f"_dn_{i}") for i, h in enumerate(res["dn"])]
        dn.append((res["dn_pre"]["pred_logits"], res["dn_pre"]["pred_keypoints"], "_dn_pre"))
        for lg, kp, n in dn:
            out["loss_vfl" + n] = weights[0] * crit.loss_vfl(lg, kp, m, sizes, tgt_labels, tgt_kps, tgt_area, K, nb,
                                                             ncls)
            l1, lo = crit.loss_keypoints(kp, m, sizes, tgt_kps, tgt_area, K, nb)
            out["loss_keypoints" + n] = weights[1] * l1
            out["loss_oks" + n] = weights[2] * lo
    return dict(sorted(out.items())), matches, go


# ----------------------------------------------------------------------------- encoder (training)

def _bn_train(x, P, p, stats=None):
    """nn.BatchNorm2d in training mode (hybrid_encoder.py:68, 124): batch statistics over
    (N, H, W), biased variance for the normalisation; running statistics updated with momentum
    0.1 and the unbiased variance (F.batch_norm). stats: name -> running tensor (updated in
    place) or None."""
    rm = rv = None
    if stats is not None:
        rm, rv = stats[p + ".running_mean"], stats[p + ".running_var"]
    y = F.batch_norm(x, rm, rv, P[p + ".weight"], P[p + ".bias"], True, 0.1, 1e-5)
    if y.requires_grad:
        # torch 2.10's CPU batch-norm backward (training mode) returns wrong input / weight
        # gradients when the incoming gradient is channels-last strided while x is NCHW
        # contiguous — the layout the memory's flatten(2).permute(0, 2, 1) backward hands the
        # encoder outputs (finite-difference check in DESIGN.md, "Training parity at
        # DETRPose-L"): hand it a contiguous gradient
        y.register_hook(lambda g: g.contiguous())
    return y


def _act(x, name):
    if name is None:
        return x
    return {"relu": F.relu, "silu": F.silu, "gelu": F.gelu}[name](x)


def _conv_norm_t(x, P, p, stats, stride=1, groups=1, act=None):
    """ConvNormLayer_fuse.forward before deploy (hybrid_encoder.py:100-128), training mode."""
    w = P[p + ".conv.weight"]
    k = w.shape[-1]
    x = F.conv2d(x, w, P.get(p + ".conv.bias"), stride, (k - 1) // 2, 1, groups)
    return _act(_bn_train(x, P, p + ".norm", stats), act)


def _conv_norm_tap(x, P, p, stats, stride=1, groups=1, act=None):
    """_conv_norm_t, its output a stored layer output (the test hook oracle.detrpose_cpu.TAP)."""
    return tap(p, _conv_norm_t(x, P, p, stats, stride, groups, act))


def _vgg_t(x, P, p, stats, act):
    """VGGBlock.forward, training (hybrid_encoder.py:139-154): act(BN(conv3x3) + BN(conv1x1))."""
    return _act(_conv_norm_t(x, P, p + ".conv1", stats) + _conv_norm_t(x, P, p + ".conv2", stats), act)


def _csp_t(x, P, p, stats, nblk, act):
    """CSPLayer.forward (hybrid_encoder.py:215-240)."""
    x1 = _conv_norm_tap(x, P, p + ".conv1", stats, act=act)
    for i in range(nblk):
        x1 = _vgg_t(x1, P, f"{p}.bottlenecks.{i}", stats, act)
        if i < nblk - 1:   # the last block's output is stored with the conv2 branch added
            x1 = tap(f"{p}.bottlenecks.{i}", x1)
    return tap(p, x1 + _conv_norm_tap(x, P, p + ".conv2", stats, act=act))


def _elan_t(x, P, p, stats, nblk, act="silu"):
    """RepNCSPELAN4.forward (hybrid_encoder.py:192-212)."""
    y = _conv_norm_tap(x, P, p + ".cv1", stats, act=act)
    c = y.shape[1] // 2
    ys = [y[:, :c], y[:, c:]]
    z = _csp_t(ys[-1], P, p + ".cv2.0", stats, nblk, act)
    ys.append(_conv_norm_tap(z, P, p + ".cv2.1", stats, act=act))
    z = _csp_t(ys[-1], P, p + ".cv3.0", stats, nblk, act)
    ys.append(_conv_norm_tap(z, P, p + ".cv3.1", stats, act=act))
    return _conv_norm_tap(torch.cat(ys, 1), P, p + ".cv4", stats, act=act)


def train_encoder(feats, P, cfg, stats=None):
    """HybridEncoder.forward in training mode (hybrid_encoder.py:462-507): BatchNorm2d on batch
    statistics (sync_bn over one process), the AIFI TransformerEncoderLayer (270-296, post-norm,
    dropout 0), FPN / PAN as oracle.detrpose_cpu.encoder. feats: backbone outputs (leaves or
    detached); P: name -> tensor, encoder parameters as autograd leaves; stats: running
    statistics updated in place (optional)."""
    from oracle.detrpose_cpu import sine_pos_embed_2d
    C = cfg["hidden_dim"]
    nlev = cfg["n_levels"]
    nblk = round(3 * cfg["depth_mult"])
    enc_idx = cfg.get("use_encoder_idx", [2])
    E = "encoder."
    proj = [tap(f"{E}input_proj.{i}",
                _bn_train(F.conv2d(f, P[f"{E}input_proj.{i}.conv.weight"]), P, f"{E}input_proj.{i}.norm", stats))
            for i, f in enumerate(feats)]
    for i, ei in enumerate(enc_idx):
        B, _, H, W = proj[ei].shape
        src = proj[ei].flatten(2).permute(0, 2, 1)
        pos = sine_pos_embed_2d(W, H, C // 2, cfg["temperatureW"])
        p = f"{E}encoder.{i}.layers.0"
        q = src + pos
        Wi, bi = P[p + ".self_attn.in_proj_weight"], P[p + ".self_attn.in_proj_bias"]
        nh = cfg["nhead"]
        dh = C // nh
        Q = F.linear(q, Wi[:C], bi[:C]).reshape(B, -1, nh, dh).transpose(1, 2)
        K = F.linear(q, Wi[C:2 * C], bi[C:2 * C]).reshape(B, -1, nh, dh).transpose(1, 2)
        V = F.linear(src, Wi[2 * C:], bi[2 * C:]).reshape(B, -1, nh, dh).transpose(1, 2)
        o = (torch.softmax((Q / math.sqrt(dh)) @ K.transpose(-1, -2), -1) @ V).transpose(1, 2).reshape(B, -1, C)
        s2 = F.linear(o, P[p + ".self_attn.out_proj.weight"], P[p + ".self_attn.out_proj.bias"])
        src = _ln(src + s2, P, p + ".norm1")
        s2 = _lin(_act(_lin(src, P, p + ".linear1"), cfg["enc_act"]), P, p + ".linear2")
        src = _ln(src + s2, P, p + ".norm2")
        proj[ei] = tap(p, src.permute(0, 2, 1).reshape(B, C, H, W))
    inner = [proj[-1]]
    for idx in range(nlev - 1, 0, -1):
        j = nlev - 1 - idx
        high = _conv_norm_tap(inner[0], P, f"{E}lateral_convs.{j}", stats, act=cfg["act"])
        inner[0] = high
        up = F.interpolate(high, scale_factor=2.0, mode="nearest")
        inner.insert(0, _elan_t(torch.cat([up, proj[idx - 1]], 1), P, f"{E}fpn_blocks.{j}", stats, nblk))
    outs = [inner[0]]
    for idx in range(nlev - 1):
        d = _conv_norm_tap(outs[-1], P, f"{E}downsample_convs.{idx}.0.cv1", stats)
        d = _conv_norm_tap(d, P, f"{E}downsample_convs.{idx}.0.cv2", stats, stride=2, groups=d.shape[1])
        outs.append(_elan_t(torch.cat([d, inner[idx + 1]], 1), P, f"{E}pan_blocks.{idx}", stats, nblk))
    return outs
