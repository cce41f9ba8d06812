"""ORACLE — TEST INFRASTRUCTURE ONLY.

CPU fp32 restatement of the reference DETRPose inference forward (eval mode,
targets=None), written from the reference's math, driven by a state_dict in the
reference's key layout. It exists to CHECK the HIP path (tests/, smoke()) and to be
timed as the CPU baseline in bench.py (`cpu_baseline.kind = "port"`). The product
path (detrpose_amd) never imports it.

Pinned against the reference: tests/test_oracle_golden.py compares it with the
golden fixtures that tests/golden/make_golden.py produced by running the reference
itself (read-only at /root/reference) in the build container.

Every function cites the reference lines it restates. Conventions kept on purpose:
  * the backbone BN is FrozenBatchNorm2d x*scale+bias (hgnetv2.py:53-61), applied
    after the conv, not folded;
  * the decoder's `with_pos_embed` adds the query pos IN PLACE
    (transformer.py:360-370), so residuals carry pos;
  * bilinear sampling follows F.grid_sample(bilinear, zeros, align_corners=False)
    at grid = 2*loc-1, written as an explicit 4-corner gather.
"""
from __future__ import annotations

import math

import torch
import torch.nn.functional as F

# ----------------------------------------------------------------------------- helpers

# Test hook (tests/test_gpu_full_train_step_l.py, "teacher forcing"): when set, TAP(name, y) is
# applied to every stored layer output of the backbone / training encoder (name = the layer's
# reference prefix) and returns the tensor to continue with. The forced-state check returns
# y + (gpu_value - y).detach(): the GPU run's stored forward value, with y's gradient path.
TAP = None


def tap(name, y):
    return y if TAP is None else TAP(name, y)



def _bn_eval(x, sd, p, eps=1e-5):
    """nn.BatchNorm2d in eval == (x-mean)/sqrt(var+eps)*w+b (NCHW)."""
    w, b, rm, rv = (sd[p + s] for s in (".weight", ".bias", ".running_mean", ".running_var"))
    scale = w / torch.sqrt(rv + eps)
    return x * scale[None, :, None, None] + (b - rm * scale)[None, :, None, None]


def _frozen_bn(x, sd, p, eps=1e-5):
    """FrozenBatchNorm2d.forward, hgnetv2.py:53-61."""
    w, b, rm, rv = (sd[p + s] for s in (".weight", ".bias", ".running_mean", ".running_var"))
    scale = w * (rv + eps).rsqrt()
    bias = b - rm * scale
    return x * scale.reshape(1, -1, 1, 1) + bias.reshape(1, -1, 1, 1)


def _act(x, name):
    if name is None:
        return x
    return {"relu": F.relu, "silu": F.silu, "gelu": F.gelu}[name](x)


def bilinear_gather(value, loc):
    """F.grid_sample(value, 2*loc-1, bilinear, zeros, align_corners=False) restated.

    value: (N, H, W, C) channels-last; loc: (N, Q, 2) as (x, y) in [0,1].
    returns (N, Q, C).  Pixel coordinate = loc*size - 0.5; out-of-range corners read 0.
    """
    N, H, W, C = value.shape
    x = loc[..., 0] * W - 0.5
    y = loc[..., 1] * H - 0.5
    x0 = torch.floor(x)
    y0 = torch.floor(y)
    fx = x - x0
    fy = y - y0
    x0 = x0.long()
    y0 = y0.long()
    flat = value.reshape(N, H * W, C)
    out = torch.zeros(N, loc.shape[1], C, dtype=value.dtype)
    for dy, dx, w in ((0, 0, (1 - fx) * (1 - fy)), (0, 1, fx * (1 - fy)),
                      (1, 0, (1 - fx) * fy), (1, 1, fx * fy)):
        xi = x0 + dx
        yi = y0 + dy
        ok = (xi >= 0) & (xi < W) & (yi >= 0) & (yi < H)
        idx = (yi.clamp(0, H - 1) * W + xi.clamp(0, W - 1))
        g = torch.gather(flat, 1, idx.unsqueeze(-1).expand(-1, -1, C))
        out = out + g * (w * ok.to(value.dtype)).unsqueeze(-1)
    return out


def msda_core(value, spatial_shapes, loc, attn):
    """ms_deform_attn_core_pytorch (ms_deform_attn.py:145-193), default branch.

    value: (N, S, nH*Dh) encoder memory (levels concatenated, head-major channels)
    loc:   (N, Lq, nH, L, P, 2) in [0,1];  attn: (N, Lq, nH, L, P) (already softmaxed)
    returns (N, Lq, nH*Dh)
    """
    N, S, C = value.shape
    _, Lq, nH, L, P, _ = loc.shape
    Dh = C // nH
    out = torch.zeros(N, Lq, nH, Dh, dtype=value.dtype)
    start = 0
    for l, (h, w) in enumerate(spatial_shapes):
        v = value[:, start:start + h * w].reshape(N, h, w, nH, Dh)
        start += h * w
        # fold heads into the batch: (N*nH, h, w, Dh)
        v = v.permute(0, 3, 1, 2, 4).reshape(N * nH, h, w, Dh)
        lq = loc[:, :, :, l].permute(0, 2, 1, 3, 4).reshape(N * nH, Lq * P, 2)
        s = bilinear_gather(v, lq).reshape(N, nH, Lq, P, Dh)
        a = attn[:, :, :, l].permute(0, 2, 1, 3)  # (N, nH, Lq, P)
        out += (s * a.unsqueeze(-1)).sum(3).permute(0, 2, 1, 3)
    return out.reshape(N, Lq, C)


def _linear(x, sd, p):
    return F.linear(x, sd[p + ".weight"], sd.get(p + ".bias"))


def _mlp(x, sd, p, num_layers):
    """utils.py:75-87: ReLU between layers, none after the last."""
    for i in range(num_layers):
        x = _linear(x, sd, f"{p}.layers.{i}")
        if i < num_layers - 1:
            x = F.relu(x)
    return x


def _layer_norm(x, sd, p, eps=1e-5):
    return F.layer_norm(x, (x.shape[-1],), sd[p + ".weight"], sd[p + ".bias"], eps)


def _mha(q, k, v, sd, p, nhead):
    """nn.MultiheadAttention(batch_first=True), eval, no mask: packed in_proj then
    per-head softmax(QK^T/sqrt(dh))V and out_proj."""
    W = sd[p + ".in_proj_weight"]
    b = sd[p + ".in_proj_bias"]
    C = q.shape[-1]
    Q = F.linear(q, W[:C], b[:C])
    K = F.linear(k, W[C:2 * C], b[C:2 * C])
    V = F.linear(v, W[2 * C:], b[2 * C:])
    B, L, _ = Q.shape
    dh = C // nhead
    Q = Q.reshape(B, L, nhead, dh).transpose(1, 2)
    K = K.reshape(B, -1, nhead, dh).transpose(1, 2)
    V = V.reshape(B, -1, nhead, dh).transpose(1, 2)
    a = torch.softmax((Q / math.sqrt(dh)) @ K.transpose(-1, -2), dim=-1)
    o = (a @ V).transpose(1, 2).reshape(B, L, C)
    return F.linear(o, sd[p + ".out_proj.weight"], sd[p + ".out_proj.bias"])


# ----------------------------------------------------------------------------- backbone

# HGNetv2.arch_configs, hgnetv2.py:398-476 (stem channels, per-stage
# [in, mid, out, blocks, downsample, light, kernel, layers])
ARCH = {
    "B0": ([3, 16, 16], [[16, 16, 64, 1, False, False, 3, 3], [64, 32, 256, 1, True, False, 3, 3],
                         [256, 64, 512, 2, True, True, 5, 3], [512, 128, 1024, 1, True, True, 5, 3]]),
    "B4": ([3, 32, 48], [[48, 48, 128, 1, False, False, 3, 6], [128, 96, 512, 1, True, False, 3, 6],
                         [512, 192, 1024, 3, True, True, 5, 6], [1024, 384, 2048, 1, True, True, 5, 6]]),
    "B5": ([3, 32, 64], [[64, 64, 128, 1, False, False, 3, 6], [128, 128, 512, 2, True, False, 3, 6],
                         [512, 256, 1024, 5, True, True, 5, 6], [1024, 512, 2048, 2, True, True, 5, 6]]),
}


def conv_bn_act(x, sd, p, stride=1, groups=1, act=True, lab=False, same_pad=False):
    """ConvBNAct.forward, hgnetv2.py:82-134: conv (no bias, pad (k-1)//2) ->
    FrozenBN -> ReLU -> LearnableAffineBlock (scale*x+bias) when act and lab."""
    w = sd[p + ".conv.weight"]
    k = w.shape[-1]
    x = F.conv2d(x, w, None, stride, (k - 1) // 2, 1, groups)
    x = _frozen_bn(x, sd, p + ".bn")
    if act:
        x = F.relu(x)
        if lab:
            x = sd[p + ".lab.scale"] * x + sd[p + ".lab.bias"]
    return x


def backbone(x, sd, name, return_idx, use_lab):
    """HGNetv2.forward, hgnetv2.py:586-593 with StemBlock 210-220, HG_Stage 380-383,
    HG_Block 319-329 (agg='se': squeeze 1x1 -> excitation 1x1), LightConvBNAct 163-166."""
    stem_ch, stages = ARCH[name]
    p = "backbone.stem"
    x = tap(p + ".stem1", conv_bn_act(x, sd, p + ".stem1", stride=2, lab=use_lab))
    x = F.pad(x, (0, 1, 0, 1))
    x2 = tap(p + ".stem2a", conv_bn_act(x, sd, p + ".stem2a", lab=use_lab))
    x2 = F.pad(x2, (0, 1, 0, 1))
    x2 = tap(p + ".stem2b", conv_bn_act(x2, sd, p + ".stem2b", lab=use_lab))
    x1 = F.max_pool2d(x, 2, 1, ceil_mode=True)
    x = torch.cat([x1, x2], 1)
    x = tap(p + ".stem3", conv_bn_act(x, sd, p + ".stem3", stride=2, lab=use_lab))
    x = tap(p + ".stem4", conv_bn_act(x, sd, p + ".stem4", lab=use_lab))
    outs = []
    for si, (cin, mid, cout, nblk, down, light, k, nlayer) in enumerate(stages):
        sp = f"backbone.stages.{si}"
        if down:
            x = tap(sp + ".downsample",
                    conv_bn_act(x, sd, sp + ".downsample", stride=2, groups=cin, act=False, lab=use_lab))
        for bi in range(nblk):
            bp = f"{sp}.blocks.{bi}"
            identity = x
            feats = [x]
            for li in range(nlayer):
                lp = f"{bp}.layers.{li}"
                if light:
                    x = tap(lp + ".conv1", conv_bn_act(x, sd, lp + ".conv1", act=False, lab=use_lab))
                    x = tap(lp + ".conv2", conv_bn_act(x, sd, lp + ".conv2", groups=x.shape[1], lab=use_lab))
                else:
                    x = tap(lp, conv_bn_act(x, sd, lp, lab=use_lab))
                feats.append(x)
            x = torch.cat(feats, 1)
            x = tap(bp + ".aggregation.0", conv_bn_act(x, sd, bp + ".aggregation.0", lab=use_lab))
            x = conv_bn_act(x, sd, bp + ".aggregation.1", lab=use_lab)
            if bi > 0:
                x = x + identity
            x = tap(bp + ".aggregation.1", x)
        if si in return_idx:
            outs.append(x)
    return outs


# ----------------------------------------------------------------------------- encoder


def _conv_norm(x, sd, p, stride=1, groups=1, act=None):
    """ConvNormLayer / ConvNormLayer_fuse (non-deploy form), hybrid_encoder.py:56-128."""
    w = sd[p + ".conv.weight"]
    k = w.shape[-1]
    x = F.conv2d(x, w, sd.get(p + ".conv.bias"), stride, (k - 1) // 2, 1, groups)
    return _act(_bn_eval(x, sd, p + ".norm"), act)


def _vgg(x, sd, p, act):
    """VGGBlock.forward (non-deploy), hybrid_encoder.py:139-154."""
    return _act(_conv_norm(x, sd, p + ".conv1") + _conv_norm(x, sd, p + ".conv2"), act)


def _csp(x, sd, p, nblk, act):
    """CSPLayer.forward, hybrid_encoder.py:215-240 (conv3 is Identity: hidden == out)."""
    x1 = _conv_norm(x, sd, p + ".conv1", act=act)
    for i in range(nblk):
        x1 = _vgg(x1, sd, f"{p}.bottlenecks.{i}", act)
    x2 = _conv_norm(x, sd, p + ".conv2", act=act)
    return x1 + x2


def _elan(x, sd, p, nblk, act="silu"):
    """RepNCSPELAN4.forward, hybrid_encoder.py:192-212."""
    y = _conv_norm(x, sd, p + ".cv1", act=act)
    c = y.shape[1] // 2
    ys = [y[:, :c], y[:, c:]]
    z = _csp(ys[-1], sd, p + ".cv2.0", nblk, act)
    ys.append(_conv_norm(z, sd, p + ".cv2.1", act=act))
    z = _csp(ys[-1], sd, p + ".cv3.0", nblk, act)
    ys.append(_conv_norm(z, sd, p + ".cv3.1", act=act))
    return _conv_norm(torch.cat(ys, 1), sd, p + ".cv4", act=act)


def sine_pos_embed_2d(w, h, dim, temperature):
    """HybridEncoder.create_sinehw_position_embedding, hybrid_encoder.py:431-460."""
    gw = torch.arange(1, w + 1, dtype=torch.float32)
    gh = torch.arange(1, h + 1, dtype=torch.float32)
    gh, gw = torch.meshgrid(gh, gw, indexing="ij")
    eps = 1e-6
    gw = gw / (w + eps) * (2 * math.pi)
    gh = gh / (h + eps) * (2 * math.pi)
    d = torch.arange(dim, dtype=torch.float32)
    d = temperature ** (2 * torch.div(d, 2, rounding_mode="floor") / dim)
    px = gw[..., None] / d
    py = gh[..., None] / d
    px = torch.stack((px[..., 0::2].sin(), px[..., 1::2].cos()), 3).flatten(2)
    py = torch.stack((py[..., 0::2].sin(), py[..., 1::2].cos()), 3).flatten(2)
    return torch.cat((py, px), 2).reshape(1, h * w, 2 * dim)


def encoder(feats, sd, cfg):
    """HybridEncoder.forward, hybrid_encoder.py:462-507."""
    C = cfg["hidden_dim"]
    nlev = cfg["n_levels"]
    nblk = round(3 * cfg["depth_mult"])
    enc_idx = cfg.get("use_encoder_idx", [2])
    proj = [_bn_eval(F.conv2d(f, sd[f"encoder.input_proj.{i}.conv.weight"]), sd, f"encoder.input_proj.{i}.norm")
            for i, f in enumerate(feats)]
    for i, ei in enumerate(enc_idx):
        B, _, H, W = proj[ei].shape
        src = proj[ei].flatten(2).permute(0, 2, 1)
        pos = sine_pos_embed_2d(W, H, C // 2, cfg["temperatureW"])
        p = f"encoder.encoder.{i}.layers.0"
        # TransformerEncoderLayer.forward (post-norm), hybrid_encoder.py:270-296
        q = src + pos
        s2 = _mha(q, q, src, sd, p + ".self_attn", cfg["nhead"])
        src = _layer_norm(src + s2, sd, p + ".norm1")
        s2 = _linear(_act(_linear(src, sd, p + ".linear1"), cfg["enc_act"]), sd, p + ".linear2")
        src = _layer_norm(src + s2, sd, p + ".norm2")
        proj[ei] = src.permute(0, 2, 1).reshape(B, C, H, W)
    inner = [proj[-1]]
    for idx in range(nlev - 1, 0, -1):
        j = nlev - 1 - idx
        high = _conv_norm(inner[0], sd, f"encoder.lateral_convs.{j}", act=cfg["act"])
        inner[0] = high
        up = F.interpolate(high, scale_factor=2.0, mode="nearest")
        inner.insert(0, _elan(torch.cat([up, proj[idx - 1]], 1), sd, f"encoder.fpn_blocks.{j}", nblk))
    outs = [inner[0]]
    for idx in range(nlev - 1):
        d = _conv_norm(outs[-1], sd, f"encoder.downsample_convs.{idx}.0.cv1")
        d = _conv_norm(d, sd, f"encoder.downsample_convs.{idx}.0.cv2", stride=2, groups=d.shape[1])
        outs.append(_elan(torch.cat([d, inner[idx + 1]], 1), sd, f"encoder.pan_blocks.{idx}", nblk))
    return outs


# ----------------------------------------------------------------------------- transformer


def weighting_function(reg_max, up, reg_scale):
    """transformer.py:152-195 (values identical in deploy and train forms)."""
    ub1 = abs(up) * abs(reg_scale)
    ub2 = ub1 * 2
    step = (ub1 + 1) ** (2 / (reg_max - 2))
    left = [-(step ** i) + 1 for i in range(reg_max // 2 - 1, 0, -1)]
    right = [step ** i - 1 for i in range(1, reg_max // 2)]
    return torch.tensor([-ub2] + left + [0.0] + right + [ub2], dtype=torch.float32)


def anchors_and_mask(feat_strides, size=(640, 640)):
    """Transformer._generate_anchors, transformer.py:1179-1200: logit anchors and the
    INVALID mask (the buffer named valid_mask stores ~valid)."""
    anchors = []
    for s in feat_strides:
        h, w = int(size[0] / s), int(size[1] / s)
        gy, gx = torch.meshgrid(torch.linspace(0, h - 1, h), torch.linspace(0, w - 1, w), indexing="ij")
        g = (torch.stack([gx, gy], -1) + 0.5) / torch.tensor([w, h], dtype=torch.float32)
        anchors.append(g.reshape(1, -1, 2))
    a = torch.cat(anchors, 1)
    valid = ((a > 0.01) & (a < 0.99)).all(-1, keepdim=True)
    return torch.log(a / (1 - a)), ~valid


def sine_embedding(pos, dim_t):
    """TransformerDecoder.sine_embedding for 2-D points, transformer.py:518-540."""
    scale = 2 * math.pi
    px = pos[..., 0:1] * scale / dim_t
    py = pos[..., 1:2] * scale / dim_t
    px = torch.stack((px[..., 0::2].sin(), px[..., 1::2].cos()), dim=4).flatten(3)
    py = torch.stack((py[..., 0::2].sin(), py[..., 1::2].cos()), dim=4).flatten(3)
    return torch.cat((py, px), dim=3)


def inverse_sigmoid(x, eps=1e-3):
    """utils.py:133-137."""
    x = x.clamp(0, 1)
    return torch.log(x.clamp(min=eps) / (1 - x).clamp(min=eps))


def decoder_layer(tgt, pos, ref, memory, shapes, sd, p, nhead, n_levels, n_points):
    """DeformableTransformerDecoderLayer.forward, transformer.py:387-442 (default path).
    tgt: (B, Q, 1+K, C); pos: (B, Q, K, C); ref: (B, Q, 1+K, 2)."""
    B, Q, T, C = tgt.shape
    tgt = tgt.clone()
    # in-place with_pos_embed (transformer.py:360-370): q = k = v = residual = tgt+pos
    tgt[:, :, 1:] += pos
    x = tgt.flatten(0, 1)
    t2 = _mha(x, x, x, sd, p + ".within_attn", nhead).reshape(B, Q, T, C)
    tgt = _layer_norm(tgt + t2, sd, p + ".within_norm")
    x = tgt.transpose(1, 2).flatten(0, 1)  # (B*T, Q, C)
    t2 = _mha(x, x, x, sd, p + ".across_attn", nhead)
    tgt = _layer_norm(x + t2, sd, p + ".across_norm").reshape(B, T, Q, C).transpose(1, 2)
    tgt = tgt.clone()
    tgt[:, :, 1:] += pos  # second in-place add (transformer.py:422)
    # MSDeformAttn.forward default branch, ms_deform_attn.py:384-444
    query = tgt.flatten(1, 2)  # (B, Q*T, C)
    Lq = Q * T
    off = _linear(query, sd, p + ".cross_attn.sampling_offsets").reshape(B, Lq, nhead, n_levels, n_points, 2)
    aw = _linear(query, sd, p + ".cross_attn.attention_weights").reshape(B, Lq, nhead, n_levels * n_points)
    aw = torch.softmax(aw, -1).reshape(B, Lq, nhead, n_levels, n_points)
    norm = torch.tensor([[w, h] for h, w in shapes], dtype=torch.float32).reshape(1, 1, 1, n_levels, 1, 2)
    r = ref.reshape(B, Lq, 1, 1, 1, 2)
    loc = r + off / norm
    x2 = msda_core(memory, shapes, loc, aw).reshape(B, Q, T, C)
    # Gate, transformer.py:222-235
    g = torch.sigmoid(_linear(torch.cat([tgt, x2], -1), sd, p + ".gateway.gate"))
    g1, g2 = g.chunk(2, -1)
    tgt = _layer_norm(g1 * tgt + g2 * x2, sd, p + ".gateway.norm")
    # FFN, transformer.py:371-385 (activation relu)
    t2 = _linear(F.relu(_linear(tgt, sd, p + ".linear1")), sd, p + ".linear2")
    return _layer_norm(tgt + t2, sd, p + ".norm2")


def lqe(scores, kps, feat_nhwc, sd, p, k=4):
    """LQE.forward, transformer.py:275-288: sample feats[0] at the keypoints, top-k
    over channels + their mean -> MLP -> added to the class logits."""
    B, Q, K, _ = kps.shape
    s = bilinear_gather(feat_nhwc, kps.reshape(B, Q * K, 2)).reshape(B, Q, K, -1)
    top = s.topk(k, dim=-1)[0]
    stat = torch.cat([top, top.mean(-1, keepdim=True)], -1).reshape(B, Q, -1)
    return scores + _mlp(stat, sd, p + ".reg_conf", 2)


def transformer(feats, sd, cfg, force_topk=None):
    """Transformer.forward (eval, deploy), transformer.py:1209-1387, and
    TransformerDecoder.forward, transformer.py:558-925 (default path).

    force_topk (B, nq) int64, test-side only: replaces the two-stage selection's
    topk indices (transformer.py:1240-1242) so a reduced-precision forward, whose
    near-tied scores may select a different query set, can be compared with this
    fp32 restatement query by query on the SAME selection."""
    C = cfg["hidden_dim"]
    nhead = cfg["nhead"]
    nq = cfg["num_queries"]
    K = cfg["num_body_points"]
    nlayers = cfg["num_decoder_layers"]
    reg_scale = float(cfg["reg_scale"])
    reg_max = cfg["reg_max"]
    B = feats[0].shape[0]
    shapes = [(f.shape[2], f.shape[3]) for f in feats]
    memory = torch.cat([f.flatten(2).permute(0, 2, 1) for f in feats], 1)  # (B, S, C)
    anchors, invalid = anchors_and_mask(cfg["feat_strides"], cfg["eval_spatial_size"])
    om = memory.masked_fill(invalid, 0.0)
    om = _layer_norm(_linear(om, sd, "transformer.enc_output"), sd, "transformer.enc_output_norm")
    cls = _linear(om, sd, "transformer.enc_out_class_embed")
    topk_idx = torch.topk(cls.max(-1)[0], nq, dim=1)[1]
    if force_topk is not None:
        topk_idx = torch.as_tensor(force_topk, dtype=torch.int64).reshape(B, nq)
    tmem = torch.gather(om, 1, topk_idx.unsqueeze(-1).expand(-1, -1, C))
    tanc = torch.gather(anchors.expand(B, -1, -1), 1, topk_idx.unsqueeze(-1).expand(-1, -1, 2))
    delta = _mlp(tmem, sd, "transformer.enc_pose_embed", 4).reshape(B, nq, K, 2)
    kp = torch.sigmoid(delta + tanc.unsqueeze(-2))
    ref = torch.cat([kp.mean(2, keepdim=True), kp], 2)  # (B, Q, 1+K, 2)
    # query construction, transformer.py:1253-1261
    tgt_kp = sd["transformer.keypoint_embedding.weight"][None, None] + sd["transformer.tgt_embed.weight"][None, :, None]
    tgt_inst = sd["transformer.instance_embedding.weight"][None, None].expand(1, nq, 1, C)
    tgt = torch.cat([tgt_inst, tgt_kp], 2).expand(B, -1, -1, -1)
    project = weighting_function(reg_max, 0.5, reg_scale)
    dim_t = sd.get("transformer.decoder.dim_t")
    if dim_t is None:
        d = torch.arange(C // 2, dtype=torch.float32)
        dim_t = 10000 ** (2 * torch.div(d, 2, rounding_mode="floor") / (C // 2))
    out = tgt
    prev_pose = 0
    prev_corners = 0
    res = {"topk_idx": topk_idx, "layers": [], "corners": []}
    for l in range(nlayers):
        ref_kp = ref[:, :, 1:]
        pos = _mlp(sine_embedding(ref_kp, dim_t), sd, "transformer.decoder.half_pose_ref_point_head", 2)
        if l > 0:
            # Aliasing quirk: output_pose_detach is a VIEW of the previous layer's
            # output (transformer.py:716,922), and this layer's in-place
            # with_pos_embed (transformer.py:369, on that same tensor) adds pos to it.
            prev_pose = prev_pose + pos
        out = decoder_layer(out, pos, ref, memory, shapes, sd, f"transformer.decoder.layers.{l}",
                            nhead, cfg["num_feature_levels"], cfg["dec_n_points"])
        res["layers"].append(out)
        pose = out[:, :, 1:]
        inst = out[:, :, 0]
        if l == 0:
            pre = torch.sigmoid(_mlp(pose, sd, "transformer.pre_pose_embed", 3) + inverse_sigmoid(ref_kp))
            ref_init = pre
        corners = _mlp(pose + prev_pose, sd, f"transformer.pose_embed.{l}", 3) + prev_corners
        res["corners"].append(corners)
        # Integral (transformer.py:253-260) + distance2pose (198-219)
        prob = torch.softmax(corners.reshape(-1, reg_max + 1), 1)
        d = F.linear(prob, project[None]).reshape(B, nq, K, 2)
        kps = ref_init + d / abs(reg_scale)
        ref = torch.cat([kps.mean(2, keepdim=True), kps], 2)
        if l == nlayers - 1:
            score = _linear(inst, sd, f"transformer.class_embed.{l}")
            logit = lqe(score, kps, feats[0].permute(0, 2, 3, 1), sd, f"transformer.lqe_embed.{l}")
            res.update(pred_logits=logit, pred_keypoints=kps)
        prev_corners = corners
        prev_pose = pose
    return res


# ----------------------------------------------------------------------------- top level


class OracleDETRPose:
    """CPU fp32 DETRPose eval forward from a reference-layout state_dict."""

    def __init__(self, cfg: dict, state_dict: dict):
        self.cfg = cfg
        self.sd = {k: v.detach().to("cpu", torch.float32) for k, v in state_dict.items()}

    @torch.no_grad()
    def forward(self, images: torch.Tensor, intermediates: bool = False, force_topk=None):
        bcfg, ecfg, tcfg = self.cfg["backbone"], self.cfg["encoder"], self.cfg["transformer"]
        x = images.to(torch.float32)
        bb = backbone(x, self.sd, bcfg["name"], bcfg["return_idx"], bcfg["use_lab"])
        en = encoder(bb, self.sd, ecfg)
        tr = transformer(en, self.sd, tcfg, force_topk=force_topk)
        out = {"pred_logits": tr["pred_logits"], "pred_keypoints": tr["pred_keypoints"]}
        if intermediates:
            out.update(backbone=bb, encoder=en, topk_idx=tr["topk_idx"], layers=tr["layers"], corners=tr["corners"])
        return out

    __call__ = forward


@torch.no_grad()
def postprocess(pred_logits, pred_keypoints, target_sizes, num_select=60):
    """PostProcess.forward deploy branch (postprocesses.py:15-30), for any batch:
    sigmoid -> topk over (query x class) -> gather keypoints -> scale by [w, h]."""
    B, Q, NC = pred_logits.shape
    prob = pred_logits.sigmoid().reshape(B, -1)
    scores, idx = torch.topk(prob, num_select, dim=1)
    q = torch.div(idx, NC, rounding_mode="floor")
    labels = idx % NC
    K = pred_keypoints.shape[2]
    kp = torch.gather(pred_keypoints, 1, q[..., None, None].expand(B, num_select, K, 2))
    return scores, labels, kp * target_sizes[:, None, None, :]
