"""Transformer (two-stage query selection + pose decoder): constructor and parameter
layout of src/models/detrpose/transformer.py and ms_deform_attn.py.

Parameter containers with the reference's names; the forward is planned over HIP
kernels by detrpose_amd.engine. The experimental branches of the reference (energy
refinement, KAN FFN, grid attention, modulation, region sampling, global context,
grouped offsets; SURVEY.md §2 "OUT OF SCOPE") are accepted as constructor kwargs
only when disabled, exactly like the N/L/X configs use them.
"""
from __future__ import annotations

import math

import torch
from torch import nn


class MLP(nn.Module):
    """utils.py:75-87 (ReLU between layers)."""

    def __init__(self, input_dim, hidden_dim, output_dim, num_layers):
        super().__init__()
        self.num_layers = num_layers
        h = [hidden_dim] * (num_layers - 1)
        self.layers = nn.ModuleList(nn.Linear(n, k) for n, k in zip([input_dim] + h, h + [output_dim]))


class MSDeformAttn(nn.Module):
    """ms_deform_attn.py:196-513, default (local) branch: no value/output projection."""

    def __init__(self, d_model=256, n_levels=4, n_heads=8, n_points=4, use_4D_normalizer=False, **flags):
        super().__init__()
        for k, v in flags.items():
            if k in ("use_grid_fusion", "grid_num_points", "region_kernel_size", "num_groups"):
                continue
            if v:
                raise NotImplementedError(f"MSDeformAttn({k}={v}) is an experimental branch outside the hot path")
        if d_model % n_heads:
            raise ValueError(f"d_model must be divisible by n_heads, got {d_model} and {n_heads}")
        self.d_model, self.n_levels, self.n_heads, self.n_points = d_model, n_levels, n_heads, n_points
        self.sampling_offsets = nn.Linear(d_model, n_heads * n_levels * n_points * 2)
        self.attention_weights = nn.Linear(d_model, n_heads * n_levels * n_points)

    def forward(self, query, reference_points, value, input_spatial_shapes):
        """ms_deform_attn.py:359-444 (default branch), differentiable: the two Linear layers
        (torch), then one fused HIP op for softmax + sampling locations + bilinear gather +
        weighted sum (dp_msda; backward dp_msda_bwd). query (N, Lq, C); reference_points with
        one 2-D point per query, shaped as the decoder passes it ((N, Q, 1, T, 2), transposed
        and flattened to (N, Lq, 1, 2) as at :412); value: the reference's per-level list
        [(N*nH, Dh, H*W)] or the encoder memory (N, S, C)."""
        from .msda import msdeform_attn, value_from_levels
        N, Lq, _ = query.shape
        ref = torch.transpose(reference_points, 2, 3).flatten(1, 2) if reference_points.dim() == 5 else reference_points
        if ref.shape[-1] != 2 or ref.shape[1] != Lq:
            raise ValueError(f"reference_points {tuple(reference_points.shape)}: one 2-D point per query expected")
        if ref.dim() == 4:
            if ref.shape[2] != 1:
                raise NotImplementedError("per-level reference points (n_levels > 1 in dim 2) are not used by DETRPose")
            ref = ref[:, :, 0]
        if isinstance(value, (list, tuple)):
            value = value_from_levels(value, self.n_heads)
        oa = torch.cat([self.sampling_offsets(query), self.attention_weights(query)], -1)
        return msdeform_attn(value, [tuple(int(v) for v in hw) for hw in input_spatial_shapes],
                             oa.reshape(N * Lq, -1), ref.reshape(N * Lq, 2), self.n_heads, self.n_points)


class Gate(nn.Module):
    """transformer.py:222-235."""

    def __init__(self, d_model):
        super().__init__()
        self.gate = nn.Linear(2 * d_model, 2 * d_model)
        self.norm = nn.LayerNorm(d_model)


class LQE(nn.Module):
    """transformer.py:263-288."""

    def __init__(self, topk, hidden_dim, num_layers, num_body_points):
        super().__init__()
        self.k = topk
        self.hidden_dim = hidden_dim
        self.reg_conf = MLP(num_body_points * (topk + 1), hidden_dim, 1, num_layers)
        self.num_body_points = num_body_points


class DeformableTransformerDecoderLayer(nn.Module):
    """transformer.py:291-442 (default path: MHA within/across, MSDA, Gate, ReLU FFN)."""

    def __init__(self, d_model=256, d_ffn=1024, dropout=0.1, activation="relu", n_levels=4, n_heads=8, n_points=4,
                 use_kan=False, kan_grid=3, **flags):
        super().__init__()
        if use_kan:
            raise NotImplementedError("use_kan=True (FastKAN FFN) is an experimental branch outside the hot path")
        if activation != "relu":
            raise NotImplementedError("decoder activation must be relu (configs use relu)")
        msda_flags = {k: v for k, v in flags.items() if k not in ("is_energy", "energy_in_dim", "energy_out_dim",
                                                                  "normalize_energy")}
        if flags.get("is_energy"):
            raise NotImplementedError("energy layers are outside the hot path")
        self.within_attn = nn.MultiheadAttention(d_model, n_heads, dropout=dropout, batch_first=True)
        self.within_norm = nn.LayerNorm(d_model)
        self.across_attn = nn.MultiheadAttention(d_model, n_heads, dropout=dropout, batch_first=True)
        self.across_norm = nn.LayerNorm(d_model)
        self.cross_attn = MSDeformAttn(d_model, n_levels, n_heads, n_points, **msda_flags)
        self.gateway = Gate(d_model)
        self.linear1 = nn.Linear(d_model, d_ffn)
        self.linear2 = nn.Linear(d_ffn, d_model)
        self.norm2 = nn.LayerNorm(d_model)


class TransformerDecoder(nn.Module):
    """transformer.py:446-925 (eval path)."""

    def __init__(self, decoder_layer_kwargs, num_layers, hidden_dim=256, num_body_points=17):
        super().__init__()
        self.layers = nn.ModuleList([DeformableTransformerDecoderLayer(**decoder_layer_kwargs)
                                     for _ in range(num_layers)])
        self.hidden_dim = hidden_dim
        self.num_layers = num_layers
        self.num_body_points = num_body_points
        self.half_pose_ref_point_head = MLP(hidden_dim, hidden_dim, hidden_dim, 2)
        self.eval_idx = num_layers - 1
        d = torch.arange(hidden_dim // 2, dtype=torch.float32)
        self.register_buffer("dim_t", 10000 ** (2 * torch.div(d, 2, rounding_mode="floor") / (hidden_dim // 2)))


def generate_anchors(feat_strides, eval_spatial_size):
    """Transformer._generate_anchors (transformer.py:1179-1200): logit anchors (1,S,2) and
    the INVALID mask (1,S,1) (the reference names the buffer valid_mask)."""
    anchors = []
    eh, ew = eval_spatial_size
    for s in feat_strides:
        h, w = int(eh / s), int(ew / s)
        gy, gx = torch.meshgrid(torch.linspace(0, h - 1, h), torch.linspace(0, w - 1, w), indexing="ij")
        grid = (torch.stack([gx, gy], -1)[None] + 0.5) / torch.tensor([w, h], dtype=torch.float32)
        anchors.append(grid.reshape(1, -1, 2))
    a = torch.cat(anchors, 1)
    valid = ((a > 0.01) & (a < 0.99)).all(-1, keepdim=True)
    return torch.log(a / (1 - a)), ~valid


def weighting_function(reg_max, up, reg_scale):
    """transformer.py:152-195 (deploy form): the 33-bin projection W(n)."""
    ub1 = abs(float(up)) * abs(float(reg_scale))
    ub2 = ub1 * 2
    step = (ub1 + 1) ** (2 / (reg_max - 2))
    left = [-(step ** i) + 1 for i in range(reg_max // 2 - 1, 0, -1)]
    right = [step ** i - 1 for i in range(1, reg_max // 2)]
    return torch.tensor([-ub2] + left + [0.0] + right + [ub2], dtype=torch.float32)


class Transformer(nn.Module):
    """transformer.py:929-1419 (constructor kwargs identical; experimental ones must be off)."""

    def __init__(self, hidden_dim=256, nhead=8, num_queries=300, num_decoder_layers=6, dim_feedforward=2048,
                 dropout=0.0, activation="relu", normalize_before=False, return_intermediate_dec=False,
                 num_feature_levels=1, enc_n_points=4, dec_n_points=4, learnable_tgt_init=False, two_stage_type="no",
                 num_classes=2, aux_loss=True, dec_pred_class_embed_share=False, dec_pred_pose_embed_share=False,
                 two_stage_class_embed_share=True, two_stage_bbox_embed_share=True, cls_no_bias=False,
                 num_body_points=17, feat_strides=None, eval_spatial_size=None, reg_max=32, reg_scale=4.0,
                 use_kan=False, kan_grid=3, **experimental):
        super().__init__()
        for k in ("use_energy_refinement", "use_intermediate_energy_refinement", "use_modulation",
                  "use_region_sampling", "use_global_context", "use_grouped_offsets", "use_grid_attention",
                  "use_grid_offsets", "train_energy_by_loss", "freeze_network"):
            if experimental.get(k):
                raise NotImplementedError(f"Transformer({k}=True) is outside the DETRPose hot path")
        if two_stage_type != "standard":
            raise NotImplementedError("only two_stage_type='standard' is used by DETRPose")
        if not learnable_tgt_init:
            raise NotImplementedError("learnable_tgt_init=False is not used by the DETRPose configs")
        if dec_pred_class_embed_share or dec_pred_pose_embed_share or two_stage_class_embed_share or \
                two_stage_bbox_embed_share or cls_no_bias:
            raise NotImplementedError("shared / bias-free heads are not used by the DETRPose configs")
        self.hidden_dim, self.nhead = hidden_dim, nhead
        self.num_queries, self.num_decoder_layers, self.dec_layers = num_queries, num_decoder_layers, num_decoder_layers
        self.num_feature_levels, self.dec_n_points = num_feature_levels, dec_n_points
        self.num_classes, self.num_body_points = num_classes, num_body_points
        self.dim_feedforward = dim_feedforward
        self.reg_max = reg_max
        self.feat_strides, self.eval_spatial_size = feat_strides, eval_spatial_size
        layer_kw = dict(d_model=hidden_dim, d_ffn=dim_feedforward, dropout=dropout, activation=activation,
                        n_levels=num_feature_levels, n_heads=nhead, n_points=dec_n_points, use_kan=use_kan,
                        kan_grid=kan_grid)
        self.decoder = TransformerDecoder(layer_kw, num_decoder_layers, hidden_dim, num_body_points)
        self.keypoint_embedding = nn.Embedding(num_body_points, hidden_dim)
        self.instance_embedding = nn.Embedding(1, hidden_dim)
        self.tgt_embed = nn.Embedding(num_queries, hidden_dim)
        self.label_enc = nn.Embedding(80 + 1, hidden_dim)          # training-only (DN), kept for key parity
        self.pose_enc = nn.Embedding(num_body_points, hidden_dim)  # training-only (DN)
        self.enc_output = nn.Linear(hidden_dim, hidden_dim)
        self.enc_output_norm = nn.LayerNorm(hidden_dim)
        self.class_embed = nn.ModuleList([nn.Linear(hidden_dim, num_classes) for _ in range(num_decoder_layers)])
        self.pose_embed = nn.ModuleList([MLP(hidden_dim, hidden_dim, 2 * (reg_max + 1), 3)
                                         for _ in range(num_decoder_layers)])
        self.lqe_embed = nn.ModuleList([LQE(4, 256, 2, num_body_points) for _ in range(num_decoder_layers)])
        self.pre_pose_embed = MLP(hidden_dim, hidden_dim, 2, 3)
        self.up = nn.Parameter(torch.tensor([1 / 2]), requires_grad=False)
        self.reg_scale = nn.Parameter(torch.tensor([float(reg_scale)]), requires_grad=False)
        self.enc_pose_embed = MLP(hidden_dim, 2 * hidden_dim, 2 * num_body_points, 4)
        self.enc_out_class_embed = nn.Linear(hidden_dim, num_classes)
        if not eval_spatial_size:
            raise NotImplementedError("eval_spatial_size is required (anchors are precomputed for inference)")
        anchors, invalid = generate_anchors(feat_strides, eval_spatial_size)
        self.register_buffer("anchors", anchors)
        self.register_buffer("valid_mask", invalid)
        prior = -math.log((1 - 0.01) / 0.01)
        for m in list(self.class_embed) + [self.enc_out_class_embed]:
            nn.init.constant_(m.bias, prior)

    def forward(self, feats, targets=None, samples=None):
        raise NotImplementedError("run the full model through DETRPose.forward (HIP engine)")
