"""HybridEncoder: constructor and parameter layout of src/models/detrpose/hybrid_encoder.py.

Parameter containers with the reference's names (non-deploy layout, which is what
checkpoints hold). The encoder forward (AIFI + CCFF FPN/PAN) is planned over HIP
kernels by detrpose_amd.engine; `deploy()`-style BN folding happens there.
"""
from __future__ import annotations

import copy
from collections import OrderedDict

from torch import nn


class ConvNormLayer_fuse(nn.Module):
    """hybrid_encoder.py:56-111 (conv + BN + act; folded at pack time)."""

    def __init__(self, ch_in, ch_out, kernel_size, stride, g=1, padding=None, bias=False, act=None):
        super().__init__()
        padding = (kernel_size - 1) // 2 if padding is None else padding
        self.conv = nn.Conv2d(ch_in, ch_out, kernel_size, stride, groups=g, padding=padding, bias=bias)
        self.norm = nn.BatchNorm2d(ch_out)
        self.act_name = act
        self.ch_in, self.ch_out, self.kernel_size, self.stride, self.g, self.padding = \
            ch_in, ch_out, kernel_size, stride, g, padding


class ConvNormLayer(nn.Module):
    """hybrid_encoder.py:114-128."""

    def __init__(self, ch_in, ch_out, kernel_size, stride, padding=None, bias=False, act=None):
        super().__init__()
        padding = (kernel_size - 1) // 2 if padding is None else padding
        self.conv = nn.Conv2d(ch_in, ch_out, kernel_size, stride, padding=padding, bias=bias)
        self.norm = nn.BatchNorm2d(ch_out)
        self.act_name = act
        self.kernel_size, self.stride = kernel_size, stride


class SCDown(nn.Module):
    """hybrid_encoder.py:130-137: 1x1 conv+BN then depthwise k x k stride s conv+BN."""

    def __init__(self, c1, c2, k, s):
        super().__init__()
        self.cv1 = ConvNormLayer_fuse(c1, c2, 1, 1)
        self.cv2 = ConvNormLayer_fuse(c2, c2, k, s, c2)


class VGGBlock(nn.Module):
    """hybrid_encoder.py:139-189: 3x3 conv+BN + 1x1 conv+BN, summed, act (RepVGG)."""

    def __init__(self, ch_in, ch_out, act="relu"):
        super().__init__()
        self.ch_in, self.ch_out = ch_in, ch_out
        self.conv1 = ConvNormLayer(ch_in, ch_out, 3, 1, padding=1, act=None)
        self.conv2 = ConvNormLayer(ch_in, ch_out, 1, 1, padding=0, act=None)
        self.act_name = act


class CSPLayer(nn.Module):
    """hybrid_encoder.py:215-240."""

    def __init__(self, in_channels, out_channels, num_blocks=3, expansion=1.0, bias=None, act="silu",
                 bottletype=VGGBlock):
        super().__init__()
        hidden = int(out_channels * expansion)
        self.conv1 = ConvNormLayer(in_channels, hidden, 1, 1, bias=bias, act=act)
        self.conv2 = ConvNormLayer(in_channels, hidden, 1, 1, bias=bias, act=act)
        self.bottlenecks = nn.Sequential(*[bottletype(hidden, hidden, act=act) for _ in range(num_blocks)])
        if hidden != out_channels:
            raise NotImplementedError("CSPLayer with conv3 (expansion != 1) is not built by HybridEncoder")
        self.conv3 = nn.Identity()
        self.num_blocks = num_blocks


class RepNCSPELAN4(nn.Module):
    """hybrid_encoder.py:192-212."""

    def __init__(self, c1, c2, c3, c4, n=3, bias=False, act="silu"):
        super().__init__()
        self.c = c3 // 2
        self.c1, self.c2, self.c3, self.c4, self.n, self.act_name = c1, c2, c3, c4, n, act
        self.cv1 = ConvNormLayer_fuse(c1, c3, 1, 1, bias=bias, act=act)
        self.cv2 = nn.Sequential(CSPLayer(c3 // 2, c4, n, 1, bias=bias, act=act, bottletype=VGGBlock),
                                 ConvNormLayer_fuse(c4, c4, 3, 1, bias=bias, act=act))
        self.cv3 = nn.Sequential(CSPLayer(c4, c4, n, 1, bias=bias, act=act, bottletype=VGGBlock),
                                 ConvNormLayer_fuse(c4, c4, 3, 1, bias=bias, act=act))
        self.cv4 = ConvNormLayer_fuse(c3 + (2 * c4), c2, 1, 1, bias=bias, act=act)


class TransformerEncoderLayer(nn.Module):
    """hybrid_encoder.py:244-296 (post-norm)."""

    def __init__(self, d_model, nhead, dim_feedforward=2048, dropout=0.1, activation="relu", normalize_before=False):
        super().__init__()
        if normalize_before:
            raise NotImplementedError("normalize_before=True is not used by DETRPose")
        self.self_attn = nn.MultiheadAttention(d_model, nhead, dropout, batch_first=True)
        self.linear1 = nn.Linear(d_model, dim_feedforward)
        self.linear2 = nn.Linear(dim_feedforward, d_model)
        self.norm1 = nn.LayerNorm(d_model)
        self.norm2 = nn.LayerNorm(d_model)
        self.activation_name = activation
        self.nhead = nhead


class TransformerEncoder(nn.Module):
    def __init__(self, encoder_layer, num_layers, norm=None):
        super().__init__()
        self.layers = nn.ModuleList([copy.deepcopy(encoder_layer) for _ in range(num_layers)])
        self.num_layers = num_layers
        if norm is not None:
            raise NotImplementedError("TransformerEncoder.norm is not used by HybridEncoder")


class HybridEncoder(nn.Module):
    """hybrid_encoder.py:324-507."""

    def __init__(self, in_channels=(512, 1024, 2048), feat_strides=(8, 16, 32), n_levels=3, hidden_dim=256, nhead=8,
                 dim_feedforward=1024, dropout=0.0, enc_act="gelu", use_encoder_idx=(2,), num_encoder_layers=1,
                 expansion=1.0, depth_mult=1.0, act="silu", eval_spatial_size=None, temperatureH=20,
                 temperatureW=20, freeze_network=False):
        super().__init__()
        self.in_channels = list(in_channels)
        self.feat_strides = list(feat_strides)
        self.n_levels = n_levels
        self.hidden_dim = hidden_dim
        self.nhead = nhead
        self.use_encoder_idx = list(use_encoder_idx)
        self.num_encoder_layers = num_encoder_layers
        self.eval_spatial_size = eval_spatial_size
        self.temperatureW, self.temperatureH = temperatureW, temperatureH
        self.enc_act = enc_act
        self.act = act
        self.c4 = round(expansion * hidden_dim // 2)
        self.n_blocks = round(3 * depth_mult)
        self.input_proj = nn.ModuleList([
            nn.Sequential(OrderedDict([("conv", nn.Conv2d(c, hidden_dim, kernel_size=1, bias=False)),
                                       ("norm", nn.BatchNorm2d(hidden_dim))]))
            for c in self.in_channels])
        layer = TransformerEncoderLayer(hidden_dim, nhead=nhead, dim_feedforward=dim_feedforward, dropout=dropout,
                                        activation=enc_act)
        self.encoder = nn.ModuleList([TransformerEncoder(copy.deepcopy(layer), num_encoder_layers)
                                      for _ in range(len(self.use_encoder_idx))])
        self.lateral_convs = nn.ModuleList()
        self.fpn_blocks = nn.ModuleList()
        for _ in range(n_levels - 1, 0, -1):
            self.lateral_convs.append(ConvNormLayer(hidden_dim, hidden_dim, 1, 1, act=act))
            self.fpn_blocks.append(RepNCSPELAN4(hidden_dim * 2, hidden_dim, hidden_dim * 2, self.c4, self.n_blocks))
        self.downsample_convs = nn.ModuleList()
        self.pan_blocks = nn.ModuleList()
        for _ in range(n_levels - 1):
            self.downsample_convs.append(nn.Sequential(SCDown(hidden_dim, hidden_dim, 3, 2)))
            self.pan_blocks.append(RepNCSPELAN4(hidden_dim * 2, hidden_dim, hidden_dim * 2, self.c4, self.n_blocks))
        if freeze_network:
            for p in self.parameters():
                p.requires_grad = False

    def forward(self, feats):
        raise NotImplementedError("run the full model through DETRPose.forward (HIP engine)")


def sine_pos_embed_2d(w, h, dim, temperature_w=20.0, temperature_h=20.0):
    """HybridEncoder.create_sinehw_position_embedding (hybrid_encoder.py:431-460):
    (1, h*w, 2*dim) with [pos_y | pos_x], sin/cos interleaved, grid from 1..n / (n+1e-6)."""
    import math

    import torch
    gw = torch.arange(1, int(w) + 1, dtype=torch.float32)
    gh = torch.arange(1, int(h) + 1, dtype=torch.float32)
    gh, gw = torch.meshgrid(gh, gw, indexing="ij")
    gw = gw / (int(w) + 1e-6) * (2 * math.pi)
    gh = gh / (int(h) + 1e-6) * (2 * math.pi)
    d = torch.arange(dim, dtype=torch.float32)
    dx = temperature_w ** (2 * torch.div(d, 2, rounding_mode="floor") / dim)
    dy = temperature_h ** (2 * torch.div(d, 2, rounding_mode="floor") / dim)
    px = gw[..., None] / dx
    py = gh[..., None] / dy
    px = torch.stack((px[..., 0::2].sin(), px[..., 1::2].cos()), 3).flatten(2)
    py = torch.stack((py[..., 0::2].sin(), py[..., 1::2].cos()), 3).flatten(2)
    return torch.cat((py, px), 2).reshape(1, int(h) * int(w), 2 * dim)
