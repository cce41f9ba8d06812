"""Constructor kwargs for the DETRPose N / L / X models.

These are the kwargs the reference's LazyConfig files hand to its constructors,
restated as plain dicts (LazyConfig/omegaconf is out of scope):

* common model block:  configs/detrpose/include/detrpose_hgnetv2.py:29-84
* postprocessor:       configs/detrpose/include/detrpose_hgnetv2.py:100
* N overrides:         configs/detrpose/detrpose_hgnetv2_n.py:42-60
* X overrides:         configs/detrpose/detrpose_hgnetv2_x.py:42-47
* L:                   configs/detrpose/detrpose_hgnetv2_l.py (no model overrides)
"""
from __future__ import annotations

import copy

EVAL_SPATIAL_SIZE = (640, 640)

_BASE = {
    "backbone": dict(
        name="B4",
        use_lab=False,
        return_idx=[1, 2, 3],
        freeze_stem_only=True,
        freeze_at=-1,
        freeze_norm=True,
        pretrained=False,  # True downloads weights (hgnetv2.py:548); never offline
    ),
    "encoder": dict(
        in_channels=[512, 1024, 2048],
        feat_strides=[8, 16, 32],
        n_levels=3,
        hidden_dim=256,
        nhead=8,
        dim_feedforward=1024,
        dropout=0.0,
        enc_act="gelu",
        expansion=1.0,
        depth_mult=1.0,
        act="silu",
        temperatureH=20,
        temperatureW=20,
        eval_spatial_size=EVAL_SPATIAL_SIZE,
    ),
    "transformer": dict(
        hidden_dim=256,
        dropout=0.0,
        nhead=8,
        num_queries=60,
        dim_feedforward=1024,
        num_decoder_layers=6,
        normalize_before=False,
        return_intermediate_dec=True,
        activation="relu",
        num_feature_levels=3,
        dec_n_points=4,
        learnable_tgt_init=True,
        two_stage_type="standard",
        num_body_points=17,
        aux_loss=True,
        num_classes=2,
        dec_pred_class_embed_share=False,
        dec_pred_pose_embed_share=False,
        two_stage_class_embed_share=False,
        two_stage_bbox_embed_share=False,
        cls_no_bias=False,
        feat_strides=[8, 16, 32],
        eval_spatial_size=EVAL_SPATIAL_SIZE,
        reg_max=32,
        reg_scale=4,
        energy_decrease_weight=0.0,
    ),
    "postprocessor": dict(num_select=60, num_body_points=17),
}


def _n(cfg):
    # configs/detrpose/detrpose_hgnetv2_n.py:42-60
    cfg["backbone"].update(name="B0", use_lab=True, return_idx=[2, 3])
    cfg["encoder"].update(in_channels=[512, 1024], feat_strides=[16, 32], n_levels=2,
                          use_encoder_idx=[1], depth_mult=0.5, expansion=0.34,
                          hidden_dim=128, dim_feedforward=512)
    cfg["transformer"].update(num_decoder_layers=3, num_feature_levels=2, dim_feedforward=512,
                              feat_strides=[16, 32], hidden_dim=128, dec_n_points=6,
                              use_kan=False, kan_grid=3)
    return cfg


def _x(cfg):
    # configs/detrpose/detrpose_hgnetv2_x.py:42-47
    cfg["backbone"].update(name="B5")
    cfg["encoder"].update(hidden_dim=384, dim_feedforward=2048)
    cfg["transformer"].update(hidden_dim=384, reg_scale=8)
    return cfg


def get_config(size: str) -> dict:
    """Return a deep copy of the constructor kwargs for size 'n' | 'l' | 'x'."""
    size = size.lower()
    cfg = copy.deepcopy(_BASE)
    if size == "n":
        return _n(cfg)
    if size == "l":
        return cfg
    if size == "x":
        return _x(cfg)
    raise ValueError(f"unknown DETRPose size {size!r} (expected n, l or x)")


# The training loop's hyper-parameters (configs/detrpose/include/detrpose_hgnetv2.py:13-21
# training_params: clip 0.1, grad_accum_steps 2 unless a size file overrides it; the size files'
# AdamW (lr 1e-4, betas (0.9, 0.999), weight_decay 1e-4) with the backbone parameter group's lr,
# ModelEMA(0.9999, warmups 2000)): detrpose_hgnetv2_n.py:13, 26; detrpose_hgnetv2_l.py:25 (no
# grad_accum override); detrpose_hgnetv2_x.py:13, 26.
TRAINING = {
    "n": dict(grad_accum_steps=1, backbone_lr=1e-4),
    "l": dict(grad_accum_steps=2, backbone_lr=1e-5),
    "x": dict(grad_accum_steps=1, backbone_lr=5e-5),
}
TRAINING_COMMON = dict(lr=1e-4, betas=(0.9, 0.999), weight_decay=1e-4, max_norm=0.1, ema_decay=0.9999,
                       ema_warmups=2000)


def training_params(size: str) -> dict:
    return {**TRAINING_COMMON, **TRAINING[size.lower()]}


# Algorithmic forward FLOPs per 640x640 image (2 FLOP / MAC), measured with
# torch.utils.flop_counter on the reference in the survey.
GFLOP_PER_IMAGE = {"n": 8.91, "l": 103.86, "x": 232.04}
