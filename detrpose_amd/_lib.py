"""ctypes binding of libdetrpose_hip.so (include/detrpose_hip.h).

Loading fails loudly: there is no CPU or eager-PyTorch fallback for any op of the
forward. Build the library with `python -m detrpose_amd.build` (or
__graft_entry__.build()).
"""
from __future__ import annotations

import ctypes as C
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("DETRPOSE_HIP_LIB", os.path.join(_HERE, "lib", "libdetrpose_hip.so"))

DP_F32, DP_BF16 = 0, 1
DP_SQNORM_PARTS = 1024   # upper bound of dp_grad_sqnorm_ws_floats(n)
DP_ACT_NONE, DP_ACT_RELU, DP_ACT_SILU, DP_ACT_GELU = 0, 1, 2, 3
DP_MSDA_OFFATTN_F32 = 0x100
ACT = {None: 0, "none": 0, "relu": 1, "silu": 2, "gelu": 3}

i32, i64, f32, vp = C.c_int32, C.c_int64, C.c_float, C.c_void_p


class ConvDesc(C.Structure):
    """Mirror of dp_conv_desc."""
    _fields_ = [
        ("in_", vp), ("in_bstride", i64), ("in_pstride", i32), ("in_h", i32), ("in_w", i32), ("cin", i32),
        ("weight", vp), ("kpad", i32),
        ("bias", vp),
        ("kh", i32), ("kw", i32), ("stride", i32), ("pad_t", i32), ("pad_l", i32),
        ("out", vp), ("out_bstride", i64), ("out_pstride", i32), ("out_h", i32), ("out_w", i32), ("cout", i32),
        ("res", vp), ("res_bstride", i64), ("res_pstride", i32),
        ("batch", i32),
        ("act", i32), ("has_lab", i32), ("lab_scale", f32), ("lab_bias", f32),
        ("dtype", i32),
        ("up", vp), ("up_bstride", i64), ("up_pstride", i32),
        ("out_f32", i32),
        ("in_seg_ch", i32), ("in_seg_stride", i64),
    ]


class RowMap(C.Structure):
    """Mirror of dp_rowmap: row r -> base + (r // group) * stride_g + (r % group) * stride_r."""
    _fields_ = [("base", i64), ("group", i32), ("stride_g", i64), ("stride_r", i64)]


class StemWeights(C.Structure):
    """dp_stem_weights (include/detrpose_hip.h)."""
    _fields_ = [("w1", vp), ("b1", vp), ("w2a", vp), ("b2a", vp), ("w2b", vp), ("b2b", vp), ("w3", vp), ("b3", vp),
                ("w4", vp), ("b4", vp), ("k2a", i32), ("k2b", i32), ("k3", i32), ("k4", i32), ("mid", i32),
                ("cout", i32), ("has_lab", i32), ("lab", (f32 * 2) * 5)]


class LossHead(C.Structure):
    """Mirror of dp_loss_head."""
    _fields_ = [("logits", vp), ("lg_b", i64), ("lg_q", i32), ("kps", vp), ("kp_b", i64), ("kp_q", i32),
                ("match", vp)]


class GemmDesc(C.Structure):
    """Mirror of dp_gemm_desc."""
    _fields_ = [("a", vp), ("a_bs", i64), ("a_rs", i64), ("a_ks", i64),
                ("b", vp), ("b_bs", i64), ("b_ks", i64), ("b_ns", i64),
                ("c", vp), ("c_bs", i64), ("c_rs", i64),
                ("batch", i32), ("m", i32), ("n", i32), ("k", i32),
                ("in_dtype", i32), ("out_dtype", i32),
                ("bias", vp), ("alpha", f32), ("beta", f32), ("act", i32),
                ("gate", vp), ("gate_bs", i64), ("gate_rs", i64), ("gate_dtype", i32),
                ("split_k", i32), ("colsum", vp)]


class PackDesc(C.Structure):
    """Mirror of dp_pack_desc."""
    _fields_ = [("w", vp), ("out", vp), ("scale", vp), ("cout", i32), ("cin", i32), ("kh", i32), ("kw", i32),
                ("kpad", i32), ("kc", i32), ("mode", i32), ("dtype", i32)]


class RowCopyDesc(C.Structure):
    """Mirror of dp_rowcopy_desc."""
    _fields_ = [("src0", vp), ("src1", vp), ("dst", vp), ("ld_src0", i64), ("ld_src1", i64), ("ld_dst", i64),
                ("rows", i32), ("n", i32)]


def rowmap(base=0, group=1, stride_g=0, stride_r=0) -> RowMap:
    return RowMap(int(base), int(group), int(stride_g), int(stride_r))


def contiguous_rows(ld: int, base: int = 0) -> RowMap:
    return RowMap(int(base), 1, int(ld), 0)


_SIGS = {
    "dp_last_error": (C.c_char_p, []),
    "dp_version": (i32, []),
    "dp_source_hash": (C.c_char_p, []),
    "dp_conv2d": (i32, [C.POINTER(ConvDesc), vp]),
    "dp_conv2d_describe": (i32, [C.POINTER(ConvDesc), C.c_char_p, i32]),
    "dp_dwconv2d": (i32, [C.POINTER(ConvDesc), vp]),
    "dp_stem_conv": (i32, [vp, i32, i32, i32, vp, vp, i32, i32, f32, f32, vp, i64, i32, i32, vp]),
    "dp_maxpool2x2_pad_rb": (i32, [vp, i64, i32, i32, i32, i32, i32, vp, i64, i32, i32, vp]),
    "dp_conv2d_pool": (i32, [C.POINTER(ConvDesc), vp, i64, i32, vp]),
    "dp_stem_fused": (i32, [vp, i32, i32, i32, C.POINTER(StemWeights), vp, i64, i32, vp]),
    "dp_add_rows": (i32, [vp, RowMap, vp, RowMap, vp, RowMap, i32, i32, i32, vp]),
    "dp_layernorm": (i32, [vp, RowMap, vp, RowMap, vp, RowMap, vp, vp, f32, i32, i32, vp, RowMap, i32, i32,
                           vp, i32, vp, i32, vp]),
    "dp_gate_layernorm": (i32, [vp, i32, vp, vp, vp, vp, f32, i32, i32, i32, vp]),
    "dp_attention": (i32, [vp, i32, vp, vp, i32, vp, i32, i32, i32, i64, i64, i64, i32, i32, i32, i32, vp]),
    "dp_msda": (i32, [vp, i32, i32, vp, i32, vp, vp, vp, i32, i32, i32, i32, i32, i32, vp]),
    "dp_layernorm_classmax": (i32, [vp, vp, vp, vp, f32, i32, i32, vp, i32, vp, vp, vp, i32, vp, i32, vp]),
    "dp_resize_pad": (i32, [vp, i32, i32, i32, i32, vp, i32, i32, f32, vp]),
    "dp_msda_core_fwd": (i32, [vp, i32, i32, vp, i32, vp, vp, vp, i32, i32, i32, i32, i32, vp]),
    "dp_msda_core_bwd": (i32, [vp, i32, i32, vp, i32, vp, vp, vp, i32, i32, i32, i32, vp, vp, vp, i32, vp]),
    "dp_msda_bwd": (i32, [vp, i32, i32, vp, i32, vp, vp, vp, i32, i32, i32, i32, i32, vp, i32, vp, vp, i32, vp]),
    "dp_msda_bwd_ws_bytes": (i64, [i32, i32, vp, i32, i32, i32, i32]),
    "dp_msda_bwd_sorted": (i32, [vp, i32, i32, vp, i32, vp, vp, vp, i32, i32, i32, i32, i32, vp, i32, vp, vp, vp, i64,
                                 i32, vp]),
    "dp_topk": (i32, [vp, i32, i32, i32, i32, vp, vp, vp]),
    "dp_class_max": (i32, [vp, i32, i32, vp, vp, i32, vp, i32, vp]),
    "dp_gather_rows": (i32, [vp, i64, vp, i32, i32, i32, vp, i32, vp]),
    "dp_refpoint_init": (i32, [vp, vp, vp, i32, i32, i32, vp, vp]),
    "dp_broadcast": (i32, [vp, i64, vp, i32, vp]),
    "dp_sine_embed": (i32, [vp, i32, i32, i32, vp, vp, i32, vp]),
    "dp_linear_small": (i32, [vp, RowMap, i32, i32, i32, vp, vp, i32, i32, i32, vp, vp, vp]),
    "dp_pose_refine": (i32, [vp, vp, i32, vp, f32, i32, i32, vp, vp, vp]),
    "dp_pre_pose": (i32, [vp, vp, i32, i32, vp, vp]),
    "dp_lqe_stats": (i32, [vp, i64, i32, i32, i32, vp, i32, i32, i32, vp, i32, vp]),
    "dp_postprocess": (i32, [vp, vp, vp, i32, i32, i32, i32, i32, vp, vp, vp, vp]),
    "dp_linear_layernorm": (i32, [vp, RowMap, vp, RowMap, i32, vp, vp, vp, RowMap, vp, vp, f32, i32, i32, vp, RowMap,
                                  i32, i32, vp]),
    "dp_gate_linear_layernorm": (i32, [vp, RowMap, vp, RowMap, vp, vp, vp, vp, f32, i32, i32, vp]),
    "dp_linear_layernorm_classmax": (i32, [vp, vp, i32, i32, vp, vp, vp, vp, f32, vp, i32, vp, vp, vp, i32, vp, vp]),
    "dp_mha_layernorm": (i32, [vp, RowMap, vp, RowMap, i32, i32, i64, i64, i64, i32, vp, vp, vp, vp, vp, vp, f32, i32,
                               i32, vp, RowMap, i32, i32, vp, i32, vp, vp, i32, vp]),
    "dp_ffn_layernorm": (i32, [vp, RowMap, vp, RowMap, vp, vp, i32, vp, vp, vp, vp, f32, i32, i32, vp]),
    "dp_query_pos": (i32, [vp, i32, i32, vp, vp, vp, vp, vp, vp, vp, RowMap, i32, vp]),
    "dp_pose_mlp": (i32, [vp, RowMap, vp, RowMap, i32, vp, vp, vp, vp, vp, vp, i32, vp, vp, i32, vp]),
    "dp_hungarian_match": (i32, [vp, i64, i64, i32, i32, vp, i64, i64, i32, i32, vp, vp, vp, vp, i32, i32, i32, i32,
                                 f32, f32, f32, f32, vp, vp, vp, vp]),
    "dp_match_union": (i32, [vp, i32, i32, i32, vp, vp, vp]),
    "dp_pose_loss": (i32, [C.POINTER(LossHead), i32, i32, i32, i32, i32, vp, vp, vp, vp, vp, vp, f32, f32, vp, vp,
                           f32, f32, f32, f32, vp, vp, vp, vp, vp]),
    # training step (include/detrpose_hip.h, "Training step")
    "dp_gemm": (i32, [C.POINTER(GemmDesc), vp]),
    "dp_ln_fwd": (i32, [vp, i32, vp, vp, vp, vp, vp, vp, f32, i32, i32, vp, i32, i32, i32, vp]),
    "dp_ln_bwd": (i32, [vp, vp, i32, vp, vp, vp, i32, i32, vp, vp, i32, i32, vp]),
    "dp_conv_wgrad": (i32, [vp, i64, i32, i32, i32, i32, i32, vp, i64, i32, i32, i32, i32, i32, i32, i32, vp, vp,
                            i32, vp]),
    "dp_conv_wgrad_zs": (i32, [vp, i64, i32, i32, i32, i32, i32, vp, i64, i32, i32, i32, i32, i32, i32, i32, vp,
                               vp, i32, vp]),
    "dp_colsum": (i32, [vp, i64, i32, i32, vp, i32, i32, vp]),
    "dp_attn_fwd": (i32, [vp, i32, vp, vp, i32, vp, i32, vp, vp, i32, i32, i64, i64, i64, i32, i32, i32, i32, vp]),
    "dp_attn_bwd": (i32, [vp, i32, vp, vp, i32, vp, vp, vp, i32, vp, i32, vp, vp, i32, i32, i32, i64, i64, i64, i32, i32,
                          i32, i32, vp]),
    "dp_gate_fwd": (i32, [vp, vp, vp, vp, i32, i32, i32, vp]),
    "dp_gate_bwd": (i32, [vp, vp, vp, vp, vp, i32, i32, i32, vp]),
    "dp_query_build": (i32, [vp, vp, vp, vp, vp, vp, i32, i32, i32, i32, i32, vp, i32, vp]),
    "dp_query_build_bwd": (i32, [vp, vp, i32, i32, i32, i32, i32, vp, vp, vp, vp, i32, vp, i32, vp]),
    "dp_pose_refine_bwd": (i32, [vp, vp, i32, f32, vp, i32, i32, vp, i32, vp]),
    "dp_sigmoid_bwd": (i32, [vp, vp, vp, i32, i32, i64, i64, i64, vp]),
    "dp_lqe_stats_bwd": (i32, [vp, i64, i32, i32, i32, vp, vp, i32, i32, i32, vp, vp, i64, i32, vp]),
    "dp_scatter_rows": (i32, [vp, i32, vp, vp, i32, i32, i32, i32, vp, i64, i32, i32, i32, vp]),
    "dp_gather_rows_masked": (i32, [vp, i64, vp, vp, i32, i32, i32, i32, vp, i32, vp]),
    "dp_convert_rows": (i32, [vp, i32, i64, vp, i32, i64, i32, i32, f32, i32, vp]),
    "dp_copy_rows_check": (i32, [vp, i32]),
    "dp_copy_rows_batch": (i32, [vp, i32, i32, vp]),
    "dp_zero": (i32, [vp, i64, vp]),
    "dp_cdn_build": (i32, [vp, vp, vp, vp, vp, vp, i32, i32, i32, i32, f32, i32, f32, f32, C.c_uint64, vp, vp, vp]),
    "dp_grad_sqnorm": (i32, [vp, i64, vp, vp, i64, vp]),
    "dp_grad_sqnorm_ws_floats": (i64, [i64]),
    "dp_adamw": (i32, [vp, vp, vp, vp, i64, f32, f32, f32, f32, f32, i32, f32, vp, vp, vp]),
    "dp_finite_guard": (i32, [vp, i64, vp, vp]),
    "dp_ema": (i32, [vp, vp, i64, f32, vp, vp]),
    # HybridEncoder training (csrc/encoder_train.hip)
    "dp_bn_stats": (i32, [vp, i64, i32, i32, vp, vp, i64, i32, vp]),
    "dp_bn_stats_ws_bytes": (i64, [i32, i32]),
    "dp_bn_finalize": (i32, [vp, i32, f32, i32, f32, f32, vp, vp, vp, vp]),
    "dp_bn_stats_finalize": (i32, [vp, i64, i32, i32, vp, vp, i64, f32, f32, vp, vp, vp, i32, vp]),
    "dp_bn_act_fwd": (i32, [vp, i64, vp, i64, vp, vp, vp, vp, i64, vp, vp, vp, vp, i64, i32, i32, i32, i32, vp]),
    "dp_bn_act_bwd_reduce": (i32, [vp, i64, vp, i64, vp, vp, vp, vp, i64, vp, vp, vp, i32, i32, i32, vp, vp, vp, vp,
                                   vp, vp, i64, i32, vp]),
    "dp_bn_act_bwd_reduce_ws_bytes": (i64, [i32, i32]),
    "dp_bn_act_bwd_apply": (i32, [vp, i64, vp, i64, vp, i64, vp, i64, vp, vp, vp, vp, i64, vp, vp, vp, i32, i32, i32,
                                  vp, f32, i32, vp]),
    "dp_im2col": (i32, [vp, i64, i32, i64, i32, i32, i32, i32, i32, i32, i32, i32, i32, i32, vp, i32, i32, vp]),
    "dp_conv_pack": (i32, [vp, i32, i32, i32, i32, vp, i32, i32, i32, vp, i32, vp]),
    "dp_conv_pack_check": (i32, [vp, i32]),
    "dp_conv_pack_batch": (i32, [vp, i32, i32, vp]),
    "dp_frozen_act_bwd": (i32, [vp, i64, vp, i64, vp, i64, vp, i64, i32, i32, i32, vp, vp, vp, vp, vp, i32, vp]),
    "dp_col2im": (i32, [vp, i32, i32, i32, i32, i32, i32, i32, i32, i32, i32, vp, i64, i32, i32, i32, vp]),
    "dp_maxpool2x2_pad_rb_bwd": (i32, [vp, i64, i32, vp, i64, i32, i32, i32, i32, i32, vp, i64, i32, i32, vp]),
    "dp_dwconv_bwd": (i32, [vp, i64, i32, vp, i64, i32, vp, i32, i32, i32, i32, i32, i32, i32, i32, i32, vp, i64, i32,
                            vp, i32, vp]),
    "dp_upsample2x": (i32, [vp, i64, i32, i32, i32, i32, i32, vp, i64, i32, i32, i32, vp]),
    "dp_axpby_rows": (i32, [vp, i64, vp, i64, f32, vp, i64, f32, i32, i32, i32, i32, vp]),
    "dp_act_bwd": (i32, [vp, i64, vp, i64, vp, i64, i32, i32, i32, i32, vp]),
}

EXPORTED = tuple(k for k in _SIGS)

_lib = None


class HipError(RuntimeError):
    pass


def load():
    """Load and prototype the library (once). Raises if it is missing."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise HipError(f"libdetrpose_hip.so not found at {LIB_PATH}: the DETRPose forward runs only on the HIP "
                       f"kernels (no CPU fallback). Build it with `python -m detrpose_amd.build`.")
    lib = C.CDLL(LIB_PATH)
    for name, (res, args) in _SIGS.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    verify_source(lib)
    _lib = lib
    return lib


def verify_source(lib, expected: str | None = None):
    """Refuse a library built from other sources than the ones shipped beside it (the .so is
    git-ignored and travels prebuilt; a stale one would otherwise be tested and benched
    silently). DETRPOSE_ALLOW_STALE_LIB=1 skips the check (A/B variant libraries only)."""
    if os.environ.get("DETRPOSE_ALLOW_STALE_LIB"):
        return
    from .build import CSRC, lib_source_hash
    if expected is None:
        if not os.path.isdir(CSRC):
            return
        expected = lib_source_hash()
    got = lib.dp_source_hash().decode()
    if got != expected:
        raise HipError(f"{LIB_PATH} was built from sources {got}, the shipped sources are {expected}: "
                       f"rebuild it with `python -m detrpose_amd.build`")


def check(rc: int, what: str = ""):
    if rc:
        msg = load().dp_last_error().decode(errors="replace")
        raise HipError(f"{what or 'dp call'} failed (rc={rc}): {msg}")
