"""Differentiable MSDA core on the HIP kernels (training interface).

`ms_deform_attn_core(value, value_spatial_shapes, sampling_locations, attention_weights)`
is the drop-in for the reference's `ms_deform_attn_core_pytorch` default branch
(/root/reference/src/models/detrpose/ms_deform_attn.py:145-193, called at :436-441):
same math (per level F.grid_sample(bilinear, zeros, align_corners=False) at 2*loc-1, then
the attention-weighted sum), forward by `dp_msda_core_fwd` and backward by
`dp_msda_core_bwd` (grad_value by f32 atomics, grad_loc, grad_attn). Value is taken in the
encoder-memory layout (N, S, nH*Dh) the rest of this package uses, rather than the
reference's per-level (N*nH, Dh, H*W) list; `value_from_levels` converts.

There is no CPU path: the HIP library must load (see _lib.load()).
"""
from __future__ import annotations

import ctypes as C

import torch

from . import _lib

_DT = {torch.float32: _lib.DP_F32, torch.bfloat16: _lib.DP_BF16}


def _shapes_arg(shapes):
    hw = [int(v) for hw in shapes for v in hw]
    return (C.c_int32 * len(hw))(*hw), len(hw) // 2


def _check(value, shapes, loc, attn):
    N, S, Cc = value.shape
    _, Lq, nH, L, P, two = loc.shape
    if two != 2 or attn.shape != (N, Lq, nH, L, P) or loc.shape[0] != N:
        raise ValueError(f"msda core: loc {tuple(loc.shape)} / attn {tuple(attn.shape)} do not match value {tuple(value.shape)}")
    if Cc % nH:
        raise ValueError(f"msda core: {Cc} channels not divisible by {nH} heads")
    if sum(int(h) * int(w) for h, w in shapes) != S or len(shapes) != L:
        raise ValueError("msda core: spatial shapes do not match value / loc")
    if value.dtype not in _DT:
        raise TypeError(f"msda core: value dtype {value.dtype} (f32 / bf16)")
    if not value.is_cuda:
        raise RuntimeError("msda core: tensors must be on the GPU (no CPU path)")
    if loc.device != value.device or attn.device != value.device:
        raise RuntimeError(f"msda core: value on {value.device}, loc on {loc.device}, attn on {attn.device}: "
                           "all three must be on the same GPU")
    return N, S, Cc, Lq, nH, L, P


class MSDeformAttnCoreFunction(torch.autograd.Function):
    @staticmethod
    def forward(ctx, value, shapes, loc, attn):
        N, S, Cc, Lq, nH, L, P = _check(value, shapes, loc, attn)
        value = value.contiguous()
        loc = loc.contiguous().float()
        attn = attn.contiguous().float()
        out = torch.empty(N, Lq, Cc, device=value.device, dtype=value.dtype)
        hw, nl = _shapes_arg(shapes)
        lib = _lib.load()
        s = torch.cuda.current_stream(value.device).cuda_stream
        _lib.check(lib.dp_msda_core_fwd(value.data_ptr(), N, S, hw, nl, loc.data_ptr(), attn.data_ptr(), out.data_ptr(),
                                        Lq, nH, Cc // nH, P, _DT[value.dtype], C.c_void_p(s)), "dp_msda_core_fwd")
        ctx.save_for_backward(value, loc, attn)
        ctx.shapes = [tuple(int(v) for v in hw_) for hw_ in shapes]
        return out

    @staticmethod
    def backward(ctx, grad_out):
        value, loc, attn = ctx.saved_tensors
        N, S, Cc = value.shape
        _, Lq, nH, L, P, _ = loc.shape
        go = grad_out.contiguous().to(value.dtype)
        gv = torch.empty(N, S, Cc, device=value.device, dtype=torch.float32)
        gl = torch.empty_like(loc)
        ga = torch.empty_like(attn)
        hw, nl = _shapes_arg(ctx.shapes)
        lib = _lib.load()
        s = torch.cuda.current_stream(value.device).cuda_stream
        _lib.check(lib.dp_msda_core_bwd(value.data_ptr(), N, S, hw, nl, loc.data_ptr(), attn.data_ptr(), go.data_ptr(),
                                        Lq, nH, Cc // nH, P, gv.data_ptr(), gl.data_ptr(), ga.data_ptr(),
                                        _DT[value.dtype], C.c_void_p(s)), "dp_msda_core_bwd")
        return gv.to(value.dtype), None, gl, ga


def ms_deform_attn_core(value, value_spatial_shapes, sampling_locations, attention_weights):
    """value (N, S, nH*Dh); shapes [(H, W)] per level; loc (N, Lq, nH, L, P, 2) in [0, 1];
    attn (N, Lq, nH, L, P) softmaxed -> (N, Lq, nH*Dh). Differentiable in value, loc, attn."""
    return MSDeformAttnCoreFunction.apply(value, value_spatial_shapes, sampling_locations, attention_weights)


class MSDeformAttnFunction(torch.autograd.Function):
    """The fused op of MSDeformAttn.forward's default branch (ms_deform_attn.py:384-441):
    raw offsets | attention logits + reference points -> softmax, sampling locations,
    bilinear gather, weighted sum. Forward `dp_msda` (the inference kernel), backward
    `dp_msda_bwd_sorted` (softmax and location chain rule fused into the gather backward, the
    value gradient summed per pixel without float atomics; see msda_bwd)."""

    @staticmethod
    def forward(ctx, value, shapes, offattn, ref, n_heads, n_points):
        N, S, Cc = value.shape
        rows, ncol = offattn.shape
        L = len(shapes)
        if value.dtype not in _DT:
            raise TypeError(f"msda: value dtype {value.dtype} (f32 / bf16)")
        if not (value.is_cuda and offattn.device == value.device and ref.device == value.device):
            raise RuntimeError("msda: value, offattn and ref must be on the same GPU (no CPU path)")
        if ncol != n_heads * L * n_points * 3 or rows % N or ref.shape != (rows, 2) or Cc % n_heads:
            raise ValueError(f"msda: offattn {tuple(offattn.shape)} / ref {tuple(ref.shape)} do not match value "
                             f"{tuple(value.shape)} with {n_heads} heads, {L} levels, {n_points} points")
        if sum(int(h) * int(w) for h, w in shapes) != S:
            raise ValueError("msda: spatial shapes do not match value")
        lq = rows // N
        value = value.contiguous()
        # offsets / logits stay f32 whatever value's dtype (DP_MSDA_OFFATTN_F32): bf16 would round
        # offsets of tens of pixels by up to ~0.1 px, and the backward differentiates at the
        # f32 values, as the reference's f32 Linear outputs
        oa = offattn.detach().float().contiguous()
        ref = ref.detach().float().contiguous()
        out = torch.empty(N, lq, Cc, device=value.device, dtype=value.dtype)
        hw, nl = _shapes_arg(shapes)
        lib = _lib.load()
        s = torch.cuda.current_stream(value.device).cuda_stream
        _lib.check(lib.dp_msda(value.data_ptr(), N, S, hw, nl, oa.data_ptr(), ref.data_ptr(), out.data_ptr(), Cc, lq,
                               n_heads, Cc // n_heads, n_points, _DT[value.dtype] | _lib.DP_MSDA_OFFATTN_F32,
                               C.c_void_p(s)), "dp_msda")
        ctx.save_for_backward(value, oa, ref)
        ctx.shapes = [tuple(int(v) for v in hw_) for hw_ in shapes]
        ctx.n_heads, ctx.n_points = n_heads, n_points
        return out

    @staticmethod
    def backward(ctx, grad_out):
        value, oa, ref = ctx.saved_tensors
        gv, goa, gref = msda_bwd(value, ctx.shapes, oa, ref, grad_out, ctx.n_heads, ctx.n_points,
                                 want_ref=ctx.needs_input_grad[3])
        return gv.to(value.dtype), None, goa, gref, None, None


def msda_bwd(value, shapes, offattn, ref, grad_out, n_heads, n_points, want_ref=True, method="sorted"):
    """The backward of msdeform_attn as a function: (grad_value f32 (N, S, C), grad_offattn f32,
    grad_ref f32 (rows, 2) or None). method "sorted": dp_msda_bwd_sorted (value gradient by a
    per-pixel counting sort and register sums; falls to "atomic" outside its shape range),
    "atomic": dp_msda_bwd (f32 atomics)."""
    N, S, Cc = value.shape
    rows = offattn.shape[0]
    lq = rows // N
    dh = Cc // n_heads
    go = grad_out.contiguous().to(value.dtype)
    oa = offattn.detach().float().contiguous()
    ref = ref.detach().float().contiguous()
    gv = torch.empty(N, S, Cc, device=value.device, dtype=torch.float32)
    goa = torch.empty(oa.shape, device=value.device, dtype=torch.float32)
    gref = torch.empty(rows, 2, device=value.device, dtype=torch.float32) if want_ref else None
    hw, nl = _shapes_arg(shapes)
    lib = _lib.load()
    s = C.c_void_p(torch.cuda.current_stream(value.device).cuda_stream)
    args = (value.data_ptr(), N, S, hw, nl, oa.data_ptr(), ref.data_ptr(), go.data_ptr(), Cc, lq, n_heads, dh,
            n_points, gv.data_ptr(), 0, goa.data_ptr(), gref.data_ptr() if gref is not None else None)
    nb = int(lib.dp_msda_bwd_ws_bytes(N, S, hw, nl, lq, n_heads, n_points)) if method == "sorted" else -1
    if nb > 0 and dh in (8, 16, 32, 64):
        ws = torch.empty(nb, device=value.device, dtype=torch.uint8)
        _lib.check(lib.dp_msda_bwd_sorted(*args, ws.data_ptr(), nb, _DT[value.dtype], s), "dp_msda_bwd_sorted")
    elif method in ("sorted", "atomic"):
        _lib.check(lib.dp_msda_bwd(*args, _DT[value.dtype], s), "dp_msda_bwd")
    else:
        raise ValueError(f"msda_bwd: method {method!r}")
    return gv, goa, gref


def msdeform_attn(value, shapes, offattn, ref, n_heads, n_points):
    """value (N, S, C); offattn (N*Lq, nH*L*P*3) = [sampling_offsets | attention_weights]
    Linear outputs; ref (N*Lq, 2) one point per query shared by the levels -> (N, Lq, C).
    Differentiable in value, offattn and ref."""
    return MSDeformAttnFunction.apply(value, shapes, offattn, ref, n_heads, n_points)


def value_from_levels(value_list, n_heads):
    """The reference's per-level value list [(N*nH, Dh, H*W)] -> (N, S, nH*Dh)."""
    parts = []
    for v in value_list:
        NM, Dh, HW = v.shape
        parts.append(v.reshape(NM // n_heads, n_heads, Dh, HW).permute(0, 3, 1, 2).reshape(NM // n_heads, HW, n_heads * Dh))
    return torch.cat(parts, 1)
