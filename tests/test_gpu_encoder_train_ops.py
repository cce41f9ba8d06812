"""The HybridEncoder training kernels (csrc/encoder_train.hip, the AIFI attention in
csrc/train.hip) through the C ABI vs torch fp32 autograd of the same ops: BatchNorm2d in
training mode (one and two branches, SyncBN's per-rank combination, running statistics),
its backward, the conv weight gradient via im2col + dp_gemm, the flipped-weight input
gradient as a dp_conv2d, depthwise conv backward, nearest x2, GELU backward and 400-token
attention (hybrid_encoder.py:56-212, 246-296). fp32 bound: 2e-4 of the output scale."""
import ctypes as C

import pytest
import torch
import torch.nn.functional as F

from detrpose_amd import _lib
from detrpose_amd._lib import DP_BF16, DP_F32, ConvDesc, GemmDesc

pytestmark = pytest.mark.gpu
DEV = "cuda"
ACTS = {"silu": _lib.DP_ACT_SILU, "relu": _lib.DP_ACT_RELU, None: _lib.DP_ACT_NONE}


def _s():
    return C.c_void_p(torch.cuda.current_stream().cuda_stream)


def _close(got, ref, what, tol=2e-4):
    got, ref = got.float().cpu(), ref.float().cpu()
    scale = max(1.0, float(ref.abs().max()))
    err = float((got - ref).abs().max())
    print(f"{what}: max err {err:.3g} (scale {scale:.3g})")
    assert err <= tol * scale, (what, err, scale)


def _act(x, a):
    return {"silu": F.silu, "relu": F.relu, None: lambda t: t}[a](x)


_RWS = []


def _rws(lib, rows, c):
    """A workspace for dp_bn_act_bwd_reduce's per-slice partials (kept alive past the launch)."""
    t = torch.empty(int(lib.dp_bn_act_bwd_reduce_ws_bytes(rows, c)) // 4, device=DEV)
    _RWS.append(t)
    return t


def bn_stats(lib, z, count_parts=1):
    """per-part dp_bn_stats over row splits, then dp_bn_finalize: (mean_rstd, parts)."""
    rows, c = z.shape
    parts = torch.zeros(count_parts, 3, c, device=DEV)
    per = rows // count_parts
    for p in range(count_parts):
        zp = z[p * per:(p + 1) * per]
        nb = int(lib.dp_bn_stats_ws_bytes(per, c))
        ws = torch.empty(nb // 4, device=DEV)
        _lib.check(lib.dp_bn_stats(zp.data_ptr(), c, per, c, parts[p].data_ptr(), ws.data_ptr(), nb, DP_F32, _s()),
                   "bn_stats")
    return parts, per


@pytest.mark.parametrize("two,act,nparts", [(False, "silu", 1), (True, "relu", 1), (False, None, 2), (True, "silu", 2)])
def test_bn_act_train_forward_backward(two, act, nparts):
    lib = _lib.load()
    torch.manual_seed(3 + nparts)
    B, H, W, c = 4, 9, 7, 96
    rows = B * H * W
    z1 = (torch.randn(rows, c, device=DEV) * 2 + 3).requires_grad_(True)
    z2 = (torch.randn(rows, c, device=DEV) - 1).requires_grad_(True)
    g1, b1 = torch.randn(c, device=DEV).requires_grad_(True), torch.randn(c, device=DEV).requires_grad_(True)
    g2, b2 = torch.randn(c, device=DEV).requires_grad_(True), torch.randn(c, device=DEV).requires_grad_(True)
    rm1, rv1 = torch.randn(c, device=DEV), torch.rand(c, device=DEV) + 0.5
    rm1_ref, rv1_ref = rm1.clone(), rv1.clone()
    pre = F.batch_norm(z1, rm1_ref, rv1_ref, g1, b1, True, 0.1, 1e-5)
    if two:
        pre = pre + F.batch_norm(z2, None, None, g2, b2, True, 0.1, 1e-5)
    y_ref = _act(pre, act)
    dy = torch.randn_like(y_ref)
    y_ref.backward(dy)
    # forward on the kernels (SyncBN: per-part statistics combined)
    mr1, mr2 = torch.empty(2, c, device=DEV), torch.empty(2, c, device=DEV)
    parts, per = bn_stats(lib, z1.detach(), nparts)
    _lib.check(lib.dp_bn_finalize(parts.data_ptr(), nparts, float(per), c, 1e-5, 0.1, rm1.data_ptr(), rv1.data_ptr(),
                                  mr1.data_ptr(), _s()), "finalize")
    if two:
        parts2, _ = bn_stats(lib, z2.detach(), nparts)
        _lib.check(lib.dp_bn_finalize(parts2.data_ptr(), nparts, float(per), c, 1e-5, 0.1, None, None,
                                      mr2.data_ptr(), _s()), "finalize2")
    y = torch.empty(rows, c, device=DEV)
    zp2 = z2.detach() if two else None
    _lib.check(lib.dp_bn_act_fwd(y.data_ptr(), c, z1.detach().data_ptr(), c, mr1.data_ptr(), g1.detach().data_ptr(),
                                 b1.detach().data_ptr(), zp2.data_ptr() if two else None, c,
                                 mr2.data_ptr() if two else None, g2.detach().data_ptr() if two else None,
                                 b2.detach().data_ptr() if two else None, None, 0, rows, c, ACTS[act], DP_F32, _s()),
               "bn_act_fwd")
    torch.cuda.synchronize()
    _close(y, y_ref, f"bn fwd two={two} {act}")
    _close(rm1, rm1_ref, "running mean", 1e-5)
    _close(rv1, rv1_ref, "running var", 1e-5)
    # backward: reduce (+ the SyncBN all-reduce, here one rank) then apply
    sums = torch.empty(3, c, device=DEV)
    dg1, db1, dg2, db2 = (torch.zeros(c, device=DEV) for _ in range(4))
    _lib.check(lib.dp_bn_act_bwd_reduce(dy.data_ptr(), c, z1.detach().data_ptr(), c, mr1.data_ptr(),
                                        g1.detach().data_ptr(), b1.detach().data_ptr(),
                                        zp2.data_ptr() if two else None, c, mr2.data_ptr() if two else None,
                                        g2.detach().data_ptr() if two else None,
                                        b2.detach().data_ptr() if two else None, rows, c, ACTS[act], sums.data_ptr(),
                                        dg1.data_ptr(), db1.data_ptr(), dg2.data_ptr() if two else None,
                                        db2.data_ptr() if two else None, _rws(lib, rows, c).data_ptr(),
                                        int(lib.dp_bn_act_bwd_reduce_ws_bytes(rows, c)), DP_F32, _s()), "bn_bwd_reduce")
    dz1, dz2 = torch.empty(rows, c, device=DEV), torch.empty(rows, c, device=DEV)
    _lib.check(lib.dp_bn_act_bwd_apply(dz1.data_ptr(), c, dz2.data_ptr() if two else None, c, dy.data_ptr(), c,
                                       z1.detach().data_ptr(), c, mr1.data_ptr(), g1.detach().data_ptr(),
                                       b1.detach().data_ptr(), zp2.data_ptr() if two else None, c,
                                       mr2.data_ptr() if two else None, g2.detach().data_ptr() if two else None,
                                       b2.detach().data_ptr() if two else None, rows, c, ACTS[act], sums.data_ptr(),
                                       float(rows), DP_F32, _s()), "bn_bwd_apply")
    torch.cuda.synchronize()
    _close(dz1, z1.grad, "dz1")
    _close(dg1, g1.grad, "dgamma1")
    _close(db1, b1.grad, "dbeta1")
    if two:
        _close(dz2, z2.grad, "dz2")
        _close(dg2, g2.grad, "dgamma2")
        _close(db2, b2.grad, "dbeta2")


@pytest.mark.parametrize("two,act,c,res", [(False, "silu", 96, False), (True, "relu", 256, True),
                                            (True, "silu", 16, False), (False, None, 392, True)])
def test_bn_act_bf16_rows(two, act, c, res):
    """The BatchNorm row kernels on bf16 maps (the training tapes' dtype) against torch fp32
    autograd on the same bf16 values: statistics, forward (+ CSP residual) and the backward reduce
    / apply, ragged channel blocks included. bf16 outputs within 1e-2 of scale (their rounding),
    f32 sums and parameter gradients within 2e-4. (A 16-byte-vector form of these kernels
    measured no faster in the L b16 tapes and was not kept.)"""
    lib = _lib.load()
    torch.manual_seed(21 + c)
    B, H, W = 3, 11, 13
    rows = B * H * W
    bf = lambda t: t.bfloat16().float()
    z1 = bf(torch.randn(rows, c, device=DEV) * 2 + 3).requires_grad_(True)
    z2 = bf(torch.randn(rows, c, device=DEV) - 1).requires_grad_(True)
    rs = bf(torch.randn(rows, c, device=DEV))
    g1, b1 = torch.randn(c, device=DEV).requires_grad_(True), torch.randn(c, device=DEV).requires_grad_(True)
    g2, b2 = torch.randn(c, device=DEV).requires_grad_(True), torch.randn(c, device=DEV).requires_grad_(True)
    pre = F.batch_norm(z1, None, None, g1, b1, True, 0.1, 1e-5)
    if two:
        pre = pre + F.batch_norm(z2, None, None, g2, b2, True, 0.1, 1e-5)
    y_ref = _act(pre, act) + (rs if res else 0)
    dy = bf(torch.randn_like(y_ref))
    y_ref.backward(dy)
    # statistics as the tapes compute them (f32 over the bf16 maps)
    mr1, mr2 = torch.empty(2, c, device=DEV), torch.empty(2, c, device=DEV)
    zb1, zb2, rsb, dyb = (t.detach().bfloat16().contiguous() for t in (z1, z2, rs, dy))
    for zb, mr in ((zb1, mr1), (zb2, mr2)):
        parts = torch.zeros(1, 3, c, device=DEV)
        nb = int(lib.dp_bn_stats_ws_bytes(rows, c))
        ws = torch.empty(nb // 4, device=DEV)
        _lib.check(lib.dp_bn_stats(zb.data_ptr(), c, rows, c, parts.data_ptr(), ws.data_ptr(), nb, DP_BF16, _s()), "st")
        _lib.check(lib.dp_bn_finalize(parts.data_ptr(), 1, float(rows), c, 1e-5, 0.1, None, None, mr.data_ptr(), _s()),
                   "fin")
    y = torch.empty(rows, c, device=DEV, dtype=torch.bfloat16)
    _lib.check(lib.dp_bn_act_fwd(y.data_ptr(), c, zb1.data_ptr(), c, mr1.data_ptr(), g1.detach().data_ptr(),
                                 b1.detach().data_ptr(), zb2.data_ptr() if two else None, c,
                                 mr2.data_ptr() if two else None, g2.detach().data_ptr() if two else None,
                                 b2.detach().data_ptr() if two else None, rsb.data_ptr() if res else None, c, rows, c,
                                 ACTS[act], DP_BF16, _s()), "bn_act_fwd bf16")
    sums = torch.empty(3, c, device=DEV)
    dg1, db1, dg2, db2 = (torch.zeros(c, device=DEV) for _ in range(4))
    _lib.check(lib.dp_bn_act_bwd_reduce(dyb.data_ptr(), c, zb1.data_ptr(), c, mr1.data_ptr(), g1.detach().data_ptr(),
                                        b1.detach().data_ptr(), zb2.data_ptr() if two else None, c,
                                        mr2.data_ptr() if two else None, g2.detach().data_ptr() if two else None,
                                        b2.detach().data_ptr() if two else None, rows, c, ACTS[act], sums.data_ptr(),
                                        dg1.data_ptr(), db1.data_ptr(), dg2.data_ptr() if two else None,
                                        db2.data_ptr() if two else None, _rws(lib, rows, c).data_ptr(),
                                        int(lib.dp_bn_act_bwd_reduce_ws_bytes(rows, c)), DP_BF16, _s()), "reduce bf16")
    dz1, dz2 = (torch.empty(rows, c, device=DEV, dtype=torch.bfloat16) for _ in range(2))
    _lib.check(lib.dp_bn_act_bwd_apply(dz1.data_ptr(), c, dz2.data_ptr() if two else None, c, dyb.data_ptr(), c,
                                       zb1.data_ptr(), c, mr1.data_ptr(), g1.detach().data_ptr(), b1.detach().data_ptr(),
                                       zb2.data_ptr() if two else None, c, mr2.data_ptr() if two else None,
                                       g2.detach().data_ptr() if two else None, b2.detach().data_ptr() if two else None,
                                       rows, c, ACTS[act], sums.data_ptr(), float(rows), DP_BF16, _s()), "apply bf16")
    torch.cuda.synchronize()
    _close(y, y_ref, f"bn fwd bf16 c{c}", 1e-2)
    _close(dz1, z1.grad, "dz1 bf16", 1e-2)
    _close(dg1, g1.grad, "dgamma1 bf16")
    _close(db1, b1.grad, "dbeta1 bf16")
    if two:
        _close(dz2, z2.grad, "dz2 bf16", 1e-2)
        _close(dg2, g2.grad, "dgamma2 bf16")
        _close(db2, b2.grad, "dbeta2 bf16")


def _conv_desc(x, w_packed, kpad, cin, cout, h, w, k, out, res=None, B=2):
    d = ConvDesc()
    d.in_, d.in_bstride, d.in_pstride, d.in_h, d.in_w, d.cin = x.data_ptr(), h * w * cin, cin, h, w, cin
    d.weight, d.kpad, d.bias = w_packed.data_ptr(), kpad, None
    d.kh, d.kw, d.stride, d.pad_t, d.pad_l = k, k, 1, (k - 1) // 2, (k - 1) // 2
    d.out, d.out_bstride, d.out_pstride, d.out_h, d.out_w, d.cout = out.data_ptr(), h * w * cout, cout, h, w, cout
    if res is not None:
        d.res, d.res_bstride, d.res_pstride = res.data_ptr(), h * w * cout, cout
    d.batch, d.act, d.dtype = B, 0, DP_F32
    return d


@pytest.mark.parametrize("k,cin,cout", [(3, 64, 96), (1, 128, 64), (3, 32, 32)])
def test_conv_pack_forward_dgrad_wgrad(k, cin, cout):
    """Packed forward == F.conv2d; the 180-degree-rotated packing run as a conv of dz == the input
    gradient (accumulated through the residual input); im2col (cin, ky, kx) + dp_gemm == the
    weight gradient in the reference layout."""
    lib = _lib.load()
    torch.manual_seed(k * cin)
    B, h, w = 2, 11, 13
    wt = torch.randn(cout, cin, k, k, device=DEV) / (cin * k * k) ** 0.5
    x = torch.randn(B, cin, h, w, device=DEV).requires_grad_(True)
    wr = wt.clone().requires_grad_(True)
    y = F.conv2d(x, wr, None, 1, (k - 1) // 2)
    dy = torch.randn_like(y)
    y.backward(dy)
    xn = x.detach().permute(0, 2, 3, 1).contiguous()
    dyn = dy.permute(0, 2, 3, 1).contiguous()
    kpad = (k * k * cin + 31) // 32 * 32
    wp = torch.empty(cout, kpad, device=DEV)
    _lib.check(lib.dp_conv_pack(wt.data_ptr(), cout, cin, k, k, wp.data_ptr(), kpad, 0, 0, None, DP_F32, _s()), "pack")
    out = torch.empty(B, h, w, cout, device=DEV)
    d = _conv_desc(xn, wp, kpad, cin, cout, h, w, k, out)
    _lib.check(lib.dp_conv2d(C.byref(d), _s()), "fwd")
    torch.cuda.synchronize()
    _close(out, y.detach().permute(0, 2, 3, 1), f"conv{k} fwd")
    # input gradient: conv of dz with the rotated packing, accumulated onto a prior value
    kpad2 = (k * k * cout + 31) // 32 * 32
    wf = torch.empty(cin, kpad2, device=DEV)
    _lib.check(lib.dp_conv_pack(wt.data_ptr(), cout, cin, k, k, wf.data_ptr(), kpad2, 0, 1, None, DP_F32, _s()), "flip")
    prior = torch.randn(B, h, w, cin, device=DEV)
    dx = prior.clone()
    d2 = _conv_desc(dyn, wf, kpad2, cout, cin, h, w, k, dx, res=dx)
    _lib.check(lib.dp_conv2d(C.byref(d2), _s()), "dgrad")
    torch.cuda.synchronize()
    _close(dx, prior + x.grad.permute(0, 2, 3, 1), f"conv{k} dgrad")
    # weight gradient
    rows, K = B * h * w, cin * k * k
    col = torch.empty(rows, K, device=DEV)
    _lib.check(lib.dp_im2col(xn.data_ptr(), h * w * cin, cin, 1, B, h, w, cin, k, k, 1, (k - 1) // 2, h, w,
                             col.data_ptr(), DP_F32, DP_F32, _s()), "im2col")
    dW = torch.zeros(cout, K, device=DEV)
    g = GemmDesc()
    g.a, g.a_bs, g.a_rs, g.a_ks = dyn.data_ptr(), 0, 1, cout
    g.b, g.b_bs, g.b_ks, g.b_ns = col.data_ptr(), 0, K, 1
    g.c, g.c_bs, g.c_rs = dW.data_ptr(), 0, K
    g.batch, g.m, g.n, g.k = 1, cout, K, rows
    g.in_dtype, g.out_dtype = DP_F32, DP_F32
    g.alpha, g.beta = 1.0, 1.0
    _lib.check(lib.dp_gemm(C.byref(g), _s()), "wgrad")
    torch.cuda.synchronize()
    _close(dW.view(cout, cin, k, k), wr.grad, f"conv{k} wgrad")


@pytest.mark.parametrize("k,st,c", [(3, 2, 64), (5, 1, 96), (3, 1, 40), (5, 2, 68), (3, 2, 296)])
def test_depthwise_s2_backward_and_pack(k, st, c):
    """SCDown's depthwise 3x3 stride-2 conv (hybrid_encoder.py:156-170): dp_conv_pack mode 2 +
    dp_dwconv2d forward, dp_dwconv_bwd input and weight gradients vs autograd; also HGNetv2's 5x5 /
    3x3 stride-1 LightConvBNAct depthwise convs (hgnetv2.py:144-163), ragged channel blocks."""
    lib = _lib.load()
    torch.manual_seed(9)
    B, h, w = 2, 17, 12
    p = (k - 1) // 2
    wt = torch.randn(c, 1, k, k, device=DEV)
    x = torch.randn(B, c, h, w, device=DEV).requires_grad_(True)
    wr = wt.clone().requires_grad_(True)
    y = F.conv2d(x, wr, None, st, p, 1, c)
    dy = torch.randn_like(y)
    y.backward(dy)
    oh, ow = y.shape[2:]
    taps = torch.empty(k * k, c, device=DEV)
    _lib.check(lib.dp_conv_pack(wt.data_ptr(), c, 1, k, k, taps.data_ptr(), 0, 0, 2, None, DP_F32, _s()), "pack dw")
    xn = x.detach().permute(0, 2, 3, 1).contiguous()
    dyn = dy.permute(0, 2, 3, 1).contiguous()
    d = ConvDesc()
    out = torch.empty(B, oh, ow, c, device=DEV)
    d.in_, d.in_bstride, d.in_pstride, d.in_h, d.in_w, d.cin = xn.data_ptr(), h * w * c, c, h, w, c
    d.weight, d.kpad, d.bias = taps.data_ptr(), 0, None
    d.kh, d.kw, d.stride, d.pad_t, d.pad_l = k, k, st, p, p
    d.out, d.out_bstride, d.out_pstride, d.out_h, d.out_w, d.cout = out.data_ptr(), oh * ow * c, c, oh, ow, c
    d.batch, d.act, d.dtype = B, 0, DP_F32
    _lib.check(lib.dp_dwconv2d(C.byref(d), _s()), "dw fwd")
    dx = torch.zeros(B, h, w, c, device=DEV)
    dw = torch.zeros(c, k, k, device=DEV)
    _lib.check(lib.dp_dwconv_bwd(xn.data_ptr(), h * w * c, c, dyn.data_ptr(), oh * ow * c, c, taps.data_ptr(), B, h, w,
                                 c, k, st, p, oh, ow, dx.data_ptr(), h * w * c, c, dw.data_ptr(), DP_F32, _s()), "dw bwd")
    torch.cuda.synchronize()
    _close(out, y.detach().permute(0, 2, 3, 1), "dw fwd")
    _close(dx, x.grad.permute(0, 2, 3, 1), "dw dx")
    _close(dw, wr.grad.view(c, k, k), "dw dw")


@pytest.mark.parametrize("k,st,c", [(5, 1, 192), (3, 2, 384), (5, 2, 42), (3, 1, 36)])
def test_depthwise_backward_bf16(k, st, c):
    """dp_dwconv_bwd on bf16 maps (the training tapes' dtype): 4-channel vector lanes for the
    stride-2 convs when the channel rows allow it (c % 4 == 0), the scalar form otherwise (c = 42,
    the stride-1 convs), against autograd in fp32 on the
    same bf16 values; dx accumulates into a nonzero bf16 buffer (one bf16 rounding of the sum),
    dw in f32."""
    lib = _lib.load()
    torch.manual_seed(11)
    B, h, w = 2, 13, 21
    p = (k - 1) // 2
    wt = torch.randn(c, 1, k, k, device=DEV)
    x = torch.randn(B, c, h, w, device=DEV).bfloat16().float().requires_grad_(True)
    wr = wt.clone().requires_grad_(True)
    y = F.conv2d(x, wr, None, st, p, 1, c)
    dy = torch.randn_like(y).bfloat16().float()
    y.backward(dy)
    oh, ow = y.shape[2:]
    taps = wt.view(c, k * k).t().contiguous()          # [k*k][c] f32, dp_conv_pack mode 2's layout
    xn = x.detach().permute(0, 2, 3, 1).contiguous().bfloat16()
    dyn = dy.permute(0, 2, 3, 1).contiguous().bfloat16()
    dx0 = torch.randn(B, h, w, c, device=DEV).bfloat16()
    dx = dx0.clone()
    dw = torch.zeros(c, k, k, device=DEV)
    _lib.check(lib.dp_dwconv_bwd(xn.data_ptr(), h * w * c, c, dyn.data_ptr(), oh * ow * c, c, taps.data_ptr(), B, h, w,
                                 c, k, st, p, oh, ow, dx.data_ptr(), h * w * c, c, dw.data_ptr(), DP_BF16, _s()),
               "dw bwd bf16")
    torch.cuda.synchronize()
    ref_dx = dx0.float() + x.grad.permute(0, 2, 3, 1)
    err = float((dx.float() - ref_dx).abs().max())
    scale = float(ref_dx.abs().max())
    assert err <= 2 ** -7 * scale, ("dx", err, scale)       # one bf16 rounding of the sum
    _close(dw, wr.grad.view(c, k, k), "dw dw bf16")


def test_upsample_axpby_gelu_backward():
    lib = _lib.load()
    torch.manual_seed(2)
    B, h, w, c, ld = 2, 5, 6, 32, 80
    x = torch.randn(B, h, w, c, device=DEV)
    big = torch.zeros(B, 2 * h, 2 * w, ld, device=DEV)
    _lib.check(lib.dp_upsample2x(x.data_ptr(), h * w * c, c, B, h, w, c, big[..., 16:].data_ptr(), 4 * h * w * ld, ld,
                                 0, DP_F32, _s()), "up fwd")
    ref = F.interpolate(x.permute(0, 3, 1, 2), scale_factor=2.0, mode="nearest").permute(0, 2, 3, 1)
    torch.cuda.synchronize()
    _close(big[..., 16:16 + c], ref, "up fwd")
    dbig = torch.randn(B, 2 * h, 2 * w, c, device=DEV)
    dx = torch.ones(B, h, w, c, device=DEV)
    _lib.check(lib.dp_upsample2x(dbig.data_ptr(), 4 * h * w * c, c, B, h, w, c, dx.data_ptr(), h * w * c, c, 1, DP_F32,
                                 _s()), "up bwd")
    want = 1 + F.avg_pool2d(dbig.permute(0, 3, 1, 2), 2).permute(0, 2, 3, 1) * 4
    torch.cuda.synchronize()
    _close(dx, want, "up bwd")
    rows = B * h * w
    a, b = torch.randn(rows, c, device=DEV), torch.randn(rows, c, device=DEV)
    y = torch.randn(rows, c, device=DEV)
    y0 = y.clone()
    _lib.check(lib.dp_axpby_rows(y.data_ptr(), c, a.data_ptr(), c, 2.0, b.data_ptr(), c, -0.5, rows, c, 1, DP_F32, _s()),
               "axpby")
    torch.cuda.synchronize()
    _close(y, y0 + 2 * a - 0.5 * b, "axpby")
    pre = torch.randn(rows, c, device=DEV).requires_grad_(True)
    g = F.gelu(pre)
    dyy = torch.randn_like(g)
    g.backward(dyy)
    dxx = torch.empty(rows, c, device=DEV)
    _lib.check(lib.dp_act_bwd(pre.detach().data_ptr(), c, dyy.data_ptr(), c, dxx.data_ptr(), c, rows, c, _lib.DP_ACT_GELU, DP_F32,
                              _s()), "gelu bwd")
    torch.cuda.synchronize()
    _close(dxx, pre.grad, "gelu bwd")


@pytest.mark.parametrize("C_,nh", [(128, 8), (256, 8)])
def test_attention_400_tokens(C_, nh):
    """The AIFI self-attention core (400 tokens of a 20 x 20 map, hybrid_encoder.py:276-279):
    dp_attn_fwd / dp_attn_bwd vs autograd, q / k / v slices of one [rows][3C] buffer."""
    lib = _lib.load()
    torch.manual_seed(C_)
    B, L = 2, 400
    dh = C_ // nh
    qkv = torch.randn(B, L, 3 * C_, device=DEV)
    t = qkv.clone().requires_grad_(True)
    q, k, v = t.split(C_, -1)
    sh = lambda z: z.reshape(B, L, nh, dh).transpose(1, 2)   # noqa: E731
    o = (torch.softmax(sh(q) @ sh(k).transpose(-1, -2) / dh ** 0.5, -1) @ sh(v)).transpose(1, 2).reshape(B, L, C_)
    do = torch.randn_like(o)
    o.backward(do)
    out = torch.empty(B, L, C_, device=DEV)
    P = torch.empty(B * nh, L, L, device=DEV)
    base = qkv.data_ptr()
    _lib.check(lib.dp_attn_fwd(base, 3 * C_, base + 4 * C_, base + 8 * C_, 3 * C_, out.data_ptr(), C_, P.data_ptr(), None,
                               B, 1, L, 0, 1, L, nh, dh, DP_F32, _s()), "attn fwd")
    d = torch.zeros(B, L, 3 * C_, device=DEV)
    db = d.data_ptr()
    _lib.check(lib.dp_attn_bwd(base, 3 * C_, base + 4 * C_, base + 8 * C_, 3 * C_, P.data_ptr(), do.data_ptr(),
                               out.data_ptr(), C_, db,
                               3 * C_, db + 4 * C_, db + 8 * C_, 3 * C_, B, 1, L, 0, 1, L, nh, dh, DP_F32, _s()),
               "attn bwd")
    torch.cuda.synchronize()
    _close(out, o.detach(), "attn400 fwd")
    _close(d, t.grad, "attn400 bwd")


@pytest.mark.parametrize("B,h,w,cin,cout,k,st,pad,xpad", [(2, 17, 12, 48, 48, 3, 1, 1, 0), (2, 20, 20, 64, 130, 3, 2, 1, 8),
                                                         (3, 9, 13, 96, 96, 3, 1, 1, 16), (2, 10, 11, 16, 24, 2, 1, 0, 0),
                                                         # HGNetv2-L stage 0 at b16 (409,600 pixels: the gather's
                                                         # float-reciprocal pixel split far from small integers)
                                                         (16, 160, 160, 48, 48, 3, 1, 1, 0),
                                                         (5, 81, 79, 128, 128, 3, 1, 1, 0), (7, 61, 67, 32, 16, 3, 2, 1, 0)])
def test_conv_wgrad_implicit(B, h, w, cin, cout, k, st, pad, xpad):
    """dp_conv_wgrad (implicit-GEMM weight gradient, the training step's 3x3 / 2x2 convs) vs the
    fp32 autograd weight gradient on the same bf16-rounded x and dz; padded pixel strides, an
    M tile past cout, a stride-2 map, StemBlock's right/bottom-padded 2x2 (pad 0, output = input size)."""
    lib = _lib.load()
    torch.manual_seed(5)
    if k == 2:   # F.pad(x, (0, 1, 0, 1)) then a 2x2 valid conv: output h x w
        oh, ow = h, w
    else:
        oh, ow = (h + 2 * pad - k) // st + 1, (w + 2 * pad - k) // st + 1
    ps = cin + xpad
    x = torch.randn(B, h, w, ps, device=DEV).bfloat16()
    ldz = (cout + 7) // 8 * 8 + 8   # padded rows (16-byte aligned)
    dz = torch.randn(B * oh * ow, ldz, device=DEV).bfloat16()
    xr = x[..., :cin].float().permute(0, 3, 1, 2).contiguous()
    wr = torch.zeros(cout, cin, k, k, device=DEV, requires_grad=True)
    xin = F.pad(xr, (0, 1, 0, 1)) if k == 2 else xr
    y = F.conv2d(xin, wr, None, st, 0 if k == 2 else pad)
    assert y.shape[2:] == (oh, ow)
    y.backward(dz[:, :cout].float().view(B, oh, ow, cout).permute(0, 3, 1, 2))
    dw = torch.full((cout, cin, k, k), 0.5, device=DEV)   # accumulates
    scratch = torch.empty(cout * cin * k * k, device=DEV)
    _lib.check(lib.dp_conv_wgrad(x.data_ptr(), h * w * ps, ps, B, h, w, cin, dz.data_ptr(), ldz, oh, ow, cout, k,
                                 k, st, pad, scratch.data_ptr(), dw.data_ptr(), DP_BF16, _s()), "conv_wgrad")
    torch.cuda.synchronize()
    ref = wr.grad + 0.5
    err = (dw - ref).abs().max().item() / ref.abs().max().item()
    assert err < 2e-3, err
    # dp_conv_wgrad_zs: a zeroed scratch, left zeroed by each call (so two calls in a row accumulate
    # exactly twice the gradient with no zero-fill between them)
    dw2 = torch.full((cout, cin, k, k), 0.5, device=DEV)
    scratch2 = torch.zeros(cout * cin * k * k, device=DEV)
    for _ in range(2):
        _lib.check(lib.dp_conv_wgrad_zs(x.data_ptr(), h * w * ps, ps, B, h, w, cin, dz.data_ptr(), ldz, oh, ow, cout,
                                        k, k, st, pad, scratch2.data_ptr(), dw2.data_ptr(), DP_BF16, _s()), "zs")
    torch.cuda.synchronize()
    ref2 = 2 * wr.grad + 0.5
    err2 = (dw2 - ref2).abs().max().item() / ref2.abs().max().item()
    assert err2 < 2e-3 and int(scratch2.count_nonzero()) == 0, (err2, int(scratch2.count_nonzero()))


@pytest.mark.parametrize("rows,c,dt", [(6400, 256, DP_BF16), (1000, 96, DP_F32), (409600, 64, DP_BF16)])
def test_bn_stats_finalize_fused_equals_two_launch(rows, c, dt):
    """dp_bn_stats_finalize (the one-rank BatchNorm statistics with the finalize in the same
    launches) equals dp_bn_stats then dp_bn_finalize BIT FOR BIT: parts, (mean, rstd), running
    statistics."""
    lib = _lib.load()
    torch.manual_seed(rows + c)
    z = (torch.randn(rows, c, device=DEV) * 2 + 0.5).to(torch.bfloat16 if dt == DP_BF16 else torch.float32)
    nb = int(lib.dp_bn_stats_ws_bytes(rows, c))
    ws = torch.empty(nb // 4, device=DEV)
    outs = []
    for fused in (False, True):
        parts, mr = torch.zeros(3, c, device=DEV), torch.empty(2, c, device=DEV)
        rm, rv = torch.linspace(-1, 1, c, device=DEV), torch.linspace(0.5, 2, c, device=DEV)
        if fused:
            _lib.check(lib.dp_bn_stats_finalize(z.data_ptr(), c, rows, c, parts.data_ptr(), ws.data_ptr(), nb, 1e-5, 0.1,
                                                rm.data_ptr(), rv.data_ptr(), mr.data_ptr(), dt, _s()), "stats+fin")
        else:
            _lib.check(lib.dp_bn_stats(z.data_ptr(), c, rows, c, parts.data_ptr(), ws.data_ptr(), nb, dt, _s()), "st")
            _lib.check(lib.dp_bn_finalize(parts.data_ptr(), 1, float(rows), c, 1e-5, 0.1, rm.data_ptr(), rv.data_ptr(),
                                          mr.data_ptr(), _s()), "fin")
        torch.cuda.synchronize()
        outs.append((parts, mr, rm, rv))
    for a, b in zip(*outs):
        assert torch.equal(a, b)


def test_conv_wgrad_more_than_2p24_pixels():
    """dp_conv_wgrad past 2^24 output pixels (its gather's float-reciprocal split is exact below
    2^24): the batch runs as image chunks accumulating into one scratch. 4100 images of 64 x 64
    (16.8 M pixels, two chunks) vs the fp32 autograd weight gradient."""
    lib = _lib.load()
    torch.manual_seed(9)
    B, h, w, cin, cout, k = 4100, 64, 64, 8, 16, 3
    assert B * h * w >= 1 << 24
    x = torch.randn(B, h, w, cin, device=DEV).bfloat16()
    dz = torch.randn(B * h * w, cout, device=DEV).bfloat16()
    with torch.backends.cudnn.flags(enabled=True, allow_tf32=False):
        ref = torch.nn.grad.conv2d_weight(x.float().permute(0, 3, 1, 2), (cout, cin, k, k),
                                          dz.float().view(B, h, w, cout).permute(0, 3, 1, 2), 1, 1)
    dw = torch.zeros(cout, cin, k, k, device=DEV)
    scratch = torch.empty(cout * cin * k * k, device=DEV)
    _lib.check(lib.dp_conv_wgrad(x.data_ptr(), h * w * cin, cin, B, h, w, cin, dz.data_ptr(), cout, h, w, cout, k, k,
                                 1, 1, scratch.data_ptr(), dw.data_ptr(), DP_BF16, _s()), "conv_wgrad 2^24")
    torch.cuda.synchronize()
    err = (dw - ref).abs().max().item() / ref.abs().max().item()
    assert err < 2e-3, err
