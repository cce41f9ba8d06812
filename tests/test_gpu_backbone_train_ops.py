"""The backbone training kernels (csrc/backbone_train.hip) through the C ABI vs torch fp32
autograd of the same ops: ConvBNAct's epilogue backward (FrozenBatchNorm2d scale, ReLU,
LearnableAffineBlock and its scalar gradients), the strided dense conv's input gradient as
col2im, and the StemBlock max-pool backward with ties (hgnetv2.py:24-79, 129-134, 210-220).
fp32 bound: 2e-4 of the output scale."""
import ctypes as C

import pytest
import torch
import torch.nn.functional as F

from detrpose_amd import _lib
from detrpose_amd._lib import DP_BF16, DP_F32

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _s():
    return C.c_void_p(torch.cuda.current_stream().cuda_stream)


def _close(got, ref, what, tol=2e-4):
    got, ref = got.float().cpu(), ref.float().cpu()
    scale = max(1.0, float(ref.abs().max()))
    err = float((got - ref).abs().max())
    print(f"{what}: max err {err:.3g} (scale {scale:.3g})")
    assert err <= tol * scale, (what, err, scale)


@pytest.mark.parametrize("lab,dtype,bres", [(False, DP_F32, False), (True, DP_F32, False), (True, DP_BF16, False),
                                           (False, DP_BF16, False), (False, DP_BF16, True)])
def test_frozen_act_bwd(lab, dtype, bres):
    """FrozenBatchNorm2d + ReLU (+ LAB, + the HG block's identity) backward; bf16 without LAB runs
    the 16-byte channel-vector kernel."""
    lib = _lib.load()
    torch.manual_seed(5)
    rows, c = 3000, 48
    td = torch.float32 if dtype == DP_F32 else torch.bfloat16
    u = torch.randn(rows, c, device=DEV).requires_grad_(True)
    a = torch.tensor([0.7], device=DEV, requires_grad=True)
    cb = torch.tensor([0.3], device=DEV, requires_grad=True)
    s = torch.rand(c, device=DEV) + 0.5
    r = F.relu(u)
    y = a * r + cb if lab else r
    dy = torch.randn(rows, c, device=DEV)
    y.backward(dy)
    yd, dyd = y.detach().to(td), dy.to(td)
    dz = torch.empty(rows, c, device=DEV, dtype=td)
    dl = torch.zeros(2, device=DEV)
    res = torch.randn(rows, c, device=DEV).to(td)   # an HG-block identity added after the act
    use_res = dtype == DP_F32 or bres
    yd = (yd.float() + res.float()).to(td) if use_res else yd
    _lib.check(lib.dp_frozen_act_bwd(yd.data_ptr(), c, res.data_ptr() if use_res else None, c, dyd.data_ptr(),
                                     c, dz.data_ptr(), c, rows, c, _lib.DP_ACT_RELU,
                                     a.detach().data_ptr() if lab else None, cb.detach().data_ptr() if lab else None,
                                     s.data_ptr(), dl.data_ptr() if lab else None, dl.data_ptr() + 4 if lab else None,
                                     dtype, _s()), "frozen_act_bwd")
    torch.cuda.synchronize()
    want = u.grad * s   # d conv-output = d u * s (u = s z + b)
    if dtype == DP_F32:
        # y + res - res is y only up to rounding: units with a r below ~1e-6 may flip
        err = (dz - want).abs()
        bad = err > 2e-4 * float(want.abs().max())
        assert not bad.any() or float(u.detach().abs()[bad].max()) < 1e-5, float(u.detach().abs()[bad].max())
    else:
        # bf16 storage of y = a r + cb cannot tell r > 0 from r == 0 within cb's rounding: the
        # ReLU mask may differ only there (|u| within a few bf16 ulps of cb / a)
        # (with the identity added: within y + res's rounding, a few bf16 ulps of |res|)
        err = (dz.float() - want).abs()
        bad = err > 1e-2 * float(want.abs().max())
        print(f"bf16 lab={lab} res={bres}: {int(bad.sum())} of {bad.numel()} differ, max |u| there "
              f"{float(u.detach().abs()[bad].max()) if bad.any() else 0.0:.3g}")
        umax = 0.05 if bres else 0.01
        assert bad.float().mean() < 1e-2 and (not bad.any() or float(u.detach().abs()[bad].max()) < umax)
    if lab:
        _close(dl[0], a.grad[0], "d lab.scale", 1e-4 if dtype == DP_F32 else 2e-2)
        _close(dl[1], cb.grad[0], "d lab.bias", 1e-4 if dtype == DP_F32 else 2e-2)


@pytest.mark.parametrize("bf16,cin", [(False, 32), (False, 30), (True, 64), (True, 36)])
def test_col2im_strided_dgrad(bf16, cin):
    """StemBlock.stem3 (3x3, stride 2, pad 1): dx = col2im(dz W) == F.conv2d's input gradient;
    16-byte channel vectors when cin allows (32 f32, 64 bf16), the scalar form otherwise."""
    lib = _lib.load()
    torch.manual_seed(6)
    B, cout, h, w = 2, 24, 17, 22
    x = torch.randn(B, cin, h, w, device=DEV).requires_grad_(True)
    wt = torch.randn(cout, cin, 3, 3, device=DEV)
    y = F.conv2d(x, wt, None, 2, 1)
    dy = torch.randn_like(y)
    y.backward(dy)
    oh, ow = y.shape[2:]
    # columns tap-major (ky, kx, ci), the order dp_conv_pack mode 4 packs W^T in
    dcol = dy.permute(0, 2, 3, 1).reshape(-1, cout) @ wt.permute(0, 2, 3, 1).reshape(cout, -1)
    if bf16:
        dcol = dcol.bfloat16()
        dx = torch.ones(B, h, w, cin, device=DEV, dtype=torch.bfloat16)
        _lib.check(lib.dp_col2im(dcol.contiguous().data_ptr(), B, h, w, cin, 3, 3, 2, 1, oh, ow, dx.data_ptr(),
                                 h * w * cin, cin, 1, DP_BF16, _s()), "col2im bf16")
        torch.cuda.synchronize()
        # reference from the same bf16 columns, summed in f32, one bf16 rounding
        ref = torch.ones(B, h, w, cin, device=DEV)
        dc = dcol.float().reshape(B, oh, ow, 3, 3, cin)
        for ky in range(3):
            for kx in range(3):
                for oy in range(oh):
                    y_ = 2 * oy - 1 + ky
                    if 0 <= y_ < h:
                        xs = [2 * ox - 1 + kx for ox in range(ow)]
                        ok = [i for i, x_ in enumerate(xs) if 0 <= x_ < w]
                        ref[:, y_, [xs[i] for i in ok]] += dc[:, oy, ok, ky, kx]
        err = float((dx.float() - ref).abs().max())
        assert err <= 2 ** -7 * float(ref.abs().max()), err
        return
    dx = torch.ones(B, h, w, cin, device=DEV)
    _lib.check(lib.dp_col2im(dcol.contiguous().data_ptr(), B, h, w, cin, 3, 3, 2, 1, oh, ow, dx.data_ptr(), h * w * cin,
                             cin, 1, DP_F32, _s()), "col2im")
    torch.cuda.synchronize()
    _close(dx, 1 + x.grad.permute(0, 2, 3, 1), "col2im dx")
    # the W^T that produces these columns on the 1x1 conv kernel: dp_conv_pack mode 4
    kpad = 64
    wp = torch.full((9 * cin, kpad), 7.0, device=DEV)
    _lib.check(lib.dp_conv_pack(C.c_void_p(wt.data_ptr()), cout, cin, 3, 3, C.c_void_p(wp.data_ptr()), kpad, 0, 4,
                                None, DP_F32, _s()), "conv_pack mode 4")
    torch.cuda.synchronize()
    ref = torch.zeros(9 * cin, kpad, device=DEV)
    ref[:, :cout] = wt.permute(0, 2, 3, 1).reshape(cout, -1).t()
    assert torch.equal(wp, ref)


@pytest.mark.parametrize("dtype,c", [(DP_F32, 16), (DP_BF16, 16), (DP_BF16, 12), (DP_F32, 6)])
def test_maxpool_pad_rb_bwd_with_ties(dtype, c):
    """F.pad(0,1,0,1) + MaxPool2d(2, 1, ceil_mode=True) backward, ReLU'd input (many tied zeros,
    the pad zeros included); 16-byte channel vectors (c = 16) and the one-channel form."""
    lib = _lib.load()
    torch.manual_seed(7)
    td = torch.float32 if dtype == DP_F32 else torch.bfloat16
    B, h, w = 2, 13, 11
    x = F.relu(torch.randn(B, c, h, w, device=DEV)).to(td).float().requires_grad_(True)
    y = F.max_pool2d(F.pad(x, (0, 1, 0, 1)), 2, 1, ceil_mode=True)
    dy = torch.randn_like(y)
    y.backward(dy)
    xn = x.detach().permute(0, 2, 3, 1).contiguous().to(td)
    dyn = dy.permute(0, 2, 3, 1).contiguous().to(td)
    dx = torch.zeros(B, h, w, c, device=DEV, dtype=td)
    _lib.check(lib.dp_maxpool2x2_pad_rb_bwd(xn.data_ptr(), h * w * c, c, dyn.data_ptr(), h * w * c, c, B, h, w, c,
                                            dx.data_ptr(), h * w * c, c, dtype, _s()), "maxpool bwd")
    torch.cuda.synchronize()
    ref = F.max_pool2d(F.pad(x.detach(), (0, 1, 0, 1)), 2, 1, ceil_mode=True)
    assert ref.shape == y.shape
    # dy is rounded to dtype before the kernel: compare against autograd of the rounded dy
    x2 = x.detach().clone().requires_grad_(True)
    F.max_pool2d(F.pad(x2, (0, 1, 0, 1)), 2, 1, ceil_mode=True).backward(dy.to(td).float())
    _close(dx, x2.grad.permute(0, 2, 3, 1), "maxpool dx", 2e-4 if dtype == DP_F32 else 1e-2)


def test_conv_pack_scaled_and_stem_layout():
    """dp_conv_pack with the frozen-BN scale: mode 0 rows and mode 3 (dp_stem_conv's f32 OIHW)."""
    lib = _lib.load()
    torch.manual_seed(8)
    cout, cin = 16, 3
    wt = torch.randn(cout, cin, 3, 3, device=DEV)
    s = torch.rand(cout, device=DEV) + 0.5
    o3 = torch.empty(cout, 27, device=DEV)
    _lib.check(lib.dp_conv_pack(wt.data_ptr(), cout, cin, 3, 3, o3.data_ptr(), 0, 0, 3, s.data_ptr(), DP_F32, _s()), "m3")
    kpad = 64
    o0 = torch.zeros(cout, kpad, device=DEV)
    _lib.check(lib.dp_conv_pack(wt.data_ptr(), cout, cin, 3, 3, o0.data_ptr(), kpad, 4, 0, s.data_ptr(), DP_F32, _s()),
               "m0 kc=4")
    torch.cuda.synchronize()
    ws = wt * s[:, None, None, None]
    _close(o3, ws.reshape(cout, 27), "mode 3")
    want = torch.zeros(cout, 3, 3, 4, device=DEV)
    want[..., :3] = ws.permute(0, 2, 3, 1)
    _close(o0[:, :36], want.reshape(cout, 36), "mode 0 padded")
    assert float(o0[:, 36:].abs().max()) == 0.0
