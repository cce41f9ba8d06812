"""Per-kernel parity: each C-ABI entry point vs a plain fp32 reference of the same op
(torch CPU fp32 ops or the oracle restatement), fp32 and bf16 storage modes.
Tolerances: fp32 2e-4 of the output scale. bf16: the reference runs on the SAME bf16-rounded
inputs and weights the kernel reads, with the kernel's internal bf16 store points emulated
(e.g. the attention probabilities), so the only differences left are f32 summation order and
the one rounding of the output: one bf16 ulp at the output scale max(1, max|ref|)."""
import ctypes as C
import math
import os

import numpy as np
import pytest
import torch
import torch.nn.functional as F

from detrpose_amd import _lib
from detrpose_amd._lib import ConvDesc, contiguous_rows, rowmap
from detrpose_amd.engine import DTYPES, Packer
from oracle import detrpose_cpu as O

pytestmark = pytest.mark.gpu
DT = ["fp32", "bf16"]
TOL = {"fp32": 2e-4}
_KEEP = []


@pytest.fixture(autouse=True)
def _keepalive():
    yield
    torch.cuda.synchronize()
    _KEEP.clear()


def _s():
    return C.c_void_p(torch.cuda.current_stream().cuda_stream)


def _d(x, dtype=None):
    """Device copy kept alive until the test ends (kernels run asynchronously)."""
    t = (x.to("cuda", dtype) if dtype is not None else x.cuda()).contiguous()
    _KEEP.append(t)
    return t.data_ptr()


def _close(got, ref, dt, what=""):
    """fp32: 2e-4 of max(1, max|ref|); bf16: one bf16 ulp at the output scale, i.e. 2^-7 times
    the power of two at or below max(1, max|ref|) (twice the output's own rounding error)."""
    got = got.float().cpu()
    ref = ref.float().cpu()
    scale = max(1.0, ref.abs().max().item())
    tol = TOL[dt] * scale if dt == "fp32" else 2.0 ** (math.floor(math.log2(scale)) - 7)
    err = (got - ref).abs().max().item()
    print(f"{what} [{dt}]: max err {err:.3g} = {err / tol:.3g} of the bound (scale {scale:.3g})")
    assert err <= tol, f"{what}: max err {err:.3g} > {tol:.3g} (scale {scale:.3g}, dtype {dt})"


def _rb(t, dt):
    """t as the kernel reads it: bf16-rounded in bf16 mode."""
    return t.bfloat16().float() if dt == "bf16" else t


def _nhwc(x, dt):
    t = x.permute(0, 2, 3, 1).contiguous().to("cuda", DTYPES[dt][0])
    _KEEP.append(t)
    return t


def _run_conv(pc, x_nhwc, out, dt, res=None, up=None):
    lib = _lib.load()
    B, H, W, Cin = x_nhwc.shape
    d = ConvDesc()
    d.in_, d.in_bstride, d.in_pstride, d.in_h, d.in_w, d.cin = x_nhwc.data_ptr(), H * W * Cin, Cin, H, W, Cin
    d.weight, d.kpad, d.bias = pc.w.data_ptr(), pc.kpad, pc.b.data_ptr()
    d.kh, d.kw, d.stride, d.pad_t, d.pad_l = pc.kh, pc.kw, pc.stride, pc.pad, pc.pad
    _, Ho, Wo, Co = out.shape
    d.out, d.out_bstride, d.out_pstride, d.out_h, d.out_w, d.cout = out.data_ptr(), Ho * Wo * Co, Co, Ho, Wo, Co
    if res is not None:
        d.res, d.res_bstride, d.res_pstride = res.data_ptr(), Ho * Wo * Co, Co
    if up is not None:
        d.up, d.up_bstride, d.up_pstride = up.data_ptr(), 4 * Ho * Wo * Co, Co
    d.batch, d.act, d.dtype = B, pc.act, DTYPES[dt][1]
    if pc.lab:
        d.has_lab, d.lab_scale, d.lab_bias = 1, pc.lab[0], pc.lab[1]
    fn = lib.dp_dwconv2d if pc.depthwise else lib.dp_conv2d
    _lib.check(fn(C.byref(d), _s()), "conv")


@pytest.mark.parametrize("dt", DT)
@pytest.mark.parametrize("k,s,cin,cout,H,act", [
    (1, 1, 64, 96, 13, "relu"), (3, 1, 48, 48, 17, "silu"), (3, 2, 64, 32, 20, None), (1, 1, 336, 64, 9, "relu"),
    (3, 1, 24, 24, 11, "silu"), (1, 1, 256, 288, 7, None), (3, 1, 128, 128, 40, "gelu"),
    # 128x128 tiles with an N tail, and grids where each persistent block walks several tiles
    (3, 1, 64, 160, 70, "silu"), (1, 1, 64, 128, 200, "relu"), (3, 1, 32, 64, 256, None),
    (1, 1, 96, 32, 256, "gelu"),
    # 8-wave 192x256 / 256x256 / 256x128 tiles (M >= 32768; 192 vs 256 rows by round
    # quantization): N tails, 3x3 gather, 1x1
    (1, 1, 256, 320, 130, "relu"), (1, 1, 128, 288, 200, "silu"), (3, 1, 64, 96, 130, "silu"),
    (1, 1, 512, 128, 128, None),
    # LDS halo-tile path (3x3 / 2x2, cout <= 128): streamed weights with 2 / 1.5 channel
    # planes, resident weights, stride 2 with 64 outputs, ragged tile edges
    (3, 1, 128, 128, 37, "silu"), (3, 1, 96, 96, 33, "relu"), (3, 1, 48, 48, 50, "relu"), (3, 2, 64, 64, 45, None),
    (2, 1, 16, 32, 29, "relu"), (3, 1, 256, 64, 21, "silu"),
    # the 128-wide halo tile with its last 16-byte channel chunks partly / wholly past cout
    (3, 1, 64, 112, 23, "relu"), (3, 1, 96, 100, 19, None)])
def test_conv2d(dt, k, s, cin, cout, H, act):
    torch.manual_seed(k * 100 + cin)
    pk = Packer({}, dt, torch.device("cuda"))
    x = torch.randn(2, cin, H, H + 3)
    w = torch.randn(cout, cin, k, k) / (cin * k * k) ** 0.5
    b = torch.randn(cout) * 0.1
    pc = pk.conv(w.double(), b.double(), stride=s, act=act)
    ref = F.conv2d(_rb(x, dt), _rb(w, dt), b, s, (k - 1) // 2)
    ref = {"relu": F.relu, "silu": F.silu, "gelu": F.gelu, None: lambda t: t}[act](ref)
    out = torch.empty(2, ref.shape[2], ref.shape[3], pc.cout, device="cuda", dtype=DTYPES[dt][0])
    resid = _rb(torch.randn(2, ref.shape[2], ref.shape[3], pc.cout), dt)
    rd = resid.to("cuda", DTYPES[dt][0])
    _run_conv(pc, _nhwc(x, dt), out, dt, res=rd)
    torch.cuda.synchronize()
    _close(out[..., :cout], ref.permute(0, 2, 3, 1) + resid[..., :cout], dt, f"conv k{k}s{s} {cin}->{cout}")


@pytest.mark.parametrize("seg,nseg,cout,H,W", [(48, 7, 64, 64, 67), (16, 7, 32, 40, 41), (64, 7, 64, 30, 33)])
def test_conv2d_1x1_segmented_input(seg, nseg, cout, H, W):
    """The squeeze conv over an HG-block concat stored as one contiguous map per member
    (dp_conv_desc.in_seg_ch / in_seg_stride; segments not adjacent in memory) vs torch fp32 on
    the concatenated channels."""
    torch.manual_seed(seg + H)
    B, cin = 2, seg * nseg
    pk = Packer({}, "bf16", torch.device("cuda"))
    x = torch.randn(B, cin, H, W).bfloat16().float()
    w = torch.randn(cout, cin, 1, 1) / cin ** 0.5
    b = torch.randn(cout) * 0.1
    pc = pk.conv(w.double(), b.double(), act="relu")
    ref = F.relu(F.conv2d(x, _rb(w, "bf16"), b)).permute(0, 2, 3, 1)
    gap = 4096                                       # elements between one segment's end and the next
    sel = B * H * W * seg
    arena = torch.zeros(nseg * (sel + gap), device="cuda", dtype=torch.bfloat16)
    for i in range(nseg):
        arena[i * (sel + gap):i * (sel + gap) + sel] = \
            x[:, i * seg:(i + 1) * seg].permute(0, 2, 3, 1).reshape(-1).to("cuda", torch.bfloat16)
    _KEEP.append(arena)
    out = torch.empty(B, H, W, cout, device="cuda", dtype=torch.bfloat16)
    d = ConvDesc()
    d.in_, d.in_bstride, d.in_pstride, d.in_h, d.in_w, d.cin = arena.data_ptr(), H * W * seg, seg, H, W, cin
    d.weight, d.kpad, d.bias = pc.w.data_ptr(), pc.kpad, pc.b.data_ptr()
    d.kh, d.kw, d.stride = 1, 1, 1
    d.out, d.out_bstride, d.out_pstride, d.out_h, d.out_w, d.cout = out.data_ptr(), H * W * cout, cout, H, W, cout
    d.batch, d.act, d.dtype = B, pc.act, _lib.DP_BF16
    d.in_seg_ch, d.in_seg_stride = seg, sel + gap
    _lib.check(_lib.load().dp_conv2d(C.byref(d), _s()), "conv 1x1 segmented")
    torch.cuda.synchronize()
    _close(out, ref, "bf16", f"1x1 segmented {seg}x{nseg}->{cout}")


@pytest.mark.parametrize("cin,cout,H,W,ld,off,mode,act", [
    (336, 64, 64, 67, 400, 32, "plain", "relu"),    # K tail (kpad 384), input = concat slice
    (512, 256, 48, 47, 512, 0, "up", "silu"),       # nearest-x2 epilogue
    (256, 256, 70, 71, 256, 0, "f32", None),        # f32 output (linear heads)
    (576, 192, 40, 43, 640, 64, "res", "gelu"),     # N tail, residual
    (64, 48, 130, 129, 64, 0, "plain", "relu")])    # narrow cout (48 of a 64 tile)
def test_conv2d_1x1_large_m(cin, cout, H, W, ld, off, mode, act):
    """1x1 convs at M >= 16K (the persistent conv_stream tiles) with every epilogue mode
    (plain, nearest-x2 copy, f32 output, residual), K / M / cout tails and input rows that are
    a channel slice of a wider concat buffer, vs torch fp32 on the same bf16-rounded operands."""
    torch.manual_seed(cin + cout + H)
    B = 2
    pk = Packer({}, "bf16", torch.device("cuda"))
    x = torch.randn(B, cin, H, W).bfloat16().float()
    w = torch.randn(cout, cin, 1, 1) / cin ** 0.5
    b = torch.randn(cout) * 0.1
    pc = pk.conv(w.double(), b.double(), act=act)
    ref = {"relu": F.relu, "silu": F.silu, "gelu": F.gelu, None: lambda t: t}[act](F.conv2d(x, _rb(w, "bf16"), b))
    wide = torch.zeros(B, H, W, ld, device="cuda", dtype=torch.bfloat16)
    wide[..., off:off + cin] = x.permute(0, 2, 3, 1).to("cuda", torch.bfloat16)
    _KEEP.append(wide)
    odt = torch.float32 if mode == "f32" else torch.bfloat16
    out = torch.empty(B, H, W, cout, device="cuda", dtype=odt)
    d = ConvDesc()
    d.in_, d.in_bstride, d.in_pstride, d.in_h, d.in_w, d.cin = wide.data_ptr() + 2 * off, H * W * ld, ld, H, W, cin
    d.weight, d.kpad, d.bias = pc.w.data_ptr(), pc.kpad, pc.b.data_ptr()
    d.kh, d.kw, d.stride = 1, 1, 1
    d.out, d.out_bstride, d.out_pstride, d.out_h, d.out_w, d.cout = out.data_ptr(), H * W * cout, cout, H, W, cout
    d.batch, d.act, d.dtype = B, pc.act, _lib.DP_BF16
    d.out_f32 = 1 if mode == "f32" else 0
    want = ref.permute(0, 2, 3, 1)
    if mode == "res":
        r = torch.randn(B, H, W, cout).bfloat16()
        rd = r.to("cuda")
        _KEEP.append(rd)
        d.res, d.res_bstride, d.res_pstride = rd.data_ptr(), H * W * cout, cout
        want = want + r.float()
    if mode == "up":
        up = torch.empty(B, 2 * H, 2 * W, cout, device="cuda", dtype=torch.bfloat16)
        d.up, d.up_bstride, d.up_pstride = up.data_ptr(), 4 * H * W * cout, cout
    _lib.check(_lib.load().dp_conv2d(C.byref(d), _s()), "conv 1x1")
    torch.cuda.synchronize()
    _close(out, want, "bf16", f"1x1 {cin}->{cout} {mode}")
    if mode == "up":
        _close(up, F.interpolate(ref, scale_factor=2.0, mode="nearest").permute(0, 2, 3, 1), "bf16", "1x1 up")


@pytest.mark.parametrize("B,cin,cout,H,W,act", [
    (64, 128, 128, 80, 80, "silu"), (16, 128, 128, 40, 40, "silu"), (8, 128, 128, 20, 20, None),
    (4, 128, 128, 64, 70, "relu"), (16, 64, 64, 40, 40, "relu"), (8, 96, 96, 33, 35, "silu")])
def test_conv2d_halo_streamed_plain(B, cin, cout, H, W, act):
    """The streamed-weight halo tiles as the encoder runs them: no residual, every output channel
    present, so a block's next tile starts on the counted vmcnt waits that leave the previous
    tile's epilogue stores in flight (the pipelined K loop's per-step counts included); batches
    with several tiles per persistent block (L b64 80x80: 1600 tiles), ragged edges."""
    torch.manual_seed(B * H + cin)
    pk = Packer({}, "bf16", torch.device("cuda"))
    x = torch.randn(B, cin, H, W).bfloat16().float()
    w = torch.randn(cout, cin, 3, 3) / (cin * 9) ** 0.5
    b = torch.randn(cout) * 0.1
    pc = pk.conv(w.double(), b.double(), act=act)
    with torch.backends.cudnn.flags(enabled=True, allow_tf32=False):   # fp32 reference, no xf32
        ref = F.conv2d(x.cuda(), _rb(w, "bf16").cuda(), b.cuda(), 1, 1)
    ref = {"relu": F.relu, "silu": F.silu, None: lambda t: t}[act](ref)
    out = torch.full((B, H, W, cout), 7.0, device="cuda", dtype=torch.bfloat16)
    _run_conv(pc, _nhwc(x, "bf16"), out, "bf16")
    torch.cuda.synchronize()
    _close(out, ref.permute(0, 2, 3, 1), "bf16", f"halo {cin}->{cout} {H}x{W} b{B}")


@pytest.mark.parametrize("H,W,act", [(50, 53, "relu"), (160, 160, "silu"), (17, 9, None)])
def test_conv2d_halo_48(H, W, act):
    """The 48-wide natural-order halo tile (HG stage-0 3x3 48->48 convs, no residual) writing a
    channel slice of a wider concat buffer, as the HG_Block layers do; ragged 16x16 tiles and
    the model's 160x160 map."""
    torch.manual_seed(H * W)
    pk = Packer({}, "bf16", torch.device("cuda"))
    B, cin, cout, ld = 2, 48, 48, 336
    x = torch.randn(B, cin, H, W).bfloat16().float()
    w = torch.randn(cout, cin, 3, 3) / (cin * 9) ** 0.5
    b = torch.randn(cout) * 0.1
    pc = pk.conv(w.double(), b.double(), act=act)
    ref = {"relu": F.relu, "silu": F.silu, None: lambda t: t}[act](F.conv2d(x, _rb(w, "bf16"), b, 1, 1))
    wide = torch.full((B, H, W, ld), 3.0, device="cuda", dtype=torch.bfloat16)
    xi = _nhwc(x, "bf16")
    d = ConvDesc()
    d.in_, d.in_bstride, d.in_pstride, d.in_h, d.in_w, d.cin = xi.data_ptr(), H * W * cin, cin, H, W, cin
    d.weight, d.kpad, d.bias = pc.w.data_ptr(), pc.kpad, pc.b.data_ptr()
    d.kh, d.kw, d.stride, d.pad_t, d.pad_l = 3, 3, 1, 1, 1
    d.out, d.out_bstride, d.out_pstride = wide.data_ptr() + 2 * 96, H * W * ld, ld
    d.out_h, d.out_w, d.cout = H, W, cout
    d.batch, d.act, d.dtype = B, pc.act, _lib.DP_BF16
    _lib.check(_lib.load().dp_conv2d(C.byref(d), _s()), "conv halo48")
    torch.cuda.synchronize()
    _close(wide[..., 96:96 + cout], ref.permute(0, 2, 3, 1), "bf16", "halo 48")
    assert (wide[..., :96] == 3.0).all() and (wide[..., 96 + cout:] == 3.0).all(), "wrote outside its slice"


@pytest.mark.parametrize("dt", DT)
def test_conv2d_stem_pad_and_upsample(dt):
    """2x2 conv over F.pad(0,1,0,1) (StemBlock) and the x2 nearest upsample epilogue."""
    torch.manual_seed(3)
    pk = Packer({}, dt, torch.device("cuda"))
    x = torch.randn(1, 32, 10, 12)
    w = torch.randn(16, 32, 2, 2) / 11.0
    b = torch.randn(16) * 0.1
    pc = pk.conv(w.double(), b.double(), act="relu", pad=0, lab=(1.3, -0.2))
    ref = 1.3 * F.relu(F.conv2d(F.pad(_rb(x, dt), (0, 1, 0, 1)), _rb(w, dt), b)) - 0.2
    out = torch.empty(1, 10, 12, 16, device="cuda", dtype=DTYPES[dt][0])
    up = torch.empty(1, 20, 24, 16, device="cuda", dtype=DTYPES[dt][0])
    _run_conv(pc, _nhwc(x, dt), out, dt, up=up)
    torch.cuda.synchronize()
    _close(out, ref.permute(0, 2, 3, 1), dt, "stem2a")
    _close(up, F.interpolate(ref, scale_factor=2.0, mode="nearest").permute(0, 2, 3, 1), dt, "upsample")


@pytest.mark.parametrize("dt", DT)
@pytest.mark.parametrize("k,s", [(3, 2), (5, 1), (3, 1)])
def test_dwconv(dt, k, s):
    torch.manual_seed(k + s)
    pk = Packer({}, dt, torch.device("cuda"))
    Cc = 64
    x = torch.randn(2, Cc, 15, 16)
    w = torch.randn(Cc, 1, k, k) / k
    b = torch.randn(Cc) * 0.1
    pc = pk.dwconv(w.double(), b.double(), s, act="relu")
    ref = F.relu(F.conv2d(_rb(x, dt), w, b, s, (k - 1) // 2, groups=Cc))
    out = torch.empty(2, ref.shape[2], ref.shape[3], Cc, device="cuda", dtype=DTYPES[dt][0])
    _run_conv(pc, _nhwc(x, dt), out, dt)
    torch.cuda.synchronize()
    _close(out, ref.permute(0, 2, 3, 1), dt, f"dw{k}s{s}")


@pytest.mark.parametrize("k,s,c,hw", [(5, 1, 192, 40), (3, 2, 512, 80), (3, 2, 128, 33), (5, 1, 384, 20)])
def test_dwconv_model_shapes(k, s, c, hw):
    """The LDS-tiled bf16 depthwise path at HGNetv2-L stage shapes (several tiles per image,
    partial edge tiles, 64-channel blocks) vs torch fp32 conv2d on the bf16-rounded input."""
    torch.manual_seed(k * c)
    pk = Packer({}, "bf16", torch.device("cuda"))
    x = torch.randn(3, c, hw, hw).bfloat16().float()
    w = torch.randn(c, 1, k, k) / k
    b = torch.randn(c) * 0.1
    pc = pk.dwconv(w.double(), b.double(), s, act="relu")
    ref = F.relu(F.conv2d(x, w, b, s, (k - 1) // 2, groups=c))
    out = torch.empty(3, ref.shape[2], ref.shape[3], c, device="cuda", dtype=torch.bfloat16)
    _run_conv(pc, _nhwc(x, "bf16"), out, "bf16")
    torch.cuda.synchronize()
    _close(out, ref.permute(0, 2, 3, 1), "bf16", f"dw{k}s{s}c{c}")


@pytest.mark.parametrize("h,w,c", [(37, 23, 128), (50, 19, 64), (9, 40, 192), (41, 40, 64), (3, 7, 64)])
def test_dwconv5_ragged(h, w, c):
    """Both bf16 5x5 paths on ragged rectangles: maps at most 20 wide (one 4 x 20 tile per block,
    4 outputs per thread: 50x19, 3x7) and wider ones (persistent 8 x 20 tiles: 37x23, 9x40,
    41x40): partial tiles in both directions, fewer rows than one tile."""
    torch.manual_seed(h * w)
    pk = Packer({}, "bf16", torch.device("cuda"))
    x = torch.randn(2, c, h, w).bfloat16().float()
    wt = torch.randn(c, 1, 5, 5) / 5
    b = torch.randn(c) * 0.1
    pc = pk.dwconv(wt.double(), b.double(), 1, act="relu")
    ref = F.relu(F.conv2d(x, wt, b, 1, 2, groups=c))
    out = torch.full((2, h, w, c), 7.0, device="cuda", dtype=torch.bfloat16)
    _run_conv(pc, _nhwc(x, "bf16"), out, "bf16")
    torch.cuda.synchronize()
    _close(out, ref.permute(0, 2, 3, 1), "bf16", f"dw5 rows {h}x{w}c{c}")


@pytest.mark.parametrize("dt", DT)
def test_stem_conv_and_pool(dt):
    lib = _lib.load()
    torch.manual_seed(5)
    img = torch.rand(2, 3, 22, 26)
    w = torch.randn(32, 3, 3, 3) / 5
    b = torch.randn(32) * 0.1
    # bf16: the image and the weights are the MFMA's bf16 operands (stem1_mfma_kernel)
    ref = F.relu(F.conv2d(_rb(img, dt), _rb(w, dt), b, 2, 1))
    out = torch.empty(2, 11, 13, 32, device="cuda", dtype=DTYPES[dt][0])
    _lib.check(lib.dp_stem_conv(_d(img), 2, 22, 26, _d(w.reshape(32, 27)), _d(b), 32, 0, C.c_float(1),
                                C.c_float(0), out.data_ptr(), 11 * 13 * 32, 32, DTYPES[dt][1], _s()))
    torch.cuda.synchronize()
    _close(out, ref.permute(0, 2, 3, 1), dt, "stem1")
    x = torch.randn(2, 16, 9, 7)
    pool = torch.empty(2, 9, 7, 16, device="cuda", dtype=DTYPES[dt][0])
    xi = _nhwc(x, dt)
    _lib.check(lib.dp_maxpool2x2_pad_rb(xi.data_ptr(), 9 * 7 * 16, 16, 2, 9, 7, 16, pool.data_ptr(), 9 * 7 * 16, 16,
                                        DTYPES[dt][1], _s()))
    torch.cuda.synchronize()
    refp = F.max_pool2d(F.pad(x.to(DTYPES[dt][0]).float(), (0, 1, 0, 1)), 2, 1, ceil_mode=True)
    _close(pool, refp.permute(0, 2, 3, 1), dt, "pool")


@pytest.mark.parametrize("cin,cout,H,W,lab", [(32, 16, 37, 45, None), (16, 8, 20, 17, (1.3, -0.2)),
                                              (64, 32, 9, 70, None)])
def test_conv2d_pool_fused(cin, cout, H, W, lab):
    """dp_conv2d_pool (stem2a + stem max-pool in one pass): the conv as dp_conv2d's bf16
    tolerance, the pool bit-exact vs F.max_pool2d(F.pad(x,(0,1,0,1)), 2, 1) of the same bf16
    input, written into a channel slice of a wider (concat) buffer; ragged 8x16 tiles."""
    lib = _lib.load()
    torch.manual_seed(cin + H)
    pk = Packer({}, "bf16", torch.device("cuda"))
    # lab case: shifted negative, so the F.pad zeros must win the max at the right/bottom edge
    x = (torch.randn(3, cin, H, W) - (0.5 if lab else 0.0)).bfloat16().float()
    w = torch.randn(cout, cin, 2, 2) / (2 * cin ** 0.5)
    b = torch.randn(cout) * 0.1
    pc = pk.conv(w.double(), b.double(), act="relu", pad=0, lab=lab)
    ref = F.relu(F.conv2d(F.pad(x, (0, 1, 0, 1)), _rb(w, "bf16"), b))
    if lab:
        ref = lab[0] * ref + lab[1]
    xi = _nhwc(x, "bf16")
    out = torch.empty(3, H, W, cout, device="cuda", dtype=torch.bfloat16)
    cat = torch.full((3, H, W, 2 * cin), 7.0, device="cuda", dtype=torch.bfloat16)
    d = ConvDesc()
    d.in_, d.in_bstride, d.in_pstride, d.in_h, d.in_w, d.cin = xi.data_ptr(), H * W * cin, cin, H, W, cin
    d.weight, d.kpad, d.bias = pc.w.data_ptr(), pc.kpad, pc.b.data_ptr()
    d.kh, d.kw, d.stride, d.pad_t, d.pad_l = 2, 2, 1, 0, 0
    d.out, d.out_bstride, d.out_pstride, d.out_h, d.out_w, d.cout = out.data_ptr(), H * W * cout, cout, H, W, cout
    d.batch, d.act, d.dtype = 3, pc.act, _lib.DP_BF16
    if lab:
        d.has_lab, d.lab_scale, d.lab_bias = 1, lab[0], lab[1]
    _lib.check(lib.dp_conv2d_pool(C.byref(d), cat.data_ptr(), H * W * 2 * cin, 2 * cin, _s()), "conv2d_pool")
    torch.cuda.synchronize()
    _close(out, ref.permute(0, 2, 3, 1), "bf16", "stem2a (fused)")
    refp = F.max_pool2d(F.pad(x, (0, 1, 0, 1)), 2, 1, ceil_mode=True).permute(0, 2, 3, 1)
    assert torch.equal(cat[..., :cin].float().cpu(), refp), "fused pool differs"
    assert (cat[..., cin:] == 7.0).all(), "fused pool wrote outside its channel slice"


@pytest.mark.parametrize("k,cin,cout,lab", [(2, 16, 32, None), (2, 8, 16, (0.9, 0.1)), (2, 32, 16, None),
                                            (2, 16, 8, None), (1, 32, 48, None), (1, 32, 64, (1.1, -0.1)),
                                            (1, 16, 16, None)])
def test_conv2d_stem_direct(k, cin, cout, lab):
    """The stem's register-direct kernels through dp_conv2d: 2x2 over F.pad(0,1,0,1) (stem2b
    writes a channel slice of the concat buffer) and the 1x1 stem4 (1-4 output tiles) vs torch
    fp32 on the bf16-rounded input, ragged 16-pixel groups."""
    torch.manual_seed(k * cin * cout)
    pk = Packer({}, "bf16", torch.device("cuda"))
    B, H, W = 2, 23, 37
    x = torch.randn(B, cin, H, W).bfloat16().float()
    w = torch.randn(cout, cin, k, k) / (k * cin ** 0.5)
    b = torch.randn(cout) * 0.1
    pc = pk.conv(w.double(), b.double(), act="relu", pad=0, lab=lab)
    ref = F.relu(F.conv2d(F.pad(x, (0, 1, 0, 1)) if k == 2 else x, _rb(w, "bf16"), b))
    if lab:
        ref = lab[0] * ref + lab[1]
    wide = torch.full((B, H, W, 2 * cout), 5.0, device="cuda", dtype=torch.bfloat16)
    xi = _nhwc(x, "bf16")
    d = ConvDesc()
    d.in_, d.in_bstride, d.in_pstride, d.in_h, d.in_w, d.cin = xi.data_ptr(), H * W * cin, cin, H, W, cin
    d.weight, d.kpad, d.bias = pc.w.data_ptr(), pc.kpad, pc.b.data_ptr()
    d.kh, d.kw, d.stride, d.pad_t, d.pad_l = k, k, 1, 0, 0
    d.out, d.out_bstride, d.out_pstride = wide.data_ptr() + 2 * cout, H * W * 2 * cout, 2 * cout
    d.out_h, d.out_w, d.cout = H, W, cout
    d.batch, d.act, d.dtype = B, pc.act, _lib.DP_BF16
    if lab:
        d.has_lab, d.lab_scale, d.lab_bias = 1, lab[0], lab[1]
    _lib.check(_lib.load().dp_conv2d(C.byref(d), _s()), "conv2x2")
    torch.cuda.synchronize()
    _close(wide[..., cout:], ref.permute(0, 2, 3, 1), "bf16", f"stem {k}x{k} {cin}->{cout}")
    assert (wide[..., :cout] == 5.0).all(), "wrote outside the channel slice"


@pytest.mark.parametrize("dt", DT)
@pytest.mark.parametrize("rows,ncls", [(1000, 2), (8400 * 2 + 37, 3)])
def test_layernorm_classmax(dt, rows, ncls):
    """dp_layernorm_classmax (enc_output_norm + enc_out_class_embed + max, one pass): the rows
    vs torch LayerNorm with the border mask, the scores vs max_j(y . w_j + b_j) over the
    STORED rows (what dp_class_max would read), fp32 CPU reference."""
    lib = _lib.load()
    torch.manual_seed(rows + ncls)
    c, period = 256, 8400
    x = torch.randn(rows, c) * 2 + 0.3
    g = torch.rand(c) + 0.5
    b = torch.randn(c) * 0.1
    mask = (torch.rand(period) < 0.05).to(torch.uint8)
    mrow = torch.randn(c)
    w = torch.randn(ncls, c) / 16
    wb = torch.randn(ncls) * 0.1
    tdt = DTYPES[dt][0]
    xi = x.to("cuda", tdt)
    out = torch.empty(rows, c, device="cuda", dtype=tdt)
    score = torch.empty(rows, device="cuda")
    _lib.check(lib.dp_layernorm_classmax(out.data_ptr(), xi.data_ptr(), _d(g), _d(b), C.c_float(1e-5), rows, c,
                                         _d(mask), period, _d(mrow), _d(w), _d(wb), ncls, score.data_ptr(),
                                         DTYPES[dt][1], _s()), "ln_classmax")
    torch.cuda.synchronize()
    ref = F.layer_norm(xi.float().cpu(), (c,), g, b, 1e-5)
    m = mask[torch.arange(rows) % period].bool()
    ref[m] = mrow
    _close(out, ref, dt, "ln rows")
    y = out.float().cpu()
    sref = (y @ w.t() + wb).max(-1).values
    err = (score.cpu() - sref).abs().max().item()
    assert err <= 1e-4 * max(1.0, sref.abs().max().item()), err


@pytest.mark.parametrize("dt", DT)
@pytest.mark.parametrize("c", [128, 256, 384])
def test_layernorm_variants(dt, c):
    lib = _lib.load()
    torch.manual_seed(c)
    rows, T = 36, 18
    x = torch.randn(rows, c)
    r = torch.randn(rows, c)
    g, bb = 1 + 0.1 * torch.randn(c), 0.1 * torch.randn(c)
    post = torch.randn(rows // T * (T - 1), c)
    mask = (torch.arange(rows) % 5 == 0).to(torch.uint8)
    mrow = torch.randn(c)
    td = DTYPES[dt][0]
    out = torch.empty(rows, 2 * c, device="cuda", dtype=td)
    _lib.check(lib.dp_layernorm(out.data_ptr(), contiguous_rows(2 * c), _d(x, td), contiguous_rows(c), _d(r, td),
                                contiguous_rows(c), _d(g), _d(bb), C.c_float(1e-5), rows, c, _d(post, td),
                                contiguous_rows(c), T, 1, None, 1, None, DTYPES[dt][1], _s()))
    ref = F.layer_norm(x.to(td).float() + r.to(td).float(), (c,), g, bb)
    kp = (torch.arange(rows) % T) != 0
    ref[kp] += post.to(td).float()
    torch.cuda.synchronize()
    _close(out[:, :c], ref, dt, "ln+post")
    out2 = torch.empty(rows, c, device="cuda", dtype=td)
    _lib.check(lib.dp_layernorm(out2.data_ptr(), contiguous_rows(c), _d(x, td), contiguous_rows(c), None,
                                rowmap(group=1), _d(g), _d(bb), C.c_float(1e-5), rows, c, None, rowmap(group=1), 1, 0,
                                _d(mask), 7, _d(mrow), DTYPES[dt][1], _s()))
    ref2 = F.layer_norm(x.to(td).float(), (c,), g, bb)
    ref2[torch.arange(rows) % 7 % 5 == 0] = mrow
    torch.cuda.synchronize()
    _close(out2, ref2, dt, "ln+mask")


@pytest.mark.parametrize("dt", DT)
def test_gate_layernorm(dt):
    lib = _lib.load()
    torch.manual_seed(9)
    rows, c = 40, 256
    gt, xc = torch.randn(rows, 2 * c), torch.randn(rows, 2 * c)
    g, bb = 1 + 0.1 * torch.randn(c), 0.1 * torch.randn(c)
    td = DTYPES[dt][0]
    out = torch.empty(rows, c, device="cuda", dtype=td)
    _lib.check(lib.dp_gate_layernorm(out.data_ptr(), c, _d(gt, td), _d(xc, td), _d(g), _d(bb), C.c_float(1e-5),
                                     rows, c, DTYPES[dt][1], _s()))
    gt, xc = gt.to(td).float(), xc.to(td).float()
    s = torch.sigmoid(gt)
    ref = F.layer_norm(s[:, :c] * xc[:, :c] + s[:, c:] * xc[:, c:], (c,), g, bb)
    torch.cuda.synchronize()
    _close(out, ref, dt, "gate")


def _attn_ref(q, k, v, nh, bf16=False, block=64):
    """softmax(QK^T/sqrt(dh))V; bf16=True emulates the bf16 kernels: the unnormalised
    probabilities exp(s - m) are the bf16 MFMA operand of PV (m = the running max over the
    key blocks seen so far, 64-key blocks), the row sum stays f32, O = (P V) / sum."""
    B, L, Cc = q.shape
    dh = Cc // nh
    q = q.reshape(B, L, nh, dh).transpose(1, 2)
    k = k.reshape(B, -1, nh, dh).transpose(1, 2)
    v = v.reshape(B, -1, nh, dh).transpose(1, 2)
    s = q @ k.transpose(-1, -2) / dh ** 0.5
    if not bf16:
        a = torch.softmax(s, -1)
        return (a @ v).transpose(1, 2).reshape(B, L, Cc)
    S = s.shape[-1]
    m_fin = s.max(-1, keepdim=True).values
    o = torch.zeros(*s.shape[:-1], dh)
    m_run = torch.full_like(m_fin, float("-inf"))
    for k0 in range(0, S, block):
        sb = s[..., k0:k0 + block]
        m_run = torch.maximum(m_run, sb.max(-1, keepdim=True).values)
        pb = torch.exp(sb - m_run).bfloat16().float()
        o = o + (pb @ v[..., k0:k0 + block, :]) * torch.exp(m_run - m_fin)
    l = torch.exp(s - m_fin).sum(-1, keepdim=True)
    return (o / l).transpose(1, 2).reshape(B, L, Cc)


@pytest.mark.parametrize("dt", DT)
@pytest.mark.parametrize("geom", ["within", "across", "aifi", "aifi_x", "aifi_n", "aifi_ragged", "within_n",
                                  "across_n", "within_x", "across_x"])
def test_attention(dt, geom):
    """Decoder within / across attention (short kernel) and AIFI (long kernel, online softmax
    over 64-key blocks; a ragged 250-token sequence exercises the masked tail block)."""
    lib = _lib.load()
    torch.manual_seed(len(geom))
    B, nq, T = 2, 60, 18
    Cc = {"aifi_x": 384, "aifi_n": 128, "within_n": 128, "across_n": 128, "within_x": 384, "across_x": 384}.get(geom, 256)
    nh = 8
    S = 250 if geom == "aifi_ragged" else 400
    rows = B * S if geom.startswith("aifi") else B * nq * T
    qkv = torch.randn(rows, 3 * Cc)
    td = DTYPES[dt][0]
    qd = qkv.to("cuda", td)
    out = torch.empty(rows, Cc, device="cuda", dtype=td)
    e = qd.element_size()
    q32 = qkv.to(td).float()
    if geom.startswith("within"):
        args = (B * nq, 1, T, 0, 1, T)
        seqs = q32.reshape(B * nq, T, 3 * Cc)
    elif geom.startswith("across"):
        args = (B, T, nq * T, 1, T, nq)
        seqs = q32.reshape(B, nq, T, 3 * Cc).transpose(1, 2).reshape(B * T, nq, 3 * Cc)
    else:
        args = (B, 1, S, 0, 1, S)
        seqs = q32.reshape(B, S, 3 * Cc)
    _lib.check(lib.dp_attention(qd.data_ptr(), 3 * Cc, qd.data_ptr() + Cc * e, qd.data_ptr() + 2 * Cc * e, 3 * Cc,
                                out.data_ptr(), Cc, *args, nh, Cc // nh, DTYPES[dt][1], _s()))
    ref = _attn_ref(seqs[..., :Cc], seqs[..., Cc:2 * Cc], seqs[..., 2 * Cc:], nh, bf16=dt == "bf16")
    if geom.startswith("across"):
        ref = ref.reshape(B, T, nq, Cc).transpose(1, 2)
    torch.cuda.synchronize()
    _close(out.reshape(-1, Cc), ref.reshape(-1, Cc), dt, geom)


@pytest.mark.parametrize("dt", DT)
@pytest.mark.parametrize("size", ["n", "l", "x"])
def test_msda_golden(golden_dir, dt, size):
    """dp_msda vs the reference's ms_deform_attn_core_pytorch vectors (tests/golden/msda_*.npz).
    The kernel takes offsets + logits (as the projection GEMM emits them); the fixture's
    absolute locations are re-expressed as offsets from a per-token reference point."""
    lib = _lib.load()
    g = np.load(os.path.join(golden_dir, f"msda_{size}.npz"))
    value, loc, logits = (torch.from_numpy(g[k]) for k in ("value", "loc", "attn_logits"))
    shapes = [tuple(int(v) for v in s) for s in g["shapes"]]
    N, Lq, H, L, P, _ = loc.shape
    ref_pt = torch.rand(N, Lq, 2, generator=torch.Generator().manual_seed(1))
    wh = torch.tensor([[w, h] for h, w in shapes], dtype=torch.float32)
    off = (loc - ref_pt[:, :, None, None, None, :]) * wh[None, None, None, :, None, :]
    offattn = torch.cat([off.reshape(N * Lq, -1), logits.reshape(N * Lq, -1)], 1)
    td = DTYPES[dt][0]
    oad = offattn.to("cuda", td).contiguous()
    vd = value.to("cuda", td).contiguous()
    Cc = value.shape[2]
    out = torch.empty(N * Lq, Cc, device="cuda", dtype=td)
    hw = (C.c_int32 * (2 * L))(*[v for s in shapes for v in s])
    _lib.check(lib.dp_msda(vd.data_ptr(), N, value.shape[1], hw, L, oad.data_ptr(), _d(ref_pt), out.data_ptr(), Cc,
                           Lq, H, Cc // H, P, DTYPES[dt][1], _s()))
    torch.cuda.synchronize()
    if dt == "fp32":
        _close(out.reshape(N, Lq, Cc), torch.from_numpy(g["out"]), dt, "msda vs reference")
    else:
        # bf16: compare with the oracle on the bf16-rounded inputs
        oa = oad.float().cpu()
        loc2 = ref_pt[:, :, None, None, None, :] + oa[:, :H * L * P * 2].reshape(N, Lq, H, L, P, 2) / \
            wh[None, None, None, :, None, :]
        a2 = torch.softmax(oa[:, H * L * P * 2:].reshape(N, Lq, H, L * P), -1).reshape(N, Lq, H, L, P)
        _close(out.reshape(N, Lq, Cc), O.msda_core(vd.float().cpu(), shapes, loc2, a2), dt, "msda vs oracle(bf16)")


@pytest.mark.parametrize("size", ["n", "l", "x"])
def test_msda_batched(size):
    """dp_msda (bf16 wave-per-token path) on a multi-image batch at the model's real level
    geometry: tokens of several images, XCD-sliced block order, points falling outside the
    maps (zero corners) -- vs the oracle's ms_deform_attn_core restatement on the same
    bf16-rounded inputs (only the output is rounded: one bf16 ulp of the output scale)."""
    lib = _lib.load()
    cfg = {"n": (2, 6, 16, [(40, 40), (20, 20)]), "l": (3, 4, 32, [(80, 80), (40, 40), (20, 20)]),
           "x": (3, 4, 48, [(80, 80), (40, 40), (20, 20)])}[size]
    L, P, dh, shapes = cfg
    H, B, Lq = 8, 3, 1080
    S = sum(h * w for h, w in shapes)
    Cc = H * dh
    g = torch.Generator().manual_seed(7)
    value = torch.randn(B, S, Cc, generator=g).bfloat16()
    ref_pt = torch.rand(B, Lq, 2, generator=g) * 1.2 - 0.1
    off = torch.randn(B * Lq, H * L * P * 2, generator=g) * 3.0
    logits = torch.randn(B * Lq, H * L * P, generator=g)
    oad = torch.cat([off, logits], 1).to("cuda", torch.bfloat16).contiguous()
    vd = value.cuda()
    out = torch.empty(B * Lq, Cc, device="cuda", dtype=torch.bfloat16)
    hw = (C.c_int32 * (2 * L))(*[v for s in shapes for v in s])
    _lib.check(lib.dp_msda(vd.data_ptr(), B, S, hw, L, oad.data_ptr(), _d(ref_pt), out.data_ptr(), Cc,
                           Lq, H, dh, P, DTYPES["bf16"][1], _s()))
    torch.cuda.synchronize()
    oa = oad.float().cpu()
    wh = torch.tensor([[w, h] for h, w in shapes], dtype=torch.float32)
    loc = ref_pt[:, :, None, None, None, :] + oa[:, :H * L * P * 2].reshape(B, Lq, H, L, P, 2) / \
        wh[None, None, None, :, None, :]
    a = torch.softmax(oa[:, H * L * P * 2:].reshape(B, Lq, H, L * P), -1).reshape(B, Lq, H, L, P)
    _close(out.reshape(B, Lq, Cc), O.msda_core(value.float(), shapes, loc, a), "bf16", "msda batched vs oracle")


@pytest.mark.parametrize("n,k", [(8400, 60), (2000, 60), (120, 60), (300, 256), (17, 4)])
def test_topk(n, k):
    lib = _lib.load()
    torch.manual_seed(n)
    rows = 3
    x = torch.randn(rows, n)
    x[1, : n // 3] = 0.25  # ties: lower index first
    ov = torch.empty(rows, k, device="cuda")
    oi = torch.empty(rows, k, dtype=torch.int64, device="cuda")
    _lib.check(lib.dp_topk(_d(x), rows, n, n, k, ov.data_ptr(), oi.data_ptr(), _s()))
    torch.cuda.synchronize()
    key = torch.stack([torch.tensor(sorted(range(n), key=lambda i: (-x[r, i].item(), i))[:k]) for r in range(rows)])
    np.testing.assert_array_equal(oi.cpu().numpy(), key.numpy())
    np.testing.assert_array_equal(ov.cpu().numpy(), torch.gather(x, 1, key).numpy())


def test_decoder_head_kernels():
    """sine embed, linear_small (+add, broadcast weight), pose refine, pre-pose, LQE, postprocess
    (f32 kernels)."""
    lib = _lib.load()
    torch.manual_seed(11)
    B, nq, K, Cc = 2, 60, 17, 256
    rows = B * nq
    ref = torch.rand(B, nq, K + 1, 2)
    dim_t = (10000 ** (2 * torch.div(torch.arange(Cc // 2), 2, rounding_mode="floor") / (Cc // 2))).float()
    se = torch.empty(rows * K, Cc, device="cuda")
    _lib.check(lib.dp_sine_embed(_d(ref), rows, K, Cc, _d(dim_t), se.data_ptr(), 0, _s()))
    torch.cuda.synchronize()
    _close(se, O.sine_embedding(ref[:, :, 1:], dim_t).reshape(-1, Cc), "fp32", "sine")
    # linear_small with weight broadcast (nw=1, n=2) and add
    x = torch.randn(rows, 85)
    w = torch.randn(1, 85)
    b = torch.randn(1)
    add = torch.randn(rows, 2)
    out = torch.empty(rows, 2, device="cuda")
    _lib.check(lib.dp_linear_small(_d(x), contiguous_rows(85), 0, rows, 85, _d(w.t()), _d(b), 1, 2, 0, _d(add),
                                   out.data_ptr(), _s()))
    torch.cuda.synchronize()
    _close(out, (x @ w.t() + b) + add, "fp32", "linear_small")
    # pose refine (Integral + distance2pose + centre)
    corners = torch.randn(rows * K, 66)
    ref_init = torch.rand(rows * K, 2)
    project = O.weighting_function(32, 0.5, 4.0)
    kps = torch.empty(B, nq, K, 2, device="cuda")
    refo = torch.empty(B, nq, K + 1, 2, device="cuda")
    _lib.check(lib.dp_pose_refine(_d(corners), _d(project), 32, _d(ref_init), C.c_float(4.0), rows, K,
                                  kps.data_ptr(), refo.data_ptr(), _s()))
    prob = torch.softmax(corners.reshape(-1, 33), 1)
    d = (prob @ project).reshape(B, nq, K, 2)
    kref = ref_init.reshape(B, nq, K, 2) + d / 4.0
    torch.cuda.synchronize()
    _close(kps, kref, "fp32", "refine")
    _close(refo, torch.cat([kref.mean(2, keepdim=True), kref], 2), "fp32", "refine ref")
    # pre-pose
    pre = torch.randn(rows * K, 2)
    outp = torch.empty(rows * K, 2, device="cuda")
    _lib.check(lib.dp_pre_pose(_d(pre), _d(ref), rows, K, outp.data_ptr(), _s()))
    torch.cuda.synchronize()
    _close(outp, torch.sigmoid(pre + O.inverse_sigmoid(ref[:, :, 1:].reshape(-1, 2))), "fp32", "pre_pose")
    # LQE stats
    feat = torch.randn(B, 20, 24, Cc)
    kp = torch.rand(B, nq, K, 2) * 1.1 - 0.05
    st = torch.empty(rows, K * 5, device="cuda")
    _lib.check(lib.dp_lqe_stats(_d(feat), 20 * 24 * Cc, 20, 24, Cc, _d(kp), B, nq, K, st.data_ptr(), 0, _s()))
    s = O.bilinear_gather(feat, kp.reshape(B, nq * K, 2)).reshape(B, nq, K, Cc)
    top = s.topk(4, dim=-1)[0]
    torch.cuda.synchronize()
    _close(st, torch.cat([top, top.mean(-1, keepdim=True)], -1).reshape(rows, -1), "fp32", "lqe")
    # postprocess
    logits = torch.randn(B, nq, 2)
    ts = torch.tensor([[640.0, 480.0], [320.0, 200.0]])
    sc = torch.empty(B, 60, device="cuda")
    lb = torch.empty(B, 60, dtype=torch.int64, device="cuda")
    ok = torch.empty(B, 60, K, 2, device="cuda")
    _lib.check(lib.dp_postprocess(_d(logits), _d(kp), _d(ts), B, nq, 2, K, 60, sc.data_ptr(), lb.data_ptr(),
                                  ok.data_ptr(), _s()))
    rs, rl, rk = O.postprocess(logits, kp, ts)
    torch.cuda.synchronize()
    _close(sc, rs, "fp32", "pp scores")
    np.testing.assert_array_equal(lb.cpu().numpy(), rl.numpy())
    _close(ok, rk, "fp32", "pp kps")


@pytest.mark.parametrize("dt", DT)
@pytest.mark.parametrize("cout", [2, 34, 66])
def test_linear_f32_out(dt, cout):
    """bf16/f32 activations in, f32 out (+ f32 residual): the head layers (corners, enc pose, pre-pose)."""
    torch.manual_seed(cout)
    pk = Packer({}, dt, torch.device("cuda"))
    rows, k = 1000, 256
    x = torch.randn(rows, k)
    w = torch.randn(cout, k) / 16
    b = torch.randn(cout)
    pc = pk.linear(w, b, exact=True)
    assert pc.cout == cout
    out = torch.empty(1, 1, rows, cout, device="cuda")
    res = torch.randn(1, 1, rows, cout)
    resd = res.cuda()
    xd = x.to("cuda", DTYPES[dt][0]).reshape(1, 1, rows, k)
    lib = _lib.load()
    d = ConvDesc()
    d.in_, d.in_bstride, d.in_pstride, d.in_h, d.in_w, d.cin = xd.data_ptr(), rows * k, k, 1, rows, k
    d.weight, d.kpad, d.bias = pc.w.data_ptr(), pc.kpad, pc.b.data_ptr()
    d.kh = d.kw = d.stride = 1
    d.out, d.out_bstride, d.out_pstride, d.out_h, d.out_w, d.cout = out.data_ptr(), rows * cout, cout, 1, rows, cout
    d.res, d.res_bstride, d.res_pstride = resd.data_ptr(), rows * cout, cout
    d.batch, d.dtype, d.out_f32 = 1, DTYPES[dt][1], 1
    _lib.check(lib.dp_conv2d(C.byref(d), _s()))
    torch.cuda.synchronize()
    ref = x.to(DTYPES[dt][0]).float() @ w.to(DTYPES[dt][0]).float().t() + b + res.reshape(rows, cout)
    _close(out.reshape(rows, cout), ref, "fp32" if dt == "fp32" else "bf16", f"f32-out {cout}")
