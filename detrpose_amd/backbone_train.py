"""The HGNetv2 backbone's training step on the HIP kernels (BASELINE config 5, the backbone part):
the forward of every ConvBNAct with its FrozenBatchNorm2d folded into per-step packed weights,
and the backward to every backbone parameter (conv weights, LearnableAffineBlock scalars).

Reference: HGNetv2.forward (src/nn/backbone/hgnetv2.py:586-593) with StemBlock (169-220),
HG_Stage (332-383), HG_Block (243-329, agg 'se': squeeze + excitation ConvBNAct), LightConvBNAct
(137-166), ConvBNAct (82-134: conv -> FrozenBatchNorm2d (24-61) -> ReLU -> LAB (68-79)). The
configs train it whole: freeze_at=-1 freezes nothing (hgnetv2.py:526-530), freeze_norm=True
turns every norm into FrozenBatchNorm2d (532-533): a fixed affine y = s z + b.

Forward: the inference conv kernels with the frozen affine folded into the weights, packed from
the f32 master at the start of each step (dp_conv_pack with the per-channel scale; the shift b
is the epilogue bias), ReLU and LAB in the epilogue, the HG-block residual as its residual input,
concats written in place. Backward, per ConvBNAct: dp_frozen_act_bwd (ReLU / LAB read off the
stored output, LAB scalar gradients, times the frozen scale) gives d conv-output; then
  1x1            wgrad dp_gemm (dz^T x), dgrad dp_conv2d of dz with the transposed packing
  k x k s1       wgrad dp_im2col + dp_gemm, dgrad dp_conv2d of dz with the rotated weights
                 (stem2a / stem2b read F.pad(0,1,0,1): the rotated conv pads top / left)
  3x3 s2 dense   StemBlock.stem3: dgrad dz W on the 1x1 conv kernel (columns tap-major) + dp_col2im
  depthwise      dp_dwconv_bwd (3x3 s2 downsample, 5x5 / 3x3 LightConv)
  stem1          wgrad only (the image takes no gradient): dp_im2col over the f32 NCHW image
  max-pool       dp_maxpool2x2_pad_rb_bwd
"""
from __future__ import annotations

import ctypes as C

import torch

from . import _lib
from ._lib import DP_F32, ConvDesc
from .encoder_train import V, TapePlan, _p, pad_to

B_ = "backbone."


class BackboneTrainPlan(TapePlan):
    """Forward / backward tapes of the backbone for one batch at image size (H, W); `outs` are
    the return_idx stage outputs (the encoder's input maps, gradients accumulated into them by
    the encoder's backward)."""

    def __init__(self, eng, B: int, H: int, W: int):
        self._setup(eng)
        prev = getattr(eng, "cur", None)
        eng.cur = self
        bb = eng.model.backbone
        self.bb = bb
        arch = bb.arch_configs[bb.name]
        _, mid, sout = arch["stem_channels"]
        self.use_lab = bool(bb.use_lab)
        self.B, self.H, self.W = B, H, W
        self.labs = []          # (descriptor or None, prefix) of every LAB layer: host values per step
        self.labv = {}
        sd = {k: v.detach() for k, v in eng.model.state_dict().items()}
        self.frozen = {}
        self.image = torch.empty(B, 3, H, W, dtype=torch.float32, device=self.dev)
        self.arena.append(self.image)

        # ---------------- StemBlock (hgnetv2.py:210-220)
        st = B_ + "stem."
        h1, w1 = (H + 1) // 2, (W + 1) // 2
        s1 = self.view(B, h1, w1, mid)
        self.stem1(st + "stem1", s1, sd)
        s2a = self.view(B, h1, w1, mid // 2)
        self.cba(st + "stem2a", s1, s2a, sd, k=2, pad=0)
        cat = self.view(B, h1, w1, 2 * mid)
        self.maxpool("stem.pool", s1, cat.ch(0, mid))
        self.cba(st + "stem2b", s2a, cat.ch(mid, mid), sd, k=2, pad=0)
        h, w = (h1 + 1) // 2, (w1 + 1) // 2
        s3 = self.view(B, h, w, mid)
        self.cba(st + "stem3", cat, s3, sd, k=3, stride=2)
        x_src = s3
        first = True
        self.outs = []
        for si, key in enumerate(arch["stage_config"]):
            cin, midc, cout, nblk, down, light, ks, nl = arch["stage_config"][key]
            sp = f"{B_}stages.{si}"
            if down:
                h, w = (h + 1) // 2, (w + 1) // 2
            blocks_in = [self.view(B, h, w, (cin if bi == 0 else cout) + nl * midc) for bi in range(nblk)]
            slot0 = blocks_in[0].ch(0, cin)
            if first:
                self.cba(st + "stem4", x_src, slot0, sd, k=1)
                first = False
            if down:
                self.cba(sp + ".downsample", x_src, slot0, sd, k=3, stride=2, dw=True, act=False)
            for bi in range(nblk):
                bp = f"{sp}.blocks.{bi}"
                cb = blocks_in[bi]
                bin_ = cin if bi == 0 else cout
                prev_ = cb.ch(0, bin_)
                for li in range(nl):
                    lp = f"{bp}.layers.{li}"
                    dst = cb.ch(bin_ + li * midc, midc)
                    if light:
                        t = self.view(B, h, w, midc)
                        self.cba(lp + ".conv1", prev_, t, sd, k=1, act=False)
                        self.cba(lp + ".conv2", t, dst, sd, k=ks, dw=True)
                    else:
                        self.cba(lp, prev_, dst, sd, k=ks)
                    prev_ = dst
                sq = self.view(B, h, w, cout // 2)
                self.cba(bp + ".aggregation.0", cb, sq, sd, k=1)
                dst = blocks_in[bi + 1].ch(0, cout) if bi + 1 < nblk else self.view(B, h, w, cout)
                self.cba(bp + ".aggregation.1", sq, dst, sd, k=1, res=cb.ch(0, bin_) if bi > 0 else None)
                x_src = dst
            if si in bb.return_idx:
                self.outs.append(x_src)
        self._record_backward(zero=False)   # zeroed by the encoder's backward, which runs first
        self.batch_packs()
        eng.cur = prev

    # ------------------------------------------------------------------ frozen BN
    def _frozen(self, p, sd, cout_p):
        """FrozenBatchNorm2d (hgnetv2.py:51-61) as (scale [cout], shift [cout_p], zero-padded)."""
        if p not in self.frozen:
            w, b, rm, rv = (sd[p + ".bn." + k].double() for k in ("weight", "bias", "running_mean", "running_var"))
            s = w * torch.rsqrt(rv + 1e-5)
            sh = torch.zeros(cout_p, dtype=torch.float64)
            sh[:len(s)] = b - rm * s
            st = (s.float().to(self.dev).contiguous(), sh.float().to(self.dev).contiguous())
            self.arena += list(st)
            self.frozen[p] = st
        return self.frozen[p]

    def _lab(self, p):
        """(device scale, bias pointers, their gradient slots) of a LAB, or None."""
        if not (self.use_lab and (p + ".lab.scale") in self.eng.params):
            return None
        pr, g = self.eng.params, self.eng.grads
        return (_p(pr[p + ".lab.scale"]), _p(pr[p + ".lab.bias"]), _p(g[p + ".lab.scale"]), _p(g[p + ".lab.bias"]))

    # ------------------------------------------------------------------ layers
    def stem1(self, p, out, sd):
        """StemBlock.stem1: 3x3 s2 conv of the f32 NCHW image (dp_stem_conv), wgrad only."""
        lib = self.lib
        self.taps[p] = out
        B, H, W = self.B, self.H, self.W
        wkey = p + ".conv.weight"
        s, sh = self._frozen(p, sd, out.cp)
        w27, _ = self.packed(wkey, 3, 0, 0, scale=s)
        lab = self._lab(p)
        if lab:
            self.labs.append((None, p))
        c = out.c

        def run(stream):
            la, lb = self.labv.get(p, (1.0, 0.0))
            return lib.dp_stem_conv(_p(self.image), B, H, W, _p(w27), _p(sh), c, 1 if lab else 0, C.c_float(la),
                                    C.c_float(lb), out.xp, out.H * out.W * out.ld, out.ld, self.code, stream)
        self.fw.op("stem1", run)
        self.cost("stem1", 2.0 * out.rows * c * 27)
        G = self.eng.grads[wkey]

        def bwd():
            bw = self.bw
            dz = self._dz(out.rows, out.cp)
            self._act_bwd(bw, "stem1", out, dz, s, lab, True)
            K = 27
            col = self._colbuf(out.rows * K)
            bw.op("stem1.im2col", lib.dp_im2col, _p(self.image), 3 * H * W, 1, H * W, B, H, W, 3, 3, 3, 2, 1, out.H,
                  out.W, _p(col), DP_F32, self.code)
            self.gemm(bw, "stem1.dW", dz.xp, 1, dz.ld, _p(col), K, 1, _p(G), K, c, K, out.rows, out_code=DP_F32,
                      beta=1.0)
        self._bwd.append(bwd)

    def _act_bwd(self, bw, name, out, dz, s, lab, act, res=None):
        """dz = d conv-output from out's gradient through LAB / ReLU / the frozen scale (res: the
        residual the stored output includes)."""
        la, lb, gla, glb = lab if lab else (None, None, None, None)
        bw.op(name + ".act_bwd", self.lib.dp_frozen_act_bwd, out.xp, out.ld, res.xp if res is not None else None,
              res.ld if res is not None else 0, out.gp, out.ld, dz.xp, dz.ld, out.rows, out.c,
              _lib.DP_ACT_RELU if act else _lib.DP_ACT_NONE, la, lb, _p(s), gla, glb, self.code)

    def cba(self, p, x, out, sd, k=1, stride=1, pad=None, dw=False, act=True, res=None):
        """ConvBNAct (hgnetv2.py:82-134) from x into out (+ res, the HG block's identity)."""
        lib = self.lib
        self.taps[p] = out
        name = p[len(B_):]
        wkey = p + ".conv.weight"
        w = self.eng.params[wkey]
        cout = w.shape[0]
        pad = (k - 1) // 2 if pad is None else pad
        B, H, W_ = x.B, x.H, x.W
        oh, ow = out.H, out.W
        assert out.c == cout and (dw or w.shape[1] == x.c)
        s, sh = self._frozen(p, sd, out.cp)
        lab = self._lab(p) if act else None
        d = ConvDesc()
        d.in_, d.in_bstride, d.in_pstride, d.in_h, d.in_w, d.cin = x.xp, H * W_ * x.ld, x.ld, H, W_, x.cp
        d.kh, d.kw, d.stride, d.pad_t, d.pad_l = k, k, stride, pad, pad
        d.out, d.out_bstride, d.out_pstride, d.out_h, d.out_w, d.cout = out.xp, oh * ow * out.ld, out.ld, oh, ow, out.cp
        d.bias = _p(sh)
        if res is not None:
            d.res, d.res_bstride, d.res_pstride = res.xp, oh * ow * res.ld, res.ld
        d.batch, d.act, d.dtype = B, _lib.DP_ACT_RELU if act else _lib.DP_ACT_NONE, self.code
        if lab:
            d.has_lab, d.lab_scale, d.lab_bias = 1, 1.0, 0.0
            self.labs.append((d, p))
        if dw:
            assert x.cp == out.cp and x.c == out.c
            taps, _ = self.packed(wkey, 2, 0, 0, scale=s)
            d.weight, d.kpad = _p(taps), 0
            self.fw.keep.append(d)
            self.fw.op(name, lib.dp_dwconv2d, C.byref(d))
            self.cost(name, 2.0 * out.rows * cout * k * k)
        else:
            wf, kpad = self.packed(wkey, 0, x.cp, out.cp, scale=s)
            d.weight, d.kpad = _p(wf), kpad
            self.fw.keep.append(d)
            self.fw.op(name, lib.dp_conv2d, C.byref(d))
            self.cost(name, 2.0 * out.rows * cout * k * k * x.c)
        G = self.eng.grads[wkey]
        cin = x.c

        def bwd():
            bw = self.bw
            if res is not None:
                bw.op(name + ".dres", lib.dp_axpby_rows, res.gp, res.ld, out.gp, out.ld, C.c_float(1.0), None, 0,
                      C.c_float(0.0), out.rows, cout, 1, self.code)
            dz = self._dz(out.rows, out.cp)
            if out.cp != cout:   # the rotated-weight dgrad conv reads the pads
                bw.op(name + ".dz0", lib.dp_zero, dz.xp, out.rows * out.cp * self.es)
            self._act_bwd(bw, name, out, dz, s, lab, act, res)
            if dw:
                taps_raw, _ = self.packed(wkey, 2, 0, 0)
                bw.op(name + ".dw_bwd", lib.dp_dwconv_bwd, x.xp, H * W_ * x.ld, x.ld, dz.xp, oh * ow * dz.ld, dz.ld,
                      _p(taps_raw), B, H, W_, cout, k, stride, pad, oh, ow, x.gp, H * W_ * x.ld, x.ld, _p(G), self.code)
                return
            if k == 1 and stride == 1:
                self.gemm(bw, name + ".dW", dz.xp, 1, dz.ld, x.xp, x.ld, 1, _p(G), cin, cout, cin, out.rows,
                          out_code=DP_F32, beta=1.0)
                wb, kpad2 = self.packed(wkey, 1, dz.cp, x.cp)   # the transposed weights: dx += dz W
                self._dgrad_conv(bw, name, dz, wb, kpad2, x, 1, 0)
                return
            K = cin * k * k
            self.wgrad_kxk(bw, name, x.xp, x.ld, B, H, W_, cin, dz.xp, dz.ld, oh, ow, cout, k, stride, pad, G)
            if stride == 1:
                wb, kpad2 = self.packed(wkey, 1, dz.cp, x.cp)
                self._dgrad_conv(bw, name, dz, wb, kpad2, x, k, k - 1 - pad)
            else:   # strided dense conv (stem3): dcol = dz W, then col2im
                dcol = self._dcolbuf(out.rows * K)
                self._dcol_conv(bw, name, dz, cout, cin, k, wkey, dcol, out.rows)
                bw.op(name + ".col2im", lib.dp_col2im, _p(dcol), B, H, W_, cin, k, k, stride, pad, oh, ow, x.gp,
                      H * W_ * x.ld, x.ld, 1, self.code)
        self._bwd.append(bwd)

    def _dgrad_conv(self, bw, name, dz, wb, kpad2, x, k, pad):
        """x.g += the stride-1 conv of dz (of x's spatial size) with the rotated packing wb."""
        B, H, W_ = x.B, x.H, x.W
        dd = ConvDesc()
        dd.in_, dd.in_bstride, dd.in_pstride, dd.in_h, dd.in_w, dd.cin = dz.xp, H * W_ * dz.ld, dz.ld, H, W_, dz.cp
        dd.weight, dd.kpad, dd.bias = _p(wb), kpad2, None
        dd.kh, dd.kw, dd.stride, dd.pad_t, dd.pad_l = k, k, 1, pad, pad
        dd.out, dd.out_bstride, dd.out_pstride, dd.out_h, dd.out_w, dd.cout = x.gp, H * W_ * x.ld, x.ld, H, W_, x.cp
        dd.res, dd.res_bstride, dd.res_pstride = x.gp, H * W_ * x.ld, x.ld
        dd.batch, dd.act, dd.dtype = B, _lib.DP_ACT_NONE, self.code
        bw.keep.append(dd)
        bw.op(name + ".dx", self.lib.dp_conv2d, C.byref(dd))
        self.cost(name + ".dx", 2.0 * x.rows * x.c * k * k * dz.c)

    def _dcol_conv(self, bw, name, dz, cout, cin, k, wkey, dcol, rows):
        """dcol = dz W ([rows][cout] x [cout][k*k*cin], columns tap-major (ky, kx, ci): the order
        dp_col2im reads, so its lanes load consecutive entries) on the 1x1 conv kernel: W^T packed
        [K][pad64(cout)] by dp_conv_pack mode 4."""
        K = cin * k * k
        key = (wkey, "T")
        if key not in self._packs:
            w = self.eng.params[wkey]
            kpad = pad_to(cout, 64)
            t = torch.zeros(K, kpad, dtype=self.dt, device=self.dev)
            self.arena.append(t)
            self._packs[key] = (t, kpad)
            self.pk.op(f"pack.{wkey}.T", self.lib.dp_conv_pack, _p(w), cout, cin, k, k, _p(t), kpad, 0, 4, None,
                       self.code)
        t, kpad = self._packs[key]
        d = ConvDesc()
        d.in_, d.in_bstride, d.in_pstride, d.in_h, d.in_w, d.cin = dz.xp, rows * dz.ld, dz.ld, 1, rows, cout
        d.weight, d.kpad, d.bias = _p(t), kpad, None
        d.kh, d.kw, d.stride, d.pad_t, d.pad_l = 1, 1, 1, 0, 0
        d.out, d.out_bstride, d.out_pstride, d.out_h, d.out_w, d.cout = _p(dcol), rows * K, K, 1, rows, K
        d.batch, d.act, d.dtype = 1, _lib.DP_ACT_NONE, self.code
        bw.keep.append(d)
        bw.op(name + ".dcol", self.lib.dp_conv2d, C.byref(d))
        self.cost(name + ".dcol", 2.0 * rows * cout * K)

    def _dz(self, rows, cp):
        """d conv-output of one layer's backward: a view of one shared buffer (the layers'
        backward ops run in stream order)."""
        n = rows * cp
        if getattr(self, "_dzt", None) is None or self._dzt.numel() < n:
            self._dzt = torch.empty(n, dtype=self.dt, device=self.dev)
            self.arena.append(self._dzt)
        from .encoder_train import Buf
        return V(Buf(self._dzt[:n].view(rows, cp)), 0, cp, cp, cp, 1, 1, rows)

    def _dcolbuf(self, n):
        if getattr(self, "_dcol", None) is None or self._dcol.numel() < n:
            self._dcol = torch.empty(n, dtype=self.dt, device=self.dev)
            self.arena.append(self._dcol)
        return self._dcol

    def maxpool(self, name, x, out):
        lib = self.lib
        B, h, w, c = x.B, x.H, x.W, x.c
        self.fw.op(name, lib.dp_maxpool2x2_pad_rb, x.xp, h * w * x.ld, x.ld, B, h, w, c, out.xp, h * w * out.ld, out.ld,
                   self.code)
        self._bwd.append(lambda: self.bw.op(name + ".bwd", lib.dp_maxpool2x2_pad_rb_bwd, x.xp, h * w * x.ld, x.ld,
                                            out.gp, h * w * out.ld, out.ld, B, h, w, c, x.gp, h * w * x.ld, x.ld,
                                            self.code))

    # ------------------------------------------------------------------ run
    def sync_lab(self):
        """The LAB scalars' current values into the forward descriptors (one device -> host copy)."""
        if not self.labs:
            return
        pr = self.eng.params
        keys = sorted({p for _, p in self.labs})
        vals = torch.stack([torch.cat([pr[p + ".lab.scale"], pr[p + ".lab.bias"]]) for p in keys]).cpu().tolist()
        self.labv = {p: (v[0], v[1]) for p, v in zip(keys, vals)}
        for d, p in self.labs:
            if d is not None:
                d.lab_scale, d.lab_bias = self.labv[p]

    def set_image(self, images):
        if images.data_ptr() != self.image.data_ptr():
            self.image.copy_(images.to(torch.float32))

    def forward(self, debug=None, pack=True):
        """pack=False: the weight packs of an earlier sub-batch of the same step are current."""
        self.sync_lab()
        if pack:
            self.pk.run(debug=debug)
        self.fw.run(debug=debug)
