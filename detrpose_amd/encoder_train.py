"""The HybridEncoder's training step on the HIP kernels (BASELINE config 5, the encoder half):
training-mode forward (BatchNorm2d on batch statistics, SyncBN across ranks, running statistics
updated) and the backward through every encoder parameter down to d loss / d backbone features.

Reference: HybridEncoder.forward (src/models/detrpose/hybrid_encoder.py:462-507) with its modules
in training mode: input_proj conv + BatchNorm2d (357-366), the AIFI TransformerEncoderLayer
(244-296: post-norm, GELU FFN, dropout 0), the FPN lateral ConvNormLayer + nearest x2 + concat +
RepNCSPELAN4 (192-212; CSPLayer 215-240 of VGGBlocks 139-154), the PAN SCDown (130-137) + concat +
RepNCSPELAN4. sync_bn (include/detrpose_hgnetv2.py:18, dist_utils.py:122) makes every BatchNorm2d
a SyncBatchNorm: per-rank statistics combined across ranks in the forward, the backward's two
reduction sums all-reduced.

The reference runs this through torch autograd; here the forward records a fixed tape of C-ABI
launches, each op registering its backward, and the backward tape is those in reverse:

  conv k x k s1   dp_conv2d on weights packed per step from the f32 master (dp_conv_pack mode 0);
                  input gradient = dp_conv2d of dz with the 180-degree-rotated packing (mode 1;
                  1x1: the transposed weights) accumulated through its residual input; wgrad =
                  dp_gemm (dz^T x, split-K f32 atomics; 3x3 over dp_im2col)
  conv 1x1 over   dp_gemm forward / dgrad / wgrad on the reference weight layout [cout][cin],
  a padded concat one GEMM per segment (DETRPose-N's 21-channel CSP outputs)
  depthwise s2    dp_dwconv2d / dp_dwconv_bwd
  BatchNorm2d     dp_bn_stats (+ all-reduce of the per-rank parts) + dp_bn_finalize, then
  (+ act, + sum)  dp_bn_act_fwd (one or two branches: VGGBlock, the CSP sum fused);
                  backward dp_bn_act_bwd_reduce (+ all-reduce of the sums) + dp_bn_act_bwd_apply
  AIFI            dp_gemm + dp_attn_fwd / dp_attn_bwd + dp_ln_fwd / dp_ln_bwd + dp_act_bwd (GELU)
  concat          free: producers write their channel slice of the consumer's input buffer
  nearest x2      dp_upsample2x forward / backward

Channel counts that are not a vector multiple (DETRPose-N's c4 = 21) are stored padded to 8
(16 bytes of bf16) with zero pads: packed 3x3 weights carry zero rows / columns there, the row
kernels touch only the real channels, and no gradient is ever written to a pad.
Activations and activation gradients are of the engine's dtype; statistics, parameters and
their gradients f32 (the TrainEngine's flat buffers, reference names).
"""
from __future__ import annotations

import ctypes as C
import os

import numpy as np
import torch

from . import _lib
from ._lib import DP_BF16, DP_F32, ConvDesc, contiguous_rows, rowmap
from .hybrid_encoder import sine_pos_embed_2d

E_ = "encoder."
ACT = {"silu": _lib.DP_ACT_SILU, "relu": _lib.DP_ACT_RELU, "gelu": _lib.DP_ACT_GELU, None: _lib.DP_ACT_NONE}


def pad_to(c: int, v: int) -> int:
    return (c + v - 1) // v * v


def _p(t, off=0):
    return t.data_ptr() + off * t.element_size()


class Buf:
    """A stored activation (x) and, once the backward is recorded, its gradient (g): same shape."""

    def __init__(self, x):
        self.x, self.g = x, None


class V:
    """Channel slice [c0, c0 + cp) of an NHWC map stored as rows (B*H*W) of row stride ld; c
    real channels (cp >= c: the padded width the convs see)."""

    def __init__(self, buf, off, ld, c, cp, B, H, W):
        self.buf, self.off, self.ld, self.c, self.cp, self.B, self.H, self.W = buf, off, ld, c, cp, B, H, W

    @property
    def rows(self):
        return self.B * self.H * self.W

    @property
    def xp(self):
        return _p(self.buf.x, self.off)

    @property
    def gp(self):
        return _p(self.buf.g, self.off)

    def ch(self, c0, c, cp=None):
        return V(self.buf, self.off + c0, self.ld, c, c if cp is None else cp, self.B, self.H, self.W)


COMM_LOG = None   # when a list: every all_reduce is synchronised and timed into it (bench.py's train leg)


def all_reduce(t, async_op=False, group=None):
    """Sum over the ranks in place (RCCL on device tensors; host-staged under gloo, whose
    collectives take host tensors: the one-GPU multi-rank rehearsal and tests). async_op: return
    the RCCL work handle (wait() before reading t); host-staged reductions complete here (None)."""
    if COMM_LOG is not None:
        import time
        torch.cuda.synchronize(t.device) if t.is_cuda else None
        t0 = time.perf_counter()
        _all_reduce(t, False, group)
        torch.cuda.synchronize(t.device) if t.is_cuda else None
        COMM_LOG.append((t.numel() * t.element_size(), time.perf_counter() - t0))
        return None
    return _all_reduce(t, async_op, group)


def _all_reduce(t, async_op, group=None):
    if torch.distributed.get_backend(group) == "gloo" and t.is_cuda:
        h = t.cpu()
        torch.distributed.all_reduce(h, group=group)
        t.copy_(h)
        return None
    w = torch.distributed.all_reduce(t, async_op=async_op, group=group)
    return w if async_op else None


def _host(fn):
    """A tape op that runs host code (a collective) in stream order (keeps its tape eager)."""
    def op(stream):
        fn()
        return 0
    op.host = True
    return op


class TapePlan:
    """Shared machinery of the conv-network training tapes (encoder_train.EncoderTrainPlan,
    backbone_train.BackboneTrainPlan): stored NHWC maps with gradient buffers, per-step weight
    packing from the f32 master, the conv / BatchNorm ops that register their backward."""

    def _setup(self, eng):
        self.eng = eng
        self.lib = eng.lib
        self.model = eng.model
        self.dt, self.code = eng.tdtype, eng.code
        self.es = self.dt.itemsize
        self.vec = 8 if self.code == DP_BF16 else 4
        self.dev = eng.device
        self.op_flops = {}
        # stored layer outputs by reference prefix (the forced-state parity test reads them,
        # tests/test_gpu_full_train_step_l.py; the oracle's TAP names)
        self.taps = {}
        self.arena, self.bufs = [], []
        self._bwd = []
        self.world, self.rank = 1, 0
        if torch.distributed.is_available() and torch.distributed.is_initialized():
            self.world, self.rank = torch.distributed.get_world_size(), torch.distributed.get_rank()
        self.fw, self.bw = _lib_tape(self.lib, self.dev), _lib_tape(self.lib, self.dev)
        self.fw.deterministic = True
        # the weight packs (bf16 copies / conv layouts of the f32 master) on a tape of their own:
        # run once per optimizer step, not once per grad_accum sub-batch (forward(pack=False))
        self.pk = _lib_tape(self.lib, self.dev)
        self._packs = {}
        self._col = None

    # ------------------------------------------------------------------ storage
    def f32(self, *shape):
        t = torch.empty(*shape, dtype=torch.float32, device=self.dev)
        self.arena.append(t)
        return t

    def view(self, B, H, W, c):
        """A fresh zeroed NHWC map (pads stay zero for good), channels padded to 8."""
        cp = pad_to(c, 8)
        b = Buf(torch.zeros(B * H * W, cp, dtype=self.dt, device=self.dev))
        self.bufs.append(b)
        return V(b, 0, cp, c, cp, B, H, W)

    def scratch(self, rows, c):
        """A map without a gradient of its own (backward scratch)."""
        t = torch.empty(rows, c, dtype=self.dt, device=self.dev)
        self.arena.append(t)
        return V(Buf(t), 0, c, c, c, 1, 1, rows)

    def cost(self, name, flops):
        self.op_flops[name] = self.op_flops.get(name, 0.0) + flops

    def batch_packs(self):
        """The pack tape's launches merged into one (Tape.batch_packs; DETRPOSE_PACK_BATCH=0 keeps
        one launch per weight, A/B)."""
        if os.environ.get("DETRPOSE_PACK_BATCH", "1") != "0":
            self.pk.batch_packs()

    def _record_backward(self, zero=True, extra_zero=()):
        """Gradient buffers for every stored map (one arena), then the ops in reverse. The
        backward starts by zeroing the arena (zero=False: a later plan's backward zeroes it
        before accumulating into this plan's outputs: extra_zero = those arenas)."""
        total = sum(b.x.numel() for b in self.bufs)
        self.grad_arena = torch.empty(total, dtype=self.dt, device=self.dev)
        o = 0
        for b in self.bufs:
            n = b.x.numel()
            b.g = self.grad_arena[o:o + n].view(b.x.shape)
            o += n
        for i, t in enumerate(([self.grad_arena] if zero else []) + list(extra_zero)):
            self.bw.op(f"grads.zero{i}", self.lib.dp_zero, _p(t), t.numel() * t.element_size())
        for fn in reversed(self._bwd):
            fn()

    # ------------------------------------------------------------------ weights
    def wptr(self, key):
        """The dtype copy of a 1x1 conv / linear weight in the reference layout (the master
        itself in fp32 mode; a bf16 copy refreshed at the start of each forward)."""
        if self.code == DP_F32:
            return _p(self.eng.params[key])
        if key not in self._packs:
            src = self.eng.params[key]
            t = torch.empty(src.numel(), dtype=self.dt, device=self.dev)
            self.arena.append(t)
            self._packs[key] = t
            self.pk.op("pack." + key, self.lib.dp_convert_rows, _p(src), DP_F32, src.numel(), _p(t), self.code,
                       src.numel(), 1, src.numel(), C.c_float(1.0), 0)
        return _p(self._packs[key])

    def packed(self, key, mode, kc, rows_p, scale=None):
        """dp_conv_pack of the master weight: mode 0 / 1 [rows_p][kpad] of dtype (zero pads),
        mode 2 f32 depthwise taps, mode 3 f32 [cout][cin*kh*kw]; scale: f32 [cout] multiplier
        (a frozen BatchNorm's scale folded in)."""
        k2 = (key, mode, scale is not None)
        if k2 not in self._packs:
            w = self.eng.params[key]
            cout, cin, kh, kw = w.shape
            if mode in (2, 3):
                t = torch.empty(kh * kw * cout * cin, dtype=torch.float32, device=self.dev)
                kpad = 0
            else:
                kpad = pad_to(kh * kw * kc, 64)
                t = torch.zeros(rows_p, kpad, dtype=self.dt, device=self.dev)
            self.arena.append(t)
            self._packs[k2] = (t, kpad)
            self.pk.op(f"pack.{key}.{mode}", self.lib.dp_conv_pack, _p(w), cout, cin, kh, kw, _p(t), kpad, kc, mode,
                       _p(scale) if scale is not None else None, self.code if mode < 2 else DP_F32)
        return self._packs[k2]

    # ------------------------------------------------------------------ GEMM helper
    def gemm(self, tape, name, a, a_rs, a_ks, b, b_ks, b_ns, c, c_rs, m, n, k, out_code=None, bias=None, beta=0.0,
             act=0, colsum=None):
        self.eng._gemm(tape, name, a, a_rs, a_ks, b, b_ks, b_ns, c, c_rs, m, n, k, self.code,
                       self.code if out_code is None else out_code, bias=bias, beta=beta, act=act, colsum=colsum)

    # ------------------------------------------------------------------ layers
    def conv(self, name, wkey, segs, cout, k=1):
        """z = conv(x) without bias (every ConvNormLayer conv here is bias-free). 1x1: segs =
        [(view, k0, kc)], the weight columns k0..k0+kc applied to the view's first kc channels
        (a concat's segments). k x k (stride 1, pad k//2): one view, on dp_conv2d."""
        lib = self.lib
        x0 = segs[0][0]
        B, H, W = x0.B, x0.H, x0.W
        rows = x0.rows
        G = self.eng.grads[wkey]
        if k == 1 and len(segs) > 1:   # a padded concat read as segments: one GEMM per segment
            z = self.view(B, H, W, cout)
            Wp = self.wptr(wkey)
            cin_t = self.eng.params[wkey].shape[1]
            e = self.es
            for i, (x, k0, kc) in enumerate(segs):
                self.gemm(self.fw, f"{name}.conv{i}", x.xp, x.ld, 1, Wp + k0 * e, 1, cin_t, z.xp, z.ld, rows, cout, kc,
                          beta=1.0 if i else 0.0)

            def bwd():
                for i, (x, k0, kc) in enumerate(segs):
                    self.gemm(self.bw, f"{name}.dW{i}", z.gp, 1, z.ld, x.xp, x.ld, 1, _p(G, k0), cin_t, cout, kc, rows,
                              out_code=DP_F32, beta=1.0)
                    self.gemm(self.bw, f"{name}.dx{i}", z.gp, z.ld, 1, Wp + k0 * e, cin_t, 1, x.gp, x.ld, rows, kc,
                              cout, beta=1.0)
            self._bwd.append(bwd)
            return z
        (x, _, _), = segs
        assert x.cp % self.vec == 0 and x.ld % self.vec == 0
        z = self.view(B, H, W, cout)
        wf, kpad = self.packed(wkey, 0, x.cp, z.cp)
        self._conv2d(self.fw, name, x.xp, x.ld, x.cp, z.xp, z.ld, z.cp, wf, kpad, B, H, W, k)
        wb, kpad2 = self.packed(wkey, 1, z.cp, x.cp)
        cin = x.c

        def bwd():
            # input gradient: conv of dz with the rotated weights (1x1: the transposed weights),
            # accumulated (residual = itself)
            self._conv2d(self.bw, name + ".dx", z.gp, z.ld, z.cp, x.gp, x.ld, x.cp, wb, kpad2, B, H, W, k, res=x.gp)
            if k == 1:
                self.gemm(self.bw, name + ".dW", z.gp, 1, z.ld, x.xp, x.ld, 1, _p(G), cin, cout, cin, rows,
                          out_code=DP_F32, beta=1.0)
                return
            self.wgrad_kxk(self.bw, name, x.xp, x.ld, B, H, W, cin, z.gp, z.ld, H, W, cout, k, 1, k // 2, G)
        self._bwd.append(bwd)
        return z

    def wgrad_kxk(self, bw, name, xp, x_ld, B, H, W, cin, dzp, dz_ld, oh, ow, cout, k, stride, pad, G):
        """dW += the k x k conv's weight gradient: bf16 with 8-channel pixels on dp_conv_wgrad
        (implicit GEMM, no im2col columns), else dp_im2col + dp_gemm (dz^T col)."""
        lib = self.lib
        if self.code == DP_BF16 and cin % 8 == 0 and x_ld % 8 == 0 and dz_ld % 8 == 0:
            # zeroed once here and left zeroed by every call (dp_conv_wgrad_zs): no zero-fill launch
            scratch = self.f32(cout * cin * k * k).zero_()
            bw.op(name + ".dW", lib.dp_conv_wgrad_zs, xp, H * W * x_ld, x_ld, B, H, W, cin, dzp, dz_ld, oh, ow, cout, k,
                  k, stride, pad, _p(scratch), _p(G), self.code)
            self.cost(name + ".dW", 2.0 * B * oh * ow * cout * cin * k * k)
            return
        K = cin * k * k
        rows = B * oh * ow
        col = self._colbuf(rows * K)
        bw.op(name + ".im2col", lib.dp_im2col, xp, H * W * x_ld, x_ld, 1, B, H, W, cin, k, k, stride, pad, oh, ow,
              _p(col), self.code, self.code)
        self.gemm(bw, name + ".dW", dzp, 1, dz_ld, _p(col), K, 1, _p(G), K, cout, K, rows, out_code=DP_F32, beta=1.0)

    def _colbuf(self, n):
        if self._col is None or self._col.numel() < n:
            self._col = torch.empty(n, dtype=self.dt, device=self.dev)
            self.arena.append(self._col)
        return self._col

    def _conv2d(self, tape, name, xin, ld_in, cin, out, ld_out, cout, wt, kpad, B, H, W, k, res=None):
        d = ConvDesc()
        d.in_, d.in_bstride, d.in_pstride, d.in_h, d.in_w, d.cin = xin, H * W * ld_in, ld_in, H, W, cin
        d.weight, d.kpad, d.bias = _p(wt), kpad, None
        d.kh, d.kw, d.stride, d.pad_t, d.pad_l = k, k, 1, k // 2, k // 2
        d.out, d.out_bstride, d.out_pstride, d.out_h, d.out_w, d.cout = out, H * W * ld_out, ld_out, H, W, cout
        if res is not None:
            d.res, d.res_bstride, d.res_pstride = res, H * W * ld_out, ld_out
        d.batch, d.act, d.dtype = B, _lib.DP_ACT_NONE, self.code
        tape.keep.append(d)
        tape.op(name, self.lib.dp_conv2d, C.byref(d))
        self.cost(name, 2.0 * B * H * W * cout * k * k * cin)

    def dwconv(self, name, wkey, x, stride):
        """SCDown's depthwise k x k stride-s conv (groups = channels, bias-free)."""
        lib = self.lib
        w = self.eng.params[wkey]
        c, _, k, _ = w.shape
        B, H, W = x.B, x.H, x.W
        oh, ow = (H + 2 * (k // 2) - k) // stride + 1, (W + 2 * (k // 2) - k) // stride + 1
        z = self.view(B, oh, ow, c)
        taps, _ = self.packed(wkey, 2, 0, 0)
        d = ConvDesc()
        d.in_, d.in_bstride, d.in_pstride, d.in_h, d.in_w, d.cin = x.xp, H * W * x.ld, x.ld, H, W, c
        d.weight, d.kpad, d.bias = _p(taps), 0, _p(self.zero_bias)
        d.kh, d.kw, d.stride, d.pad_t, d.pad_l = k, k, stride, k // 2, k // 2
        d.out, d.out_bstride, d.out_pstride, d.out_h, d.out_w, d.cout = z.xp, oh * ow * z.ld, z.ld, oh, ow, c
        d.batch, d.act, d.dtype = B, _lib.DP_ACT_NONE, self.code
        self.fw.keep.append(d)
        self.fw.op(name, lib.dp_dwconv2d, C.byref(d))
        G = self.eng.grads[wkey]

        def bwd():
            self.bw.op(name + ".bwd", lib.dp_dwconv_bwd, x.xp, H * W * x.ld, x.ld, z.gp, oh * ow * z.ld, z.ld, _p(taps),
                       B, H, W, c, k, stride, k // 2, oh, ow, x.gp, H * W * x.ld, x.ld, _p(G), self.code)
        self._bwd.append(bwd)
        return z

    def bn(self, name, branches, out, act, res=None, tap=None):
        """out = act(sum_k BN_k(z_k)) [+ res], BatchNorm2d on batch statistics (SyncBN over the
        ranks), running statistics updated. branches: [(z view, BN prefix)] (one or two). tap:
        the reference prefix `out` is stored under in self.taps (default: the layer's, from the
        BN prefix)."""
        lib, eng = self.lib, self.eng
        if tap is None:
            tap = branches[0][1][:-len(".norm")]
            if len(branches) > 1:
                tap = tap[:-len(".conv1")]
        self.taps[tap] = out
        c = out.c
        rows = out.rows
        code = self.code
        fw = self.fw
        st = []
        for bi, (z, p) in enumerate(branches):
            parts = self.f32(self.world, 3, c)
            mr = self.f32(2, c)
            if self.world > 1:
                fw.op(f"{name}.bn{bi}.zero", lib.dp_zero, _p(parts), parts.numel() * 4)
            ws = self.f32(max(int(lib.dp_bn_stats_ws_bytes(rows, c)), 4) // 4)   # per-slice partial sums
            rm, rv = eng.running[p + ".running_mean"], eng.running[p + ".running_var"]
            if self.world == 1:   # statistics + finalize in the statistics' launches
                fw.op(f"{name}.bn{bi}.stats", lib.dp_bn_stats_finalize, z.xp, z.ld, rows, c, _p(parts), _p(ws),
                      ws.numel() * 4, C.c_float(1e-5), C.c_float(0.1), _p(rm), _p(rv), _p(mr), code)
            else:
                fw.op(f"{name}.bn{bi}.stats", lib.dp_bn_stats, z.xp, z.ld, rows, c, _p(parts[self.rank]), _p(ws),
                      ws.numel() * 4, code)
                fw.op(f"{name}.bn{bi}.sync", _host(lambda t=parts: all_reduce(t)))
                fw.op(f"{name}.bn{bi}.finalize", lib.dp_bn_finalize, _p(parts), self.world, C.c_float(rows), c,
                      C.c_float(1e-5), C.c_float(0.1), _p(rm), _p(rv), _p(mr))
            st.append((z, mr, eng.params[p + ".weight"], eng.params[p + ".bias"], eng.grads[p + ".weight"],
                       eng.grads[p + ".bias"]))
        z1, mr1, g1, b1, dg1, db1 = st[0]
        two = len(st) > 1
        z2, mr2, g2, b2, dg2, db2 = st[1] if two else (None,) * 6
        N = None
        fw.op(name + ".bn_act", lib.dp_bn_act_fwd, out.xp, out.ld, z1.xp, z1.ld, _p(mr1), _p(g1), _p(b1),
              z2.xp if two else N, z2.ld if two else 0, _p(mr2) if two else N, _p(g2) if two else N,
              _p(b2) if two else N, res.xp if res is not None else N, res.ld if res is not None else 0, rows, c, ACT[act],
              code)
        sums = self.f32(3, c)

        def bwd():
            bw = self.bw
            if res is not None:   # the CSP sum: d res += d out
                bw.op(name + ".dres", lib.dp_axpby_rows, res.gp, res.ld, out.gp, out.ld, C.c_float(1.0), N, 0,
                      C.c_float(0.0), rows, c, 1, code)
            rws = self.f32(max(int(lib.dp_bn_act_bwd_reduce_ws_bytes(rows, c)), 4) // 4)   # per-slice partials
            bw.op(name + ".bn_reduce", lib.dp_bn_act_bwd_reduce, out.gp, out.ld, z1.xp, z1.ld, _p(mr1), _p(g1), _p(b1),
                  z2.xp if two else N, z2.ld if two else 0, _p(mr2) if two else N, _p(g2) if two else N,
                  _p(b2) if two else N, rows, c, ACT[act], _p(sums), _p(dg1), _p(db1), _p(dg2) if two else N,
                  _p(db2) if two else N, _p(rws), rws.numel() * 4, code)
            if self.world > 1:
                bw.op(name + ".bn_sync", _host(lambda: all_reduce(sums)))
            bw.op(name + ".bn_apply", lib.dp_bn_act_bwd_apply, z1.gp, z1.ld, z2.gp if two else N, z2.ld if two else 0,
                  out.gp, out.ld, z1.xp, z1.ld, _p(mr1), _p(g1), _p(b1), z2.xp if two else N, z2.ld if two else 0,
                  _p(mr2) if two else N, _p(g2) if two else N, _p(b2) if two else N, rows, c, ACT[act], _p(sums),
                  C.c_float(rows * self.world), code)
        self._bwd.append(bwd)

    def upsample(self, name, src, dst):
        """F.interpolate(scale_factor=2, nearest) into the concat slice dst (hybrid_encoder.py:487)."""
        lib = self.lib
        B, h, w, c = src.B, src.H, src.W, src.c
        self.fw.op(name, lib.dp_upsample2x, src.xp, h * w * src.ld, src.ld, B, h, w, c, dst.xp, 4 * h * w * dst.ld,
                   dst.ld, 0, self.code)
        self._bwd.append(lambda: self.bw.op(name + ".bwd", lib.dp_upsample2x, dst.gp, 4 * h * w * dst.ld, dst.ld, B, h,
                                            w, c, src.gp, h * w * src.ld, src.ld, 1, self.code))

    # ------------------------------------------------------------------ run
    def set_inputs(self, feats):
        """feats: backbone outputs, NCHW (B, cin, H, W) or NHWC rows, any float dtype."""
        for v, f in zip(self.feats, feats):
            t = f.permute(0, 2, 3, 1) if f.dim() == 4 and f.shape[1] == v.c and f.shape[-1] != v.c else f
            v.buf.x[:, :v.c].copy_(t.reshape(v.rows, v.c).to(self.dt))

    def forward(self, debug=None, pack=True):
        """pack=False: the weight packs of an earlier sub-batch of the same step are current."""
        if pack:
            self.pk.run(debug=debug)
        self.fw.run(debug=debug)

    def backward(self, debug=None):
        self.bw.run(debug=debug)




class EncoderTrainPlan(TapePlan):
    """Buffers and tapes of the encoder's training forward / backward for one batch and feature
    shape set. eng: a TrainEngine built with train_encoder=True (the encoder parameters live in
    its flat master / gradient buffers)."""

    def __init__(self, eng, B: int, feat_shapes, feats=None, feats_plan=None):
        """feats: the backbone's output maps (backbone_train.BackboneTrainPlan.outs, their
        gradients d loss / d feats accumulated by this backward; feats_plan: that plan, whose
        gradient arena this backward zeroes first) or None: own input buffers (set_inputs)."""
        self._setup(eng)
        lib = self.lib
        enc = eng.model.encoder
        self.enc = enc
        self.B = B
        Cc, nlev = enc.hidden_dim, enc.n_levels
        self.Cc = Cc
        self.c4, self.c4p = enc.c4, pad_to(enc.c4, 8)
        self.hw = [tuple(s) for s in feat_shapes]
        self.S = sum(h * w for h, w in self.hw)
        fw = self.fw
        self.zero_bias = self.f32(max(enc.in_channels + [2 * Cc]))
        self.zero_bias.zero_()
        prev = getattr(eng, "cur", None)
        eng.cur = self

        # ---------------- inputs: backbone features (B*H*W, cin) NHWC rows
        if feats is not None:
            assert [(f.H, f.W, f.c) for f in feats] == [(h, w, c) for (h, w), c in zip(self.hw, enc.in_channels)]
            self.feats = list(feats)
        else:
            self.feats = [self.view(B, h, w, cin) for (h, w), cin in zip(self.hw, enc.in_channels)]
        self.memory = torch.empty(B, self.S, Cc, dtype=self.dt, device=self.dev)
        self.arena.append(self.memory)
        self.d_memory = torch.zeros(B, self.S, Cc, dtype=torch.float32, device=self.dev)
        self.arena.append(self.d_memory)

        # ---------------- forward (hybrid_encoder.py:462-507)
        hw = self.hw
        fcat = [self.view(B, *hw[i], 2 * Cc) for i in range(nlev - 1)]       # [up(lateral) | proj]
        pcat = [self.view(B, *hw[i + 1], 2 * Cc) for i in range(nlev - 1)]   # [down | lateral]
        proj = []
        for i, f in enumerate(self.feats):
            dst = fcat[i].ch(Cc, Cc) if i < nlev - 1 else self.view(B, *hw[i], Cc)
            p = f"{E_}input_proj.{i}"
            z = self.conv(f"enc.proj{i}", p + ".conv.weight", [(f, 0, f.c)], Cc)
            self.bn(f"enc.proj{i}", [(z, p + ".norm")], dst, None)
            proj.append(dst)
        for i, ei in enumerate(enc.use_encoder_idx):
            out = self.view(B, *hw[ei], Cc)
            self.aifi(i, proj[ei], out)
            proj[ei] = out
        high = proj[-1]
        self.levels = [None] * nlev
        for idx in range(nlev - 1, 0, -1):
            j = nlev - 1 - idx
            lat = pcat[idx - 1].ch(Cc, Cc)
            p = f"{E_}lateral_convs.{j}"
            z = self.conv(f"enc.lateral{j}", p + ".conv.weight", [(high, 0, Cc)], Cc)
            self.bn(f"enc.lateral{j}", [(z, p + ".norm")], lat, enc.act)
            self.upsample(f"enc.lateral{j}.up", lat, fcat[idx - 1].ch(0, Cc))
            dst = self.view(B, *hw[idx - 1], Cc)
            self.elan(f"enc.fpn{j}", f"{E_}fpn_blocks.{j}", fcat[idx - 1], dst)
            high = dst
        self.levels[0] = high
        low = high
        for idx in range(nlev - 1):
            p = f"{E_}downsample_convs.{idx}.0"
            t1 = self.view(B, low.H, low.W, Cc)
            z = self.conv(f"enc.down{idx}.cv1", p + ".cv1.conv.weight", [(low, 0, Cc)], Cc)
            self.bn(f"enc.down{idx}.cv1", [(z, p + ".cv1.norm")], t1, None)
            z2 = self.dwconv(f"enc.down{idx}.cv2", p + ".cv2.conv.weight", t1, 2)
            self.bn(f"enc.down{idx}.cv2", [(z2, p + ".cv2.norm")], pcat[idx].ch(0, Cc), None)
            dst = self.view(B, *hw[idx + 1], Cc)
            self.elan(f"enc.pan{idx}", f"{E_}pan_blocks.{idx}", pcat[idx], dst)
            self.levels[idx + 1] = dst
            low = dst
        # memory (B, S, C): the levels back to back per image (transformer.py:1285-1286)
        starts = [sum(h * w for h, w in hw[:i]) for i in range(nlev)]
        self.starts = starts
        for i, lv in enumerate(self.levels):
            n = lv.H * lv.W * Cc
            fw.op(f"enc.memory{i}", lib.dp_convert_rows, lv.xp, self.code, n, _p(self.memory, starts[i] * Cc), self.code,
                  self.S * Cc, B, n, C.c_float(1.0), 0)
            self._bwd.append(lambda lv=lv, i=i, n=n: self.bw.op(
                f"enc.memory{i}.bwd", lib.dp_convert_rows, _p(self.d_memory, starts[i] * Cc), DP_F32, self.S * Cc,
                lv.gp, self.code, n, B, n, C.c_float(1.0), 1))
        self._record_backward(extra_zero=[feats_plan.grad_arena] if feats_plan is not None else ())
        self.d_feats = [f.buf.g for f in self.feats]
        self.batch_packs()
        eng.cur = prev

    def csp(self, name, p, x, out):
        """CSPLayer (hybrid_encoder.py:215-240): conv1 -> VGG blocks, + conv2, both SiLU."""
        enc = self.enc
        B, H, W = x.B, x.H, x.W
        c4 = self.c4
        a = self.view(B, H, W, c4)
        z = self.conv(name + ".conv1", p + ".conv1.conv.weight", [(x, 0, x.c)], c4)
        self.bn(name + ".conv1", [(z, p + ".conv1.norm")], a, enc.act)
        x2 = self.view(B, H, W, c4)
        z = self.conv(name + ".conv2", p + ".conv2.conv.weight", [(x, 0, x.c)], c4)
        self.bn(name + ".conv2", [(z, p + ".conv2.norm")], x2, enc.act)
        cur = a
        nb = enc.n_blocks
        for i in range(nb):
            q = f"{p}.bottlenecks.{i}"
            z3 = self.conv(f"{name}.vgg{i}.c3", q + ".conv1.conv.weight", [(cur, 0, c4)], c4, k=3)
            z1 = self.conv(f"{name}.vgg{i}.c1", q + ".conv2.conv.weight", [(cur, 0, c4)], c4)
            dst = out if i == nb - 1 else self.view(B, H, W, c4)
            self.bn(f"{name}.vgg{i}", [(z3, q + ".conv1.norm"), (z1, q + ".conv2.norm")], dst, enc.act,
                    res=x2 if i == nb - 1 else None, tap=p if i == nb - 1 else None)
            cur = dst

    def elan(self, name, p, x, out):
        """RepNCSPELAN4 (hybrid_encoder.py:192-212) on the concat x (2C channels) into out (C):
        cv1 -> [y0 | y1], y2 = cv2(y1), y3 = cv3(y2), cv4([y0 | y1 | y2 | y3])."""
        enc = self.enc
        Cc, c4, c4p = self.Cc, self.c4, self.c4p
        B, H, W = x.B, x.H, x.W
        ecat = self.view(B, H, W, 2 * Cc + 2 * c4p)   # [cv1 out (2C) | y2 (c4p) | y3 (c4p)]
        y01 = ecat.ch(0, 2 * Cc)
        z = self.conv(name + ".cv1", p + ".cv1.conv.weight", [(x, 0, 2 * Cc)], 2 * Cc)
        self.bn(name + ".cv1", [(z, p + ".cv1.norm")], y01, enc.act)
        src = ecat.ch(Cc, Cc)
        for br, off in (("cv2", 2 * Cc), ("cv3", 2 * Cc + c4p)):
            t = self.view(B, H, W, c4)
            self.csp(f"{name}.{br}", f"{p}.{br}.0", src, t)
            dst = ecat.ch(off, c4, c4p)
            z = self.conv(f"{name}.{br}.1", f"{p}.{br}.1.conv.weight", [(t, 0, c4)], c4, k=3)
            self.bn(f"{name}.{br}.1", [(z, f"{p}.{br}.1.norm")], dst, enc.act)
            src = dst
        segs = [(ecat.ch(0, 2 * Cc), 0, 2 * Cc), (ecat.ch(2 * Cc, c4), 2 * Cc, c4),
                (ecat.ch(2 * Cc + c4p, c4), 2 * Cc + c4, c4)]
        if c4p == c4:
            segs = [(ecat.ch(0, 2 * Cc + 2 * c4), 0, 2 * Cc + 2 * c4)]
        z = self.conv(name + ".cv4", p + ".cv4.conv.weight", segs, Cc)
        self.bn(name + ".cv4", [(z, p + ".cv4.norm")], out, enc.act)

    def aifi(self, i, src, out):
        """TransformerEncoderLayer (hybrid_encoder.py:270-296, post-norm) on (B, HW, C) tokens:
        q = k = src + pos, v = src; LN(src + attn); LN(x + linear2(gelu(linear1(x))))."""
        lib, eng = self.lib, self.eng
        enc = self.enc
        Cc, nh = self.Cc, enc.nhead
        dh = Cc // nh
        B, H, W = src.B, src.H, src.W
        n = H * W
        rows = B * n
        code = self.code
        fw = self.fw
        lp = f"{E_}encoder.{i}.layers.0"
        ei = enc.use_encoder_idx[i]
        stride = enc.feat_strides[ei]
        if enc.eval_spatial_size:
            h0, w0 = enc.eval_spatial_size[0] // stride, enc.eval_spatial_size[1] // stride
        else:
            h0, w0 = H, W
        assert (h0, w0) == (H, W), "AIFI position embedding size"
        pos = sine_pos_embed_2d(W, H, Cc // 2, enc.temperatureW, enc.temperatureH).reshape(n, Cc).to(
            self.dev, self.dt).contiguous()
        self.arena.append(pos)
        assert src.ld == Cc and out.ld == Cc
        cr = contiguous_rows
        q = self.view(1, 1, rows, Cc)
        fw.op(f"aifi{i}.pos", lib.dp_add_rows, q.xp, cr(Cc), src.xp, cr(Cc), _p(pos), rowmap(0, n, 0, Cc), rows, Cc,
              code)
        Wi, bi = lp + ".self_attn.in_proj_weight", eng.params[lp + ".self_attn.in_proj_bias"]
        Wip = self.wptr(Wi)
        e = self.es
        qkv = self.view(1, 1, rows, 3 * Cc)
        self.gemm(fw, f"aifi{i}.qk", q.xp, Cc, 1, Wip, 1, Cc, qkv.xp, 3 * Cc, rows, 2 * Cc, Cc, bias=_p(bi))
        self.gemm(fw, f"aifi{i}.v", src.xp, Cc, 1, Wip + 2 * Cc * Cc * e, 1, Cc, qkv.xp + 2 * Cc * e, 3 * Cc, rows, Cc,
                  Cc, bias=_p(bi, 2 * Cc))
        att = self.view(1, 1, rows, Cc)
        Pm = self.f32(B * nh * n * n)
        fw.op(f"aifi{i}.attn", lib.dp_attn_fwd, qkv.xp, 3 * Cc, qkv.xp + Cc * e, qkv.xp + 2 * Cc * e, 3 * Cc, att.xp, Cc,
              _p(Pm), None, B, 1, n, 0, 1, n, nh, dh, code)
        self.cost(f"aifi{i}.attn", 4.0 * B * n * n * Cc)
        Wo = lp + ".self_attn.out_proj.weight"
        ao = self.view(1, 1, rows, Cc)
        self.gemm(fw, f"aifi{i}.out", att.xp, Cc, 1, self.wptr(Wo), 1, Cc, ao.xp, Cc, rows, Cc, Cc,
                  bias=_p(eng.params[lp + ".self_attn.out_proj.bias"]))
        x1, s1, st1 = self.view(1, 1, rows, Cc), self.view(1, 1, rows, Cc), self.f32(rows, 2)
        n1g, n1b = eng.params[lp + ".norm1.weight"], eng.params[lp + ".norm1.bias"]
        fw.op(f"aifi{i}.norm1", lib.dp_ln_fwd, x1.xp, Cc, src.xp, ao.xp, s1.xp, _p(st1), _p(n1g), _p(n1b),
              C.c_float(1e-5), rows, Cc, None, 1, 0, code)
        W1, W2 = lp + ".linear1.weight", lp + ".linear2.weight"
        F_ = eng.params[W1].shape[0]
        b1, b2 = eng.params[lp + ".linear1.bias"], eng.params[lp + ".linear2.bias"]
        pre, h = self.view(1, 1, rows, F_), self.view(1, 1, rows, F_)
        W1p, W2p = self.wptr(W1), self.wptr(W2)
        act = ACT[enc.enc_act]
        self.gemm(fw, f"aifi{i}.linear1", x1.xp, Cc, 1, W1p, 1, Cc, pre.xp, F_, rows, F_, Cc, bias=_p(b1))
        self.gemm(fw, f"aifi{i}.linear1.act", x1.xp, Cc, 1, W1p, 1, Cc, h.xp, F_, rows, F_, Cc, bias=_p(b1), act=act)
        f = self.view(1, 1, rows, Cc)
        self.gemm(fw, f"aifi{i}.linear2", h.xp, F_, 1, W2p, 1, F_, f.xp, Cc, rows, Cc, F_, bias=_p(b2))
        self.taps[lp] = out
        s2, st2 = self.view(1, 1, rows, Cc), self.f32(rows, 2)
        n2g, n2b = eng.params[lp + ".norm2.weight"], eng.params[lp + ".norm2.bias"]
        fw.op(f"aifi{i}.norm2", lib.dp_ln_fwd, out.xp, Cc, x1.xp, f.xp, s2.xp, _p(st2), _p(n2g), _p(n2b),
              C.c_float(1e-5), rows, Cc, None, 1, 0, code)
        G = eng.grads
        # the backward's own scratch (gradients of non-stored intermediates)
        ds, dh_, dsum1 = self.scratch(rows, Cc), self.scratch(rows, F_), self.scratch(rows, Cc)
        datt, dqkv = self.scratch(rows, Cc), self.scratch(rows, 3 * Cc)

        def bwd():
            bw = self.bw
            bw.op(f"aifi{i}.norm2.bwd", lib.dp_ln_bwd, ds.xp, out.gp, Cc, s2.xp, _p(st2), _p(n2g), rows, Cc,
                  _p(G[lp + ".norm2.weight"]), _p(G[lp + ".norm2.bias"]), 0, code)
            self.gemm(bw, f"aifi{i}.linear2.dW", ds.xp, 1, Cc, h.xp, F_, 1, _p(G[W2]), F_, Cc, F_, rows,
                      out_code=DP_F32, beta=1.0, colsum=_p(G[lp + ".linear2.bias"]))
            self.gemm(bw, f"aifi{i}.linear2.dx", ds.xp, Cc, 1, W2p, F_, 1, dh_.xp, F_, rows, F_, Cc)
            bw.op(f"aifi{i}.act.bwd", lib.dp_act_bwd, pre.xp, F_, dh_.xp, F_, dh_.xp, F_, rows, F_, act, code)
            self.gemm(bw, f"aifi{i}.linear1.dW", dh_.xp, 1, F_, x1.xp, Cc, 1, _p(G[W1]), Cc, F_, Cc, rows,
                      out_code=DP_F32, beta=1.0, colsum=_p(G[lp + ".linear1.bias"]))
            self.gemm(bw, f"aifi{i}.linear1.dx", dh_.xp, F_, 1, W1p, Cc, 1, ds.xp, Cc, rows, Cc, F_, beta=1.0)
            bw.op(f"aifi{i}.norm1.bwd", lib.dp_ln_bwd, dsum1.xp, ds.xp, Cc, s1.xp, _p(st1), _p(n1g), rows, Cc,
                  _p(G[lp + ".norm1.weight"]), _p(G[lp + ".norm1.bias"]), 0, code)
            self.gemm(bw, f"aifi{i}.out.dW", dsum1.xp, 1, Cc, att.xp, Cc, 1, _p(G[Wo]), Cc, Cc, Cc, rows,
                      out_code=DP_F32, beta=1.0, colsum=_p(G[lp + ".self_attn.out_proj.bias"]))
            self.gemm(bw, f"aifi{i}.out.dx", dsum1.xp, Cc, 1, self.wptr(Wo), Cc, 1, datt.xp, Cc, rows, Cc, Cc)
            bw.op(f"aifi{i}.attn.bwd", lib.dp_attn_bwd, qkv.xp, 3 * Cc, qkv.xp + Cc * e, qkv.xp + 2 * Cc * e, 3 * Cc,
                  _p(Pm), datt.xp, att.xp, Cc, dqkv.xp, 3 * Cc, dqkv.xp + Cc * e, dqkv.xp + 2 * Cc * e, 3 * Cc,
                  B, 1, n, 0, 1, n, nh, dh, code)
            GW = G[Wi]
            gib = G[lp + ".self_attn.in_proj_bias"]
            self.gemm(bw, f"aifi{i}.qk.dW", dqkv.xp, 1, 3 * Cc, q.xp, Cc, 1, _p(GW), Cc, 2 * Cc, Cc, rows,
                      out_code=DP_F32, beta=1.0, colsum=_p(gib))
            self.gemm(bw, f"aifi{i}.v.dW", dqkv.xp + 2 * Cc * e, 1, 3 * Cc, src.xp, Cc, 1, _p(GW, 2 * Cc * Cc), Cc, Cc,
                      Cc, rows, out_code=DP_F32, beta=1.0, colsum=_p(gib, 2 * Cc))
            # d src = d(src + attn) + (d q through q = src + pos) + d v
            bw.op(f"aifi{i}.dsrc", lib.dp_axpby_rows, src.gp, src.ld, dsum1.xp, Cc, C.c_float(1.0), None, 0,
                  C.c_float(0.0), rows, Cc, 1, code)
            self.gemm(bw, f"aifi{i}.qk.dx", dqkv.xp, 3 * Cc, 1, Wip, Cc, 1, src.gp, src.ld, rows, Cc, 2 * Cc, beta=1.0)
            self.gemm(bw, f"aifi{i}.v.dx", dqkv.xp + 2 * Cc * e, 3 * Cc, 1, Wip + 2 * Cc * Cc * e, Cc, 1, src.gp,
                      src.ld, rows, Cc, Cc, beta=1.0)
        self._bwd.append(bwd)

def _lib_tape(lib, dev):
    from .train_engine import Tape
    return Tape(lib, dev)
