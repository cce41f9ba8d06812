"""The DETRPose inference forward as a fixed plan of HIP kernel launches.

`Engine(model, dtype)` packs the reference-layout parameters once (BN folded into the
convs in f64, conv weights K-major [cout][(ky,kx,cin)] padded to the K-step, all
activations channels-last). `engine.plan(batch)` allocates every activation buffer
for that batch size once (HBM-resident arena, no allocation during the forward) and
records the ordered list of C-ABI calls; `Plan.run()` replays the list on the current
stream, and `Plan.graph()` captures it once into a hipGraph for replay.

Dataflow (reference call stack SURVEY.md §3.1; op-by-op citations inline):
  image f32 NCHW -> stem (NHWC) -> HG stages (concat buffers written in place by each
  layer, aggregation convs fuse the residual) -> input_proj convs write straight into
  the FPN concat buffers -> AIFI -> lateral convs write both the PAN concat slot and
  the x2-upsampled FPN slot -> ELAN blocks write the final levels straight into the
  flattened memory [B][S][C] -> two-stage top-k -> 3/6 decoder layers -> heads.
"""
from __future__ import annotations

import ctypes as C
import math
import os
from dataclasses import dataclass, field

import torch

from . import _lib
from ._lib import ACT, DP_BF16, DP_F32, ConvDesc, contiguous_rows, rowmap
from .fragments import frag_pack
from .hybrid_encoder import sine_pos_embed_2d
from .transformer import weighting_function

DTYPES = {"bf16": (torch.bfloat16, DP_BF16), "fp32": (torch.float32, DP_F32), "f32": (torch.float32, DP_F32)}


def pad8(c: int) -> int:
    return (c + 7) // 8 * 8


# ----------------------------------------------------------------------------- feature maps


class FMap:
    """Channels-last view into an arena tensor: element (b,y,x,c) at off + b*bs + (y*W+x)*ps + c."""

    __slots__ = ("t", "off", "B", "H", "W", "C", "ps", "bs")

    def __init__(self, t, off, B, H, W, C, ps, bs):
        self.t, self.off, self.B, self.H, self.W, self.C, self.ps, self.bs = t, off, B, H, W, C, ps, bs

    @property
    def ptr(self) -> int:
        return self.t.data_ptr() + self.off * self.t.element_size()

    def ch(self, c0: int, c: int) -> "FMap":
        return FMap(self.t, self.off + c0, self.B, self.H, self.W, c, self.ps, self.bs)

    def rows(self) -> int:
        return self.B * self.H * self.W

    def view(self) -> torch.Tensor:
        """Strided torch view (B,H,W,C) for inspection."""
        return self.t.as_strided((self.B, self.H, self.W, self.C), (self.bs, self.W * self.ps, self.ps, 1), self.off)


# ----------------------------------------------------------------------------- packed layers


@dataclass
class PConv:
    w: torch.Tensor          # [cout][kpad] (dtype) or f32 [kh][kw][C] for depthwise
    b: torch.Tensor          # f32 [cout]
    kh: int
    kw: int
    stride: int
    pad: int
    cin: int                 # channels read from the input map (padded)
    cout: int                # channels written (padded)
    act: int = 0
    lab: tuple | None = None
    depthwise: bool = False
    kpad: int = 0


@dataclass
class PSmall:
    """f32 head layer for dp_linear_small: w transposed [k][n]."""
    wt: torch.Tensor
    b: torch.Tensor
    k: int
    n: int
    act: int = 0


def _fold_frozen(sd, p, eps=1e-5):
    """FrozenBatchNorm2d (hgnetv2.py:53-61) / eval BatchNorm2d as scale & shift (f64)."""
    w, b, rm, rv = (sd[p + s].double() for s in (".weight", ".bias", ".running_mean", ".running_var"))
    scale = w * torch.rsqrt(rv + eps)
    return scale, b - rm * scale


class Packer:
    def __init__(self, sd, dtype, device):
        self.sd = sd
        self.tdtype, self.code = DTYPES[dtype]
        self.device = device
        self.bk = 64 if self.code == DP_BF16 else 32

    def conv(self, w, b, stride=1, act=None, lab=None, in_map=None, cin=None, cout=None, pad=None) -> PConv:
        """w: f64 (cout0, cin0, kh, kw) already BN-folded; b: f64 (cout0,)."""
        cout0, cin0, kh, kw = w.shape
        cin = cin or pad8(cin0)
        cout = cout or pad8(cout0)
        wp = torch.zeros(cout, kh, kw, cin, dtype=torch.float64)
        idx = torch.arange(cin0) if in_map is None else torch.as_tensor(in_map)
        wp[:cout0, :, :, idx] = w.permute(0, 2, 3, 1)
        K = kh * kw * cin
        kpad = (K + self.bk - 1) // self.bk * self.bk
        wk = torch.zeros(cout, kpad, dtype=torch.float64)
        wk[:, :K] = wp.reshape(cout, K)
        bp = torch.zeros(cout, dtype=torch.float64)
        bp[:cout0] = b
        return PConv(wk.to(self.tdtype).to(self.device).contiguous(), bp.float().to(self.device), kh, kw, stride,
                     (kh - 1) // 2 if pad is None else pad, cin, cout, ACT[act], lab, False, kpad)

    def dwconv(self, w, b, stride, act=None, lab=None) -> PConv:
        c, _, kh, kw = w.shape
        wt = w[:, 0].permute(1, 2, 0).contiguous().float().to(self.device)  # [kh][kw][C]
        return PConv(wt, b.float().to(self.device), kh, kw, stride, (kh - 1) // 2, c, c, ACT[act], lab, True)

    def linear(self, w, b, act=None, exact=False) -> PConv:
        """exact=True keeps cout unpadded (f32-output head layers: 2 / 34 / 66 columns)."""
        return self.conv(w.double()[:, :, None, None], b.double(), act=act, cout=w.shape[0] if exact else None)

    def small(self, w, b, act=None) -> PSmall:
        w = w.float()
        return PSmall(w.t().contiguous().to(self.device), b.float().to(self.device), w.shape[1], w.shape[0], ACT[act])

    # -- reference module patterns
    def conv_bn_act(self, p, act="relu", stride=None, **kw):
        """ConvBNAct (hgnetv2.py:82-134) with FrozenBN folded."""
        sd = self.sd
        w = sd[p + ".conv.weight"].double()
        s, sh = _fold_frozen(sd, p + ".bn")
        lab = None
        if act and (p + ".lab.scale") in sd:
            lab = (float(sd[p + ".lab.scale"]), float(sd[p + ".lab.bias"]))
        return w * s[:, None, None, None], sh, lab

    def conv_norm(self, p):
        """ConvNormLayer(_fuse) conv + BN (hybrid_encoder.py:56-128), folded (80-111)."""
        sd = self.sd
        w = sd[p + ".conv.weight"].double()
        s, sh = _fold_frozen(sd, p + ".norm")
        b = sh
        if (p + ".conv.bias") in sd:
            b = b + sd[p + ".conv.bias"].double() * s
        return w * s[:, None, None, None], b

    def vgg(self, p):
        """VGGBlock deploy fold (hybrid_encoder.py:156-189): 3x3 + padded 1x1."""
        w3, b3 = self.conv_norm(p + ".conv1")
        w1, b1 = self.conv_norm(p + ".conv2")
        w3 = w3.clone()
        w3[:, :, 1:2, 1:2] += w1
        return w3, b3 + b1

    def t(self, x, dtype=None):
        return x.to(self.device, dtype or torch.float32).contiguous()


# ----------------------------------------------------------------------------- plan


class Plan:
    """Recorded launches for one batch size. `run()` replays on the current stream."""

    def __init__(self, engine, batch):
        self.engine = engine
        self.batch = batch
        self.ops = []            # (name, cfunc, args)
        self.keep = []           # ctypes structs / arrays kept alive
        self.arena = []          # every device buffer the launches point into
        self.bufs = {}           # named FMaps / tensors for inspection
        self.op_out = {}         # op name -> output FMap (debug / tests)
        # per-launch roofline accounting (bench.py): every op records its algorithmic HBM bytes
        # (compulsory reads + writes) and FLOPs; dp_conv2d launches also the kernel
        # instantiation the dispatcher picks (dp_conv2d_describe)
        self.op_flops = {}       # op name -> algorithmic FLOPs
        self.op_bytes = {}       # op name -> algorithmic HBM bytes
        self.op_kernel = {}      # op name -> kernel instantiation (rocprofv3's demangled name)
        self.out_flat = None
        self.input = None
        self.outputs = {}
        self.post = None         # PostProcess buffers once add_postprocess() appended it
        self.post_ops = []       # its launch (kept apart: eager forwards do not rerun it)
        self.aux = False         # training-mode outputs recorded (Engine.plan(aux=True))
        self.aux_outputs = None  # their buffers (see Engine._plan_transformer)
        self._graph = None

    # -- recording
    def _op(self, name, fn, *args):
        self.ops.append((name, fn, args))

    def cost(self, name, nbytes, flops=0.0):
        self.op_bytes[name] = float(nbytes)
        self.op_flops[name] = float(flops)

    def kernel_of(self, name) -> str:
        """The kernel a launch runs: the dispatcher's choice for dp_conv2d, else the entry point."""
        k = self.op_kernel.get(name)
        if k:
            return k
        for n, fn, _ in self.ops + self.post_ops:
            if n == name:
                return fn.__name__
        raise KeyError(name)

    def run(self, stream=None, debug=None, post=False):
        """Replay the forward launches; with post=True also the appended PostProcess (the
        hipGraph always includes it; an eager forward leaves its buffers alone)."""
        s = C.c_void_p(stream if stream is not None else torch.cuda.current_stream(self.engine.device).cuda_stream)
        for name, fn, args in self.ops + (self.post_ops if post else []):
            rc = fn(*args, s)
            if rc:
                _lib.check(rc, name)
            if debug is not None:
                torch.cuda.synchronize()
                debug(name, self.op_out.get(name))

    def profile(self, reps=3):
        """Per-op device time (ms, median of `reps` passes) with HIP events around each launch
        (the forward and, when appended, PostProcess: the launches one graph replay runs)."""
        s = torch.cuda.current_stream(self.engine.device)
        ops = self.ops + self.post_ops
        times = {name: [] for name, _, _ in ops}
        for _ in range(reps):
            evs = []
            for name, fn, args in ops:
                e0 = torch.cuda.Event(enable_timing=True)
                e1 = torch.cuda.Event(enable_timing=True)
                e0.record(s)
                rc = fn(*args, C.c_void_p(s.cuda_stream))
                e1.record(s)
                if rc:
                    _lib.check(rc, name)
                evs.append((name, e0, e1))
            torch.cuda.synchronize()
            for name, e0, e1 in evs:
                times[name].append(e0.elapsed_time(e1))
        return {k: sorted(v)[len(v) // 2] for k, v in times.items()}

    def add_postprocess(self, num_select=60, target_size=(640.0, 640.0)):
        """Append PostProcess (deploy) to the plan: outputs scores / labels / keypoints.
        Idempotent per num_select; a different num_select replaces the previous one."""
        if self.post is not None and self.post["num_select"] == num_select:
            return self.post
        eng = self.engine
        logits, kps = self.outputs["pred_logits"], self.outputs["pred_keypoints"]
        B, Q, NC = logits.shape
        K = kps.shape[2]
        eng._cur = self
        ts = eng._empty(B, 2, dtype=torch.float32)
        ts[:, 0], ts[:, 1] = target_size
        sc = eng._empty(B, num_select, dtype=torch.float32)
        lb = eng._empty(B, num_select, dtype=torch.int64)
        ok = eng._empty(B, num_select, K, 2, dtype=torch.float32)
        self.post_ops = [("postprocess", eng.lib.dp_postprocess, (logits.data_ptr(), kps.data_ptr(), ts.data_ptr(), B,
                                                                  Q, NC, K, num_select, sc.data_ptr(), lb.data_ptr(),
                                                                  ok.data_ptr()))]
        self.cost("postprocess", 4 * B * Q * (NC + 2 * K) + B * num_select * (4 + 8 + 8 * K), 0)
        self.post = {"scores": sc, "labels": lb, "keypoints": ok, "target_sizes": ts, "num_select": num_select}
        self._graph = None
        return self.post

    def graph(self):
        """Capture the plan into a hipGraph once; returns the graph (replay with .replay())."""
        if self._graph is None:
            dev = self.engine.device
            with torch.cuda.device(dev):
                torch.cuda.synchronize(dev)
                side = torch.cuda.Stream(dev)
                side.wait_stream(torch.cuda.current_stream(dev))
                with torch.cuda.stream(side):
                    self.run(post=True)  # warm-up on the capture stream outside capture
                torch.cuda.current_stream(dev).wait_stream(side)
                torch.cuda.synchronize(dev)
                g = torch.cuda.CUDAGraph()
                with torch.cuda.graph(g):
                    self.run(post=True)
            self._graph = g
        return self._graph


class Engine:
    """Packs a DETRPose module (reference key layout) for the HIP kernels."""

    def __init__(self, model, dtype="bf16", device="cuda"):
        self.lib = _lib.load()
        self.model = model
        self.dtype_name = dtype
        self.tdtype, self.code = DTYPES[dtype]
        self.device = torch.device(device)
        sd = {k: v.detach().cpu() for k, v in model.state_dict().items()}
        self.sd = sd
        self.pk = Packer(sd, dtype, self.device)
        bb, enc, tr = model.backbone, model.encoder, model.transformer
        self.bb, self.enc, self.tr = bb, enc, tr
        self._pack_backbone()
        self._pack_encoder()
        self._pack_transformer()
        self.plans = {}

    # ------------------------------------------------------------------ packing
    def _pack_backbone(self):
        pk, bb = self.pk, self.bb
        stem = bb.arch_configs[bb.name]["stem_channels"]
        cfg = bb.arch_configs[bb.name]["stage_config"]
        self.stem_mid, self.stem_out = stem[1], stem[2]
        P = {}
        w, b, lab = pk.conv_bn_act("backbone.stem.stem1")
        P["stem1"] = (w.float().reshape(w.shape[0], 27).contiguous().to(self.device), b.float().to(self.device), lab)
        for n in ("stem2a", "stem2b", "stem3", "stem4"):
            w, b, lab = pk.conv_bn_act(f"backbone.stem.{n}")
            P[n] = pk.conv(w, b, stride=2 if n == "stem3" else 1, act="relu", lab=lab,
                           pad=0 if n in ("stem2a", "stem2b") else None)
        self.stages = []
        for si, k in enumerate(cfg):
            cin, mid, cout, nblk, down, light, ks, nl = cfg[k]
            sp = f"backbone.stages.{si}"
            st = {"cfg": cfg[k], "blocks": []}
            if down:
                w, b, _ = pk.conv_bn_act(sp + ".downsample")
                st["down"] = pk.dwconv(w, b, 2)
            for bi in range(nblk):
                bp = f"{sp}.blocks.{bi}"
                blk = {"layers": []}
                for li in range(nl):
                    lp = f"{bp}.layers.{li}"
                    if light:
                        w1, b1, _ = pk.conv_bn_act(lp + ".conv1", act=None)
                        w2, b2, lab2 = pk.conv_bn_act(lp + ".conv2")
                        blk["layers"].append((pk.conv(w1, b1), pk.dwconv(w2, b2, 1, act="relu", lab=lab2)))
                    else:
                        w1, b1, lab1 = pk.conv_bn_act(lp)
                        blk["layers"].append((pk.conv(w1, b1, act="relu", lab=lab1),))
                w, b, lab = pk.conv_bn_act(bp + ".aggregation.0")
                blk["squeeze"] = pk.conv(w, b, act="relu", lab=lab)
                w, b, lab = pk.conv_bn_act(bp + ".aggregation.1")
                blk["excite"] = pk.conv(w, b, act="relu", lab=lab)
                st["blocks"].append(blk)
            self.stages.append(st)
        self.bbP = P

    def _pack_elan(self, p):
        pk, enc = self.pk, self.enc
        Cc = enc.hidden_dim
        c4, c4p = enc.c4, pad8(enc.c4)
        act = enc.act
        E = {}
        w, b = pk.conv_norm(p + ".cv1")
        E["cv1"] = pk.conv(w, b, act=act)
        for name in ("cv2", "cv3"):
            cp = f"{p}.{name}.0"
            w1, b1 = pk.conv_norm(cp + ".conv1")
            w2, b2 = pk.conv_norm(cp + ".conv2")
            # conv1 | conv2 share their input: one GEMM with [x1 (c4p) | x2 (c4p)] outputs
            wcat = torch.zeros(2 * c4p, w1.shape[1], 1, 1, dtype=torch.float64)
            bcat = torch.zeros(2 * c4p, dtype=torch.float64)
            wcat[:c4], bcat[:c4] = w1, b1
            wcat[c4p:c4p + c4], bcat[c4p:c4p + c4] = w2, b2
            E[name + "_in"] = pk.conv(wcat, bcat, act=act, cout=2 * c4p)
            E[name + "_vgg"] = [pk.conv(*pk.vgg(f"{cp}.bottlenecks.{i}"), act=act, cin=c4p, cout=c4p)
                                for i in range(enc.n_blocks)]
            w, b = pk.conv_norm(f"{p}.{name}.1")
            E[name + "_out"] = pk.conv(w, b, act=act, cin=c4p, cout=c4p)
        w, b = pk.conv_norm(p + ".cv4")
        in_map = list(range(2 * Cc)) + [2 * Cc + i for i in range(c4)] + [2 * Cc + c4p + i for i in range(c4)]
        E["cv4"] = pk.conv(w, b, act=act, in_map=in_map, cin=2 * Cc + 2 * c4p)
        return E

    def _pack_encoder(self):
        pk, enc, sd = self.pk, self.enc, self.sd
        Cc = enc.hidden_dim
        self.encP = P = {}
        P["input_proj"] = []
        for i in range(len(enc.in_channels)):
            w = sd[f"encoder.input_proj.{i}.conv.weight"].double()
            s, sh = _fold_frozen(sd, f"encoder.input_proj.{i}.norm")
            P["input_proj"].append(pk.conv(w * s[:, None, None, None], sh))
        P["aifi"] = []
        for i, ei in enumerate(enc.use_encoder_idx):
            lp = f"encoder.encoder.{i}.layers.0"
            W = sd[lp + ".self_attn.in_proj_weight"].double()
            bW = sd[lp + ".self_attn.in_proj_bias"].double()
            stride = enc.feat_strides[ei]
            h, w_ = enc.eval_spatial_size[0] // stride, enc.eval_spatial_size[1] // stride
            pos = sine_pos_embed_2d(w_, h, Cc // 2, enc.temperatureW, enc.temperatureH)
            P["aifi"].append({
                "qk": pk.linear(W[:2 * Cc], bW[:2 * Cc]), "v": pk.linear(W[2 * Cc:], bW[2 * Cc:]),
                "out": pk.linear(sd[lp + ".self_attn.out_proj.weight"], sd[lp + ".self_attn.out_proj.bias"]),
                "l1": pk.linear(sd[lp + ".linear1.weight"], sd[lp + ".linear1.bias"], act=enc.enc_act),
                "l2": pk.linear(sd[lp + ".linear2.weight"], sd[lp + ".linear2.bias"]),
                "n1": (pk.t(sd[lp + ".norm1.weight"]), pk.t(sd[lp + ".norm1.bias"])),
                "n2": (pk.t(sd[lp + ".norm2.weight"]), pk.t(sd[lp + ".norm2.bias"])),
                "pos": pos.reshape(h * w_, Cc).to(self.device, self.tdtype).contiguous(), "hw": (h, w_)})
        P["lateral"] = []
        for j in range(enc.n_levels - 1):
            w, b = pk.conv_norm(f"encoder.lateral_convs.{j}")
            P["lateral"].append(pk.conv(w, b, act=enc.act))
        P["fpn"] = [self._pack_elan(f"encoder.fpn_blocks.{j}") for j in range(enc.n_levels - 1)]
        P["down"] = []
        for j in range(enc.n_levels - 1):
            w1, b1 = pk.conv_norm(f"encoder.downsample_convs.{j}.0.cv1")
            w2, b2 = pk.conv_norm(f"encoder.downsample_convs.{j}.0.cv2")
            P["down"].append((pk.conv(w1, b1), pk.dwconv(w2, b2, 2)))
        P["pan"] = [self._pack_elan(f"encoder.pan_blocks.{j}") for j in range(enc.n_levels - 1)]

    def _pack_transformer(self):
        pk, tr, sd = self.pk, self.tr, self.sd
        Cc = tr.hidden_dim
        t = "transformer."
        self.trP = P = {}
        P["enc_output"] = pk.linear(sd[t + "enc_output.weight"], sd[t + "enc_output.bias"])
        g, bta = sd[t + "enc_output_norm.weight"], sd[t + "enc_output_norm.bias"]
        P["enc_norm"] = (pk.t(g), pk.t(bta))
        # masked rows: output_memory = LN(enc_output(0)) = LN(bias)  (transformer.py:1232-1236)
        bias = sd[t + "enc_output.bias"].double()
        mr = (bias - bias.mean()) / torch.sqrt(bias.var(unbiased=False) + 1e-5) * g.double() + bta.double()
        P["masked_row"] = pk.t(mr.float())
        P["mask"] = pk.t(sd[t + "valid_mask"].reshape(-1), torch.uint8)
        P["anchors"] = pk.t(sd[t + "anchors"].reshape(-1, 2))
        P["enc_cls"] = (pk.t(sd[t + "enc_out_class_embed.weight"]), pk.t(sd[t + "enc_out_class_embed.bias"]))
        P["enc_cls_small"] = pk.small(sd[t + "enc_out_class_embed.weight"], sd[t + "enc_out_class_embed.bias"])
        ep = t + "enc_pose_embed.layers."
        P["enc_pose"] = [pk.linear(sd[ep + f"{i}.weight"], sd[ep + f"{i}.bias"], act="relu") for i in range(3)]
        P["enc_pose_last"] = pk.linear(sd[ep + "3.weight"], sd[ep + "3.bias"], exact=True)
        # query template: [instance | keypoint + tgt_embed[q]]  (transformer.py:1253-1261)
        nq, K = tr.num_queries, tr.num_body_points
        tmpl = torch.cat([sd[t + "instance_embedding.weight"][None].expand(nq, 1, Cc),
                          sd[t + "keypoint_embedding.weight"][None] + sd[t + "tgt_embed.weight"][:, None]], 1)
        P["tgt_tmpl"] = tmpl.to(self.device, self.tdtype).contiguous()
        P["dim_t"] = pk.t(sd[t + "decoder.dim_t"])
        hp = t + "decoder.half_pose_ref_point_head.layers."
        P["pos_head"] = [pk.linear(sd[hp + "0.weight"], sd[hp + "0.bias"], act="relu"),
                         pk.linear(sd[hp + "1.weight"], sd[hp + "1.bias"])]
        if self.code == _lib.DP_BF16:
            P["pos_head_frag"] = [frag_pack(pc.w) for pc in P["pos_head"]]
        P["project"] = pk.t(weighting_function(tr.reg_max, float(sd[t + "up"]), float(sd[t + "reg_scale"])))
        P["reg_scale"] = abs(float(sd[t + "reg_scale"]))
        pp = t + "pre_pose_embed.layers."
        P["pre_pose"] = [pk.linear(sd[pp + "0.weight"], sd[pp + "0.bias"], act="relu"),
                         pk.linear(sd[pp + "1.weight"], sd[pp + "1.bias"], act="relu"),
                         pk.linear(sd[pp + "2.weight"], sd[pp + "2.bias"], exact=True)]
        P["layers"] = []
        for l in range(tr.num_decoder_layers):
            lp = f"{t}decoder.layers.{l}."
            ca = lp + "cross_attn."
            woff = torch.cat([sd[ca + "sampling_offsets.weight"], sd[ca + "attention_weights.weight"]], 0)
            boff = torch.cat([sd[ca + "sampling_offsets.bias"], sd[ca + "attention_weights.bias"]], 0)
            pe = f"{t}pose_embed.{l}.layers."
            L = {
                "within_qkv": pk.linear(sd[lp + "within_attn.in_proj_weight"], sd[lp + "within_attn.in_proj_bias"]),
                "within_out": pk.linear(sd[lp + "within_attn.out_proj.weight"], sd[lp + "within_attn.out_proj.bias"]),
                "within_norm": (pk.t(sd[lp + "within_norm.weight"]), pk.t(sd[lp + "within_norm.bias"])),
                "across_qkv": pk.linear(sd[lp + "across_attn.in_proj_weight"], sd[lp + "across_attn.in_proj_bias"]),
                "across_out": pk.linear(sd[lp + "across_attn.out_proj.weight"], sd[lp + "across_attn.out_proj.bias"]),
                "across_norm": (pk.t(sd[lp + "across_norm.weight"]), pk.t(sd[lp + "across_norm.bias"])),
                "offattn": pk.linear(woff, boff),
                "gate": pk.linear(sd[lp + "gateway.gate.weight"], sd[lp + "gateway.gate.bias"]),
                "gate_norm": (pk.t(sd[lp + "gateway.norm.weight"]), pk.t(sd[lp + "gateway.norm.bias"])),
                "ffn1": pk.linear(sd[lp + "linear1.weight"], sd[lp + "linear1.bias"], act="relu"),
                "ffn2": pk.linear(sd[lp + "linear2.weight"], sd[lp + "linear2.bias"]),
                "norm2": (pk.t(sd[lp + "norm2.weight"]), pk.t(sd[lp + "norm2.bias"])),
                "pose": [pk.linear(sd[pe + "0.weight"], sd[pe + "0.bias"], act="relu"),
                         pk.linear(sd[pe + "1.weight"], sd[pe + "1.bias"], act="relu"),
                         pk.linear(sd[pe + "2.weight"], sd[pe + "2.bias"], exact=True)],
            }
            if self.code == _lib.DP_BF16:
                # MFMA-fragment copies for the row-block fused kernels (detrpose_amd/fragments.py)
                L["frag"] = {k: frag_pack(L[k].w) for k in ("within_out", "across_out", "gate", "ffn1", "ffn2",
                                                             "within_qkv", "across_qkv", "offattn")}
                L["frag"]["pose"] = [frag_pack(pc.w) for pc in L["pose"]]
            # class / LQE heads of every layer: the inference plan runs the last layer's
            # (eval_idx), the training-mode plan all of them (transformer.py:726-728)
            qp = f"{t}lqe_embed.{l}.reg_conf.layers."
            L["cls"] = pk.small(sd[f"{t}class_embed.{l}.weight"], sd[f"{t}class_embed.{l}.bias"])
            if qp + "0.weight" in sd:
                L["lqe"] = [pk.small(sd[qp + "0.weight"], sd[qp + "0.bias"], act="relu"),
                            pk.small(sd[qp + "1.weight"], sd[qp + "1.bias"])]
            P["layers"].append(L)

    # ------------------------------------------------------------------ planning helpers
    def _empty(self, *shape, dtype=None):
        """Every plan buffer is allocated here and owned by the plan (the launch list only
        holds raw pointers)."""
        t = torch.empty(*shape, dtype=dtype or self.tdtype, device=self.device)
        self._cur.arena.append(t)
        return t

    def _fmap(self, B, H, W, Cc, dtype=None):
        t = self._empty(B * H * W * Cc, dtype=dtype)
        return FMap(t, 0, B, H, W, Cc, Cc, H * W * Cc)

    def _conv(self, plan, name, x: FMap, pc: PConv, out: FMap, res: FMap | None = None, up: FMap | None = None,
              out_f32: bool = False, pool: FMap | None = None, seg: tuple | None = None):
        """seg = (channels per segment, elements between segments): x is a segmented input
        (dp_conv_desc.in_seg_ch / in_seg_stride), x.ps / x.bs the per-segment strides."""
        if pc.depthwise:
            assert x.C == pc.cin == out.C, (name, x.C, pc.cin, out.C)
        else:
            assert x.C == pc.cin and out.C == pc.cout, (name, x.C, pc.cin, out.C, pc.cout)
        ho = (x.H + 2 * pc.pad - pc.kh) // pc.stride + 1 if pc.pad or pc.kh == 1 else out.H
        wo = (x.W + 2 * pc.pad - pc.kw) // pc.stride + 1 if pc.pad or pc.kw == 1 else out.W
        if (out.B, out.H, out.W) != (x.B, ho, wo) and out.B == 1 and out.H == 1 and out.W == x.B * ho * wo:
            # plain row buffer written by a grouped-row input: view it with the input's grouping
            out = FMap(out.t, out.off, x.B, ho, wo, out.C, out.ps, ho * wo * out.ps)
            if res is not None and res.B == 1 and res.H == 1:
                res = FMap(res.t, res.off, x.B, ho, wo, res.C, res.ps, ho * wo * res.ps)
        assert (out.H, out.W, out.B) == (ho, wo, x.B), (name, out.H, out.W, ho, wo)
        d = ConvDesc()
        d.in_, d.in_bstride, d.in_pstride, d.in_h, d.in_w, d.cin = x.ptr, x.bs, x.ps, x.H, x.W, x.C
        d.weight, d.kpad, d.bias = pc.w.data_ptr(), pc.kpad, pc.b.data_ptr()
        d.kh, d.kw, d.stride, d.pad_t, d.pad_l = pc.kh, pc.kw, pc.stride, pc.pad, pc.pad
        d.out, d.out_bstride, d.out_pstride, d.out_h, d.out_w, d.cout = out.ptr, out.bs, out.ps, out.H, out.W, out.C
        if res is not None:
            assert res.C == out.C
            d.res, d.res_bstride, d.res_pstride = res.ptr, res.bs, res.ps
        if up is not None:
            assert up.C == out.C and up.H == 2 * out.H and up.W == 2 * out.W
            d.up, d.up_bstride, d.up_pstride = up.ptr, up.bs, up.ps
        d.batch, d.act, d.dtype = x.B, pc.act, self.code
        if out_f32:
            assert out.t.dtype == torch.float32 and (res is None or res.t.dtype == torch.float32)
            d.out_f32 = 1
        if pc.lab is not None:
            d.has_lab, d.lab_scale, d.lab_bias = 1, pc.lab[0], pc.lab[1]
        if seg is not None:
            d.in_seg_ch, d.in_seg_stride = seg
        plan.keep.append(d)
        plan.op_out[name] = out
        e = self.tdtype.itemsize
        rows = x.B * out.H * out.W
        if not pc.depthwise:
            # compulsory traffic: input read once, weights once, output (+residual, +x2 copy)
            eo = 4 if out_f32 else e
            plan.cost(name, e * x.B * x.H * x.W * x.C + e * pc.cout * pc.kh * pc.kw * pc.cin
                      + eo * rows * out.C * (1 + (res is not None) + 4 * (up is not None))
                      + (e * rows * pool.C if pool is not None else 0),
                      2.0 * rows * out.C * pc.kh * pc.kw * x.C)
            if pool is None:
                buf = C.create_string_buffer(256)
                if self.lib.dp_conv2d_describe(C.byref(d), buf, 256) == 0:
                    plan.op_kernel[name] = buf.value.decode()
        else:
            plan.cost(name, e * x.B * x.H * x.W * x.C + e * rows * out.C + 4 * pc.kh * pc.kw * out.C,
                      2.0 * rows * out.C * pc.kh * pc.kw)
        if pool is not None:
            # conv + MaxPool2d(2, 1) of the same padded input in one pass (dp_conv2d_pool)
            assert not pc.depthwise and pool.C == x.C and (pool.B, pool.H, pool.W) == (x.B, x.H, x.W)
            plan._op(name, self.lib.dp_conv2d_pool, C.byref(d), pool.ptr, pool.bs, pool.ps)
            return
        fn = self.lib.dp_dwconv2d if pc.depthwise else self.lib.dp_conv2d
        plan._op(name, fn, C.byref(d))

    def _rows(self, t: torch.Tensor, ld: int, off: int = 0) -> tuple:
        return t.data_ptr() + off * t.element_size(), contiguous_rows(ld)

    def _ln(self, plan, name, out_ptr, om, x_ptr, xm, res_ptr, rm, norm, rows, c, post=None, post_group=1,
            post_skip=0, mask=None):
        pm = post[1] if post else rowmap(group=1)
        mask_ptr, period, mrow = (mask[0].data_ptr(), mask[1], mask[2].data_ptr()) if mask else (None, 1, None)
        plan._op(name, self.lib.dp_layernorm, out_ptr, om, x_ptr, xm, res_ptr, rm if res_ptr else rowmap(group=1),
                 norm[0].data_ptr(), norm[1].data_ptr(), C.c_float(1e-5), rows, c, post[0] if post else None, pm,
                 post_group, post_skip, mask_ptr, period, mrow, self.code)

    # ------------------------------------------------------------------ planning
    def plan(self, batch: int, aux: bool = False) -> Plan:
        """aux=True: the training-mode forward's extra outputs too (every decoder layer's
        logits / keypoints / corners, the pre and interm heads: transformer.py:1348-1385)."""
        key = (batch, True) if aux else batch
        if key in self.plans:
            return self.plans[key]
        plan = Plan(self, batch)
        plan.aux = aux
        self._cur = plan
        img = self._empty(batch, 3, *self._img_hw(), dtype=torch.float32)
        plan.input = img
        feats = self._plan_backbone(plan, img)
        memory, shapes = self._plan_encoder(plan, feats)
        self._plan_transformer(plan, memory, shapes)
        self.plans[key] = plan
        return plan

    def _img_hw(self):
        return tuple(self.enc.eval_spatial_size)

    def _plan_backbone(self, plan, img):
        B = img.shape[0]
        H, W = img.shape[2], img.shape[3]
        P = self.bbP
        h1, w1 = (H + 1) // 2, (W + 1) // 2
        h2, w2 = (h1 + 1) // 2, (w1 + 1) // 2
        fused = self._stem_fusable()
        if fused:
            x_src = None   # the whole StemBlock runs as one launch into stage 0's concat slot
        else:
            x_src = self._plan_stem(plan, img, B, H, W, h1, w1)
        outs = []
        h, w = h2, w2
        for si, st in enumerate(self.stages):
            cin, midc, cout, nblk, down, light, ks, nl = st["cfg"]
            if down:
                h, w = (h + 1) // 2, (w + 1) // 2
            # a one-block stage whose input and layers have the same width keeps its HG-block
            # concat as one contiguous map per member (the 3x3 layers then read and write whole
            # 128-byte lines instead of 96-byte slices of 672-byte rows); the squeeze conv reads
            # the members as a segmented input (dp_conv_desc.in_seg_ch)
            segmented = (self.code == _lib.DP_BF16 and nblk == 1 and not light and cin == midc
                         and not os.environ.get("DETRPOSE_NO_SEG_CONCAT"))
            blocks_in, segs = [], None
            for bi in range(nblk):
                bin_ = cin if bi == 0 else cout
                if segmented:
                    selems = B * h * w * cin
                    t = self._empty((1 + nl) * selems)
                    segs = [FMap(t, i * selems, B, h, w, cin, cin, h * w * cin) for i in range(1 + nl)]
                    blocks_in.append(FMap(t, 0, B, h, w, cin * (1 + nl), cin, h * w * cin))
                else:
                    blocks_in.append(self._fmap(B, h, w, bin_ + nl * midc))
            # stage input -> block 0 concat slot [0:cin]
            slot0 = segs[0] if segs else blocks_in[0].ch(0, cin)
            if si == 0 and fused:
                self._stem_fused_op(plan, img, slot0)
            elif si == 0:
                self._conv(plan, "stem4", x_src, P["stem4"], slot0)
            else:
                self._conv(plan, f"s{si}.down", x_src, st["down"], slot0)
            for bi, blk in enumerate(st["blocks"]):
                cb = blocks_in[bi]
                bin_ = cin if bi == 0 else cout
                prev = segs[0] if segs else cb.ch(0, bin_)
                for li, layer in enumerate(blk["layers"]):
                    dst = segs[li + 1] if segs else cb.ch(bin_ + li * midc, midc)
                    if light:
                        tmp = plan.bufs.get(("light_tmp", si))
                        if tmp is None:
                            tmp = self._fmap(B, h, w, midc)
                            plan.bufs[("light_tmp", si)] = tmp
                        self._conv(plan, f"s{si}.b{bi}.l{li}.c1", prev, layer[0], tmp)
                        self._conv(plan, f"s{si}.b{bi}.l{li}.c2", tmp, layer[1], dst)
                    else:
                        self._conv(plan, f"s{si}.b{bi}.l{li}", prev, layer[0], dst)
                    prev = dst
                sq = self._fmap(B, h, w, blk["squeeze"].cout)
                self._conv(plan, f"s{si}.b{bi}.sq", cb, blk["squeeze"], sq,
                           seg=(cin, segs[1].off - segs[0].off) if segs else None)
                if bi + 1 < nblk:
                    dst = blocks_in[bi + 1].ch(0, cout)
                else:
                    dst = self._fmap(B, h, w, cout)
                res = cb.ch(0, bin_) if bi > 0 else None
                self._conv(plan, f"s{si}.b{bi}.ex", sq, blk["excite"], dst, res=res)
                x_src = dst
            if si in self.bb.return_idx:
                outs.append(x_src)
        plan.bufs["backbone"] = outs
        return outs

    def _stem_fusable(self):
        """dp_stem_fused covers the bf16 32-channel stems (B4 / B5: DETRPose-L / X)."""
        P = self.bbP
        return (self.code == _lib.DP_BF16 and self.stem_mid == 32 and self.stem_out in (48, 64)
                and not os.environ.get("DETRPOSE_NO_STEM_FUSE")
                and P["stem2a"].cout == 16 and P["stem2b"].cout == 32 and P["stem3"].cin == 64
                and P["stem3"].cout == 32 and P["stem3"].kpad >= 576 and P["stem4"].cin == 32
                and P["stem4"].cout == self.stem_out)

    def _stem_fused_op(self, plan, img, out: FMap):
        """StemBlock.forward (hgnetv2.py:204-220) as one dp_stem_fused launch."""
        P = self.bbP
        B, H, W = img.shape[0], img.shape[2], img.shape[3]
        w1, b1, lab1 = P["stem1"]
        sw = _lib.StemWeights()
        sw.w1, sw.b1 = w1.data_ptr(), b1.data_ptr()
        convs = [P[n] for n in ("stem2a", "stem2b", "stem3", "stem4")]
        (sw.w2a, sw.b2a, sw.k2a), (sw.w2b, sw.b2b, sw.k2b), (sw.w3, sw.b3, sw.k3), (sw.w4, sw.b4, sw.k4) = (
            (pc.w.data_ptr(), pc.b.data_ptr(), pc.kpad) for pc in convs)
        sw.mid, sw.cout = self.stem_mid, self.stem_out
        labs = [lab1] + [pc.lab for pc in convs]
        sw.has_lab = int(any(lb is not None for lb in labs))
        for i, lb in enumerate(labs):
            sw.lab[i][0], sw.lab[i][1] = (lb[0], lb[1]) if lb is not None else (1.0, 0.0)
        plan.keep.append(sw)
        assert (out.B, out.H, out.W, out.C) == (B, ((H + 1) // 2 + 1) // 2, ((W + 1) // 2 + 1) // 2, self.stem_out)
        plan._op("stem", self.lib.dp_stem_fused, img.data_ptr(), B, H, W, C.byref(sw), out.ptr, out.bs, out.ps)
        plan.op_out["stem"] = out
        h1, w1_ = (H + 1) // 2, (W + 1) // 2
        m1, m3 = B * h1 * w1_, B * out.H * out.W
        plan.cost("stem", 4.0 * B * 3 * H * W + 2.0 * m3 * out.C,
                  2.0 * (m1 * 32 * 27 + m1 * 16 * 128 + m1 * 32 * 64 + m3 * 32 * 576 + m3 * out.C * 32))

    def _plan_stem(self, plan, img, B, H, W, h1, w1):
        """StemBlock.forward (hgnetv2.py:204-220) as five launches; returns stem3's map."""
        mid = self.stem_mid
        P = self.bbP
        s1 = self._fmap(B, h1, w1, mid)
        wst, bst, lab = P["stem1"]
        plan._op("stem1", self.lib.dp_stem_conv, img.data_ptr(), B, H, W, wst.data_ptr(), bst.data_ptr(), mid,
                 1 if lab else 0, C.c_float(lab[0] if lab else 1.0), C.c_float(lab[1] if lab else 0.0), s1.ptr, s1.bs,
                 s1.ps, self.code)
        plan.cost("stem1", 4.0 * B * 3 * H * W + self.tdtype.itemsize * B * h1 * w1 * mid, 2.0 * B * h1 * w1 * mid * 27)
        s2a = self._fmap(B, h1, w1, P["stem2a"].cout)
        cat = self._fmap(B, h1, w1, 2 * mid)
        if self.code == _lib.DP_BF16 and mid % 8 == 0 and mid <= 64 and P["stem2a"].cout <= 32:
            # stem2a and the stem max-pool read the same F.pad(0,1,0,1) windows of stem1: one pass
            self._conv(plan, "stem2a", s1, P["stem2a"], s2a, pool=cat.ch(0, mid))
        else:
            self._conv(plan, "stem2a", s1, P["stem2a"], s2a)   # F.pad(0,1,0,1) == zero read past the edge
            plan._op("stem_pool", self.lib.dp_maxpool2x2_pad_rb, s1.ptr, s1.bs, s1.ps, B, h1, w1, mid, cat.ptr,
                     cat.bs, cat.ps, self.code)
            plan.cost("stem_pool", 2.0 * self.tdtype.itemsize * B * h1 * w1 * mid, 3.0 * B * h1 * w1 * mid)
        self._conv(plan, "stem2b", s2a, P["stem2b"], cat.ch(mid, mid))
        h2, w2 = (h1 + 1) // 2, (w1 + 1) // 2
        s3 = self._fmap(B, h2, w2, mid)
        self._conv(plan, "stem3", cat, P["stem3"], s3)
        return s3

    def _plan_elan(self, plan, name, x: FMap, E, out: FMap):
        """RepNCSPELAN4.forward (hybrid_encoder.py:210-212)."""
        enc = self.enc
        Cc, c4p = enc.hidden_dim, pad8(enc.c4)
        B, H, W = x.B, x.H, x.W
        Ecat = self._fmap(B, H, W, 2 * Cc + 2 * c4p)
        self._conv(plan, name + ".cv1", x, E["cv1"], Ecat.ch(0, 2 * Cc))
        src = Ecat.ch(Cc, Cc)
        for k, name2 in enumerate(("cv2", "cv3")):
            x12 = self._fmap(B, H, W, 2 * c4p)
            self._conv(plan, f"{name}.{name2}.in", src, E[name2 + "_in"], x12)
            cur = x12.ch(0, c4p)
            vggs = E[name2 + "_vgg"]
            for i, pc in enumerate(vggs):
                nxt = self._fmap(B, H, W, c4p)
                res = x12.ch(c4p, c4p) if i == len(vggs) - 1 else None   # CSP: x_1 + x_2
                self._conv(plan, f"{name}.{name2}.vgg{i}", cur, pc, nxt, res=res)
                cur = nxt
            dst = Ecat.ch(2 * Cc + k * c4p, c4p)
            self._conv(plan, f"{name}.{name2}.out", cur, E[name2 + "_out"], dst)
            src = dst
        self._conv(plan, name + ".cv4", Ecat, E["cv4"], out)

    def _plan_encoder(self, plan, feats):
        enc, P = self.enc, self.encP
        Cc, nlev = enc.hidden_dim, enc.n_levels
        B = feats[0].B
        hw = [(f.H, f.W) for f in feats]
        S = sum(h * w for h, w in hw)
        memory = self._empty(B * S * Cc, dtype=self.tdtype)
        starts = [sum(h * w for h, w in hw[:i]) for i in range(nlev)]
        mem_lvl = [FMap(memory, starts[i] * Cc, B, hw[i][0], hw[i][1], Cc, Cc, S * Cc) for i in range(nlev)]
        # FPN concat buffers [up(lateral) | proj_feat] per level < nlev-1, PAN concat [down | lateral]
        fcat = [self._fmap(B, hw[i][0], hw[i][1], 2 * Cc) for i in range(nlev - 1)]
        pcat = [self._fmap(B, hw[i + 1][0], hw[i + 1][1], 2 * Cc) for i in range(nlev - 1)]
        proj = []
        for i, f in enumerate(feats):
            if i < nlev - 1:
                dst = fcat[i].ch(Cc, Cc)
            else:
                dst = self._fmap(B, f.H, f.W, Cc)
            self._conv(plan, f"enc.proj{i}", f, P["input_proj"][i], dst)
            proj.append(dst)
        for i, ei in enumerate(enc.use_encoder_idx):
            proj[ei] = self._plan_aifi(plan, proj[ei], P["aifi"][i], f"enc.aifi{i}")
        # top-down: inner[0] = lateral(high) written into PAN concat [Cc:2Cc], its x2 upsample into fcat[idx-1][0:Cc]
        high = proj[-1]
        inner_feats = [None] * nlev
        for idx in range(nlev - 1, 0, -1):
            j = nlev - 1 - idx
            lat_dst = pcat[idx - 1].ch(Cc, Cc)
            self._conv(plan, f"enc.lateral{j}", high, P["lateral"][j], lat_dst, up=fcat[idx - 1].ch(0, Cc))
            dst = mem_lvl[0] if idx == 1 else self._fmap(B, hw[idx - 1][0], hw[idx - 1][1], Cc)
            self._plan_elan(plan, f"enc.fpn{j}", fcat[idx - 1], P["fpn"][j], dst)
            inner_feats[idx - 1] = dst
            high = dst
        outs = [mem_lvl[0]]
        for idx in range(nlev - 1):
            low = outs[-1]
            cv1, cv2 = P["down"][idx]
            t1 = self._fmap(B, low.H, low.W, Cc)
            self._conv(plan, f"enc.down{idx}.cv1", low, cv1, t1)
            self._conv(plan, f"enc.down{idx}.cv2", t1, cv2, pcat[idx].ch(0, Cc))
            self._plan_elan(plan, f"enc.pan{idx}", pcat[idx], P["pan"][idx], mem_lvl[idx + 1])
            outs.append(mem_lvl[idx + 1])
        plan.bufs["encoder"] = outs
        plan.bufs["memory"] = memory
        return memory, hw

    def _plan_aifi(self, plan, src: FMap, A, name):
        """TransformerEncoderLayer.forward (hybrid_encoder.py:270-296) on (B, HW, C)."""
        enc = self.enc
        Cc, nh = enc.hidden_dim, enc.nhead
        B, H, W = src.B, src.H, src.W
        n = H * W
        rows = B * n
        tok = FMap(src.t, src.off, 1, 1, rows, Cc, Cc, rows * Cc)
        qin = self._fmap(1, 1, rows, Cc)
        pos = A["pos"]
        plan._op(name + ".pos", self.lib.dp_add_rows, qin.ptr, contiguous_rows(Cc), tok.ptr, contiguous_rows(Cc),
                 pos.data_ptr(), rowmap(0, n, 0, Cc), rows, Cc, self.code)
        es = self.tdtype.itemsize
        plan.cost(name + ".pos", es * (2 * rows + n) * Cc, rows * Cc)
        qkv = self._empty(rows * 3 * Cc, dtype=self.tdtype)
        qkv_f = FMap(qkv, 0, 1, 1, rows, 3 * Cc, 3 * Cc, rows * 3 * Cc)
        self._conv(plan, name + ".qk", qin, A["qk"], qkv_f.ch(0, 2 * Cc))
        self._conv(plan, name + ".v", tok, A["v"], qkv_f.ch(2 * Cc, Cc))
        att = self._fmap(1, 1, rows, Cc)
        e = qkv.element_size()
        plan._op(name + ".attn", self.lib.dp_attention, qkv.data_ptr(), 3 * Cc, qkv.data_ptr() + Cc * e,
                 qkv.data_ptr() + 2 * Cc * e, 3 * Cc, att.ptr, Cc, B, 1, n, 0, 1, n, nh, Cc // nh, self.code)
        plan.cost(name + ".attn", es * rows * 4 * Cc, 4.0 * B * n * n * Cc)
        ao = self._fmap(1, 1, rows, Cc)
        self._conv(plan, name + ".out", att, A["out"], ao)
        s1 = self._fmap(1, 1, rows, Cc)
        self._ln(plan, name + ".n1", s1.ptr, contiguous_rows(Cc), tok.ptr, contiguous_rows(Cc), ao.ptr,
                 contiguous_rows(Cc), A["n1"], rows, Cc)
        plan.cost(name + ".n1", es * rows * Cc * 3, 8.0 * rows * Cc)
        f1 = self._fmap(1, 1, rows, A["l1"].cout)
        self._conv(plan, name + ".l1", s1, A["l1"], f1)
        f2 = self._fmap(1, 1, rows, Cc)
        self._conv(plan, name + ".l2", f1, A["l2"], f2)
        out = self._fmap(B, H, W, Cc)
        self._ln(plan, name + ".n2", out.ptr, contiguous_rows(Cc), s1.ptr, contiguous_rows(Cc), f2.ptr,
                 contiguous_rows(Cc), A["n2"], rows, Cc)
        plan.cost(name + ".n2", es * rows * Cc * 3, 8.0 * rows * Cc)
        return out

    def _plan_transformer(self, plan, memory, shapes):
        tr, P = self.tr, self.trP
        Cc, nh, nq, K = tr.hidden_dim, tr.nhead, tr.num_queries, tr.num_body_points
        T = K + 1
        B = plan.batch
        S = sum(h * w for h, w in shapes)
        dev, dt = self.device, self.tdtype
        lib = self.lib
        rows_m = B * S
        # ---- two-stage selection (transformer.py:1228-1254)
        mem_rows = FMap(memory, 0, 1, 1, rows_m, Cc, Cc, rows_m * Cc)
        om = self._fmap(1, 1, rows_m, Cc)
        score = self._empty(rows_m, dtype=torch.float32)
        wc, bc = P["enc_cls"]
        if (self.code == _lib.DP_BF16 and wc.shape[0] <= 4 and Cc == 256
                and not os.environ.get("DETRPOSE_NO_ENC_FUSE")):
            # enc_output + LN + masked rows + class max in one row-block pass (no eo round trip)
            g_, b_ = P["enc_norm"]
            eof = P.get("enc_output_frag")
            if eof is None:
                eof = P["enc_output_frag"] = frag_pack(P["enc_output"].w)
            plan._op("ts.enc_out_ln", lib.dp_linear_layernorm_classmax, om.ptr, memory.data_ptr(), rows_m, Cc,
                     eof.data_ptr(), P["enc_output"].b.data_ptr(), g_.data_ptr(), b_.data_ptr(), C.c_float(1e-5),
                     P["mask"].data_ptr(), S, P["masked_row"].data_ptr(), wc.data_ptr(), bc.data_ptr(), wc.shape[0],
                     score.data_ptr())
            ncl = wc.shape[0]
            plan.cost("ts.enc_out_ln", 2 * 2 * rows_m * Cc + 2 * Cc * Cc + 4 * rows_m,
                      2.0 * rows_m * Cc * Cc + 2.0 * rows_m * Cc * ncl + 8.0 * rows_m * Cc)
            eo = None
        else:
            eo = self._fmap(1, 1, rows_m, Cc)
            self._conv(plan, "ts.enc_output", mem_rows, P["enc_output"], eo)
        if eo is None:
            pass
        elif self.code == _lib.DP_BF16 and wc.shape[0] <= 4:
            # LN + class-score max in one pass over the rows (dp_layernorm_classmax)
            g_, b_ = P["enc_norm"]
            plan._op("ts.enc_norm", lib.dp_layernorm_classmax, om.ptr, eo.ptr, g_.data_ptr(), b_.data_ptr(),
                     C.c_float(1e-5), rows_m, Cc, P["mask"].data_ptr(), S, P["masked_row"].data_ptr(), wc.data_ptr(),
                     bc.data_ptr(), wc.shape[0], score.data_ptr(), self.code)
            plan.cost("ts.enc_norm", self.tdtype.itemsize * 2 * rows_m * Cc + 4 * rows_m,
                      2.0 * rows_m * Cc * wc.shape[0] + 8.0 * rows_m * Cc)
        else:
            self._ln(plan, "ts.enc_norm", om.ptr, contiguous_rows(Cc), eo.ptr, contiguous_rows(Cc), None, None,
                     P["enc_norm"], rows_m, Cc, mask=(P["mask"], S, P["masked_row"]))
            plan._op("ts.class_max", lib.dp_class_max, om.ptr, rows_m, Cc, wc.data_ptr(), bc.data_ptr(), wc.shape[0],
                     score.data_ptr(), self.code)
            plan.cost("ts.enc_norm", self.tdtype.itemsize * 2 * rows_m * Cc, 8.0 * rows_m * Cc)
            plan.cost("ts.class_max", self.tdtype.itemsize * rows_m * Cc + 4 * rows_m, 2.0 * rows_m * Cc * wc.shape[0])
        topv = self._empty(B, nq, dtype=torch.float32)
        topi = self._empty(B, nq, dtype=torch.int64)
        plan._op("ts.topk", lib.dp_topk, score.data_ptr(), B, S, S, nq, topv.data_ptr(), topi.data_ptr())
        plan.cost("ts.topk", 4 * B * S + 12 * B * nq, 0)
        tm = self._fmap(1, 1, B * nq, Cc)
        plan._op("ts.gather", lib.dp_gather_rows, om.ptr, S * Cc, topi.data_ptr(), B, nq, Cc, tm.ptr, self.code)
        plan.cost("ts.gather", 2 * dt.itemsize * B * nq * Cc + 8 * B * nq, 0)
        x = tm
        for i, pc in enumerate(P["enc_pose"]):
            y = self._fmap(1, 1, B * nq, pc.cout)
            self._conv(plan, f"ts.enc_pose{i}", x, pc, y)
            x = y
        last = P["enc_pose_last"]
        delta = self._empty(B * nq, last.cout, dtype=torch.float32)
        self._conv(plan, "ts.enc_pose3", x, last, FMap(delta, 0, 1, 1, B * nq, last.cout, last.cout, delta.numel()),
                   out_f32=True)
        ref = self._empty(B, nq, T, 2, dtype=torch.float32)
        plan._op("ts.refpoints", lib.dp_refpoint_init, delta.data_ptr(), P["anchors"].data_ptr(), topi.data_ptr(), B,
                 nq, K, ref.data_ptr())
        plan.cost("ts.refpoints", 4 * B * nq * (2 * K + 2 + 2 * T) + 8 * B * nq, 8.0 * B * nq * K)
        plan.bufs.update(topk_idx=topi, topk_val=topv, enc_output_norm=om, score=score)
        aux = plan.aux
        if aux:
            # aux_interm_outputs (transformer.py:1248-1250, 1372): every class score of the selected
            # rows, and the initial keypoint coordinates (the decoder refines ref in place)
            ecs = P["enc_cls_small"]
            interm_logits = self._empty(B, nq, ecs.n, dtype=torch.float32)
            plan._op("aux.interm_cls", lib.dp_linear_small, tm.ptr, contiguous_rows(Cc), self.code, B * nq, ecs.k,
                     ecs.wt.data_ptr(), ecs.b.data_ptr(), ecs.n, ecs.n, 0, None, interm_logits.data_ptr())
            plan.cost("aux.interm_cls", dt.itemsize * B * nq * Cc + 4 * B * nq * ecs.n, 2.0 * B * nq * Cc * ecs.n)
            interm_ref = self._empty(B, nq, T, 2, dtype=torch.float32)
            plan._op("aux.interm_ref", lib.dp_broadcast, ref.data_ptr(), ref.numel() * 4, interm_ref.data_ptr(), 1)
            plan.cost("aux.interm_ref", 8 * ref.numel(), 0)
        # ---- decoder (transformer.py:558-925)
        rows = B * nq * T               # all tokens
        krows = B * nq * K              # keypoint tokens
        tgtA = self._empty(rows * Cc, dtype=dt)
        tgtB = self._empty(rows * Cc, dtype=dt)
        tmpl = P["tgt_tmpl"]
        plan._op("dec.tgt", lib.dp_broadcast, tmpl.data_ptr(), tmpl.numel() * tmpl.element_size(), tgtA.data_ptr(), B)
        plan.cost("dec.tgt", tmpl.numel() * tmpl.element_size() * (1 + B), 0)
        kp_map = rowmap(Cc, K, T * Cc, Cc)       # keypoint token rows of a [rows][C] tensor
        # bf16: the row-block fused decoder kernels (csrc/decoder.hip); fp32 parity mode keeps
        # one launch per reference op
        fused = self.code == _lib.DP_BF16 and Cc in (128, 256, 384)
        plan.decoder_fused = fused
        # the two token attentions as one launch each (dp_mha_layernorm: C = 256, 8 heads)
        mha = (fused and Cc == 256 and nh == 8 and T == 18 and nq == 60
               and not os.environ.get("DETRPOSE_NO_MHA_FUSE"))
        pos = self._fmap(1, 1, krows, Cc)
        qkv = self._empty(rows * 3 * Cc, dtype=dt)
        att = self._fmap(1, 1, rows, Cc)
        gx = self._empty(rows * 2 * Cc, dtype=dt)   # [x1 | msda]
        nl_, npnt = tr.num_feature_levels, tr.dec_n_points
        assert (nh * nl_ * npnt * 3) % 8 == 0, "offsets|logits row must be 16-byte aligned"
        oa = self._fmap(1, 1, rows, nh * nl_ * npnt * 3)
        ph1 = self._fmap(1, 1, krows, Cc)
        ph2 = self._fmap(1, 1, krows, Cc)
        if not fused:
            se = self._fmap(1, 1, krows, Cc)
            h1 = self._fmap(1, 1, krows, Cc)
            ao = self._fmap(1, 1, rows, Cc)
            gt = self._fmap(1, 1, rows, 2 * Cc)
            f1 = self._fmap(1, 1, rows, tr.dim_feedforward)
            f2 = self._fmap(1, 1, rows, Cc)
            pin = self._fmap(1, 1, krows, Cc)
        nb = 2 * (tr.reg_max + 1)
        nlayers = tr.num_decoder_layers
        ncorn = nlayers if aux else 2
        corners = [self._empty(krows, nb, dtype=torch.float32) for _ in range(ncorn)]
        plan.bufs["corners"] = corners        # layer l writes corners[l % ncorn] (pred_corners, f32)
        pre = self._empty(krows, 2, dtype=torch.float32)
        ref_init = self._empty(krows, 2, dtype=torch.float32)
        # outputs share one contiguous f32 buffer [logits (B,nq,ncls) | keypoints (B,nq,K,2)]
        # so a data-parallel run gathers them with a single collective
        ncls = tr.num_classes
        out_flat = self._empty(B * nq * (ncls + 2 * K), dtype=torch.float32)
        plan.out_flat = out_flat
        kps = out_flat[B * nq * ncls:].view(B, nq, K, 2)
        lvl_hw = (C.c_int32 * (2 * len(shapes)))(*[v for hw in shapes for v in hw])
        plan.keep.append(lvl_hw)
        e = qkv.element_size()
        qkv_f = FMap(qkv, 0, 1, 1, rows, 3 * Cc, 3 * Cc, rows * 3 * Cc)
        gx_f = FMap(gx, 0, 1, 1, rows, 2 * Cc, 2 * Cc, rows * 2 * Cc)
        plan.bufs["layers"] = []
        plan.bufs["layer_ops"] = []           # per layer: (op that finishes its token rows, op writing its corners)
        src, dst = tgtA, tgtB
        cr = contiguous_rows
        # training mode: each layer's keypoints / logits in buffers of their own (the last
        # layer's are the outputs in out_flat)
        layer_kps = [self._empty(B, nq, K, 2, dtype=torch.float32) if aux and l < nlayers - 1 else kps
                     for l in range(nlayers)]
        layer_logits = [self._empty(B, nq, ncls, dtype=torch.float32) if aux and l < nlayers - 1 else
                        out_flat[:B * nq * ncls].view(B, nq, ncls) for l in range(nlayers)]
        pre_logits = self._empty(B, nq, ncls, dtype=torch.float32) if aux else None

        def class_lqe(n, L, x_rows, kps_l, logits_l):
            """class_embed[l] on the instance tokens + LQE (transformer.py:726-728)"""
            cls, lqe = L["cls"], L["lqe"]
            score2 = self._empty(B * nq, cls.n, dtype=torch.float32)
            plan._op(n + ".cls", lib.dp_linear_small, x_rows, rowmap(0, 1, T * Cc, 0), self.code, B * nq,
                     cls.k, cls.wt.data_ptr(), cls.b.data_ptr(), cls.n, cls.n, 0, None, score2.data_ptr())
            plan.cost(n + ".cls", e * B * nq * Cc + 4 * B * nq * cls.n, 2.0 * B * nq * Cc * cls.n)
            lv0 = plan.bufs["encoder"][0]
            st = self._empty(B * nq, K * 5, dtype=torch.float32)
            plan._op(n + ".lqe_stats", lib.dp_lqe_stats, lv0.ptr, lv0.bs, lv0.H, lv0.W, Cc, kps_l.data_ptr(), B, nq,
                     K, st.data_ptr(), self.code)
            # 4 bilinear corners of C channels per keypoint (gathered), kps in, stats out
            plan.cost(n + ".lqe_stats", 4 * e * B * nq * K * Cc + 4 * B * nq * K * 7, 8.0 * B * nq * K * Cc)
            hid = self._empty(B * nq, lqe[0].n, dtype=torch.float32)
            plan._op(n + ".lqe0", lib.dp_linear_small, st.data_ptr(), contiguous_rows(K * 5), DP_F32, B * nq,
                     lqe[0].k, lqe[0].wt.data_ptr(), lqe[0].b.data_ptr(), lqe[0].n, lqe[0].n, lqe[0].act, None,
                     hid.data_ptr())
            plan.cost(n + ".lqe0", 4 * B * nq * (K * 5 + lqe[0].n) + 4 * lqe[0].k * lqe[0].n,
                      2.0 * B * nq * lqe[0].k * lqe[0].n)
            plan._op(n + ".lqe1", lib.dp_linear_small, hid.data_ptr(), contiguous_rows(lqe[0].n), DP_F32, B * nq,
                     lqe[1].k, lqe[1].wt.data_ptr(), lqe[1].b.data_ptr(), lqe[1].n, cls.n, 0,
                     score2.data_ptr(), logits_l.data_ptr())
            plan.cost(n + ".lqe1", 4 * B * nq * (lqe[0].n + 2 * cls.n), 2.0 * B * nq * lqe[1].k * cls.n)
        eps = C.c_float(1e-5)

        def lin(pc, frag, k):
            """(fragment-layout weight, f32 bias) of a fused-kernel GEMM with k inputs"""
            assert pc.kpad == k and frag.shape[1] * 32 == k, (pc.kpad, k, tuple(frag.shape))
            return frag.data_ptr(), pc.b.data_ptr()

        for l, L in enumerate(P["layers"]):
            n = f"dec{l}"
            src_f = FMap(src, 0, 1, 1, rows, Cc, Cc, rows * Cc)
            dst_f = FMap(dst, 0, 1, 1, rows, Cc, Cc, rows * Cc)
            if fused:
                # sine embedding -> pos MLP -> pos, and the in-place with_pos_embed of the layer
                # input (transformer.py:369, 588-592): also turns the previous layer's output_pose
                # into output_pose_detach + pos (aliasing kept on purpose)
                ph = P["pos_head"]
                phf = P["pos_head_frag"]
                plan._op(n + ".pos", lib.dp_query_pos, ref.data_ptr(), krows, K, P["dim_t"].data_ptr(),
                         *lin(ph[0], phf[0], Cc), *lin(ph[1], phf[1], Cc), pos.ptr, src.data_ptr(), kp_map, Cc)
                # refs in; pos out; keypoint rows of the layer input read + written; two C x C weights
                plan.cost(n + ".pos", 8 * B * nq * T + 3 * e * krows * Cc + 2 * e * Cc * Cc,
                          4.0 * krows * Cc * Cc + 4.0 * krows * Cc)
            else:
                # query pos from the current reference points (transformer.py:588-592)
                plan._op(n + ".sine", lib.dp_sine_embed, ref.data_ptr(), B * nq, K, Cc, P["dim_t"].data_ptr(),
                         se.ptr, self.code)
                plan.cost(n + ".sine", 8 * B * nq * T + e * krows * Cc, 4.0 * krows * Cc)
                self._conv(plan, n + ".pos0", se, P["pos_head"][0], h1)
                self._conv(plan, n + ".pos1", h1, P["pos_head"][1], pos)
                # in-place with_pos_embed on the layer input (transformer.py:369): also turns the previous
                # layer's output_pose into output_pose_detach + pos (aliasing kept on purpose)
                plan._op(n + ".addpos", lib.dp_add_rows, src.data_ptr(), kp_map, src.data_ptr(), kp_map, pos.ptr,
                         contiguous_rows(Cc), krows, Cc, self.code)
                plan.cost(n + ".addpos", 3 * e * krows * Cc, krows * Cc)
            if mha:
                # within-instance MHA + out_proj + residual + LN (transformer.py:403-406), then the
                # across-instance one over the nq queries of a token slot (transformer.py:409-422)
                fr, wn, an = L["frag"], L["within_norm"], L["across_norm"]
                plan._op(n + ".w_mha", lib.dp_mha_layernorm, dst.data_ptr(), cr(Cc), src.data_ptr(), cr(Cc), B * nq, 1,
                         T, 0, 1, T, *lin(L["within_qkv"], fr["within_qkv"], Cc),
                         *lin(L["within_out"], fr["within_out"], Cc), wn[0].data_ptr(), wn[1].data_ptr(), eps, Cc, nh,
                         None, rowmap(group=1), 1, 0, None, 0, None, None, 0)
                # + the MSDA offsets/logits Linear on the rows it stores (ms_deform_attn.py:428-432)
                plan._op(n + ".a_mha", lib.dp_mha_layernorm, gx.data_ptr(), cr(2 * Cc), dst.data_ptr(), cr(Cc), B, T,
                         nq * T, 1, T, nq, *lin(L["across_qkv"], fr["across_qkv"], Cc),
                         *lin(L["across_out"], fr["across_out"], Cc), an[0].data_ptr(), an[1].data_ptr(), eps, Cc, nh,
                         pos.ptr, cr(Cc), T, 1, oa.ptr, oa.ps, *lin(L["offattn"], fr["offattn"], Cc), oa.C)
                # projections (q, k, v, out) + QK^T and PV over each token's sequence, + the fused
                # offsets/logits Linear in the across launch; rows in / out, pos rows, weights
                proj = 2.0 * rows * Cc * 4 * Cc
                plan.cost(n + ".w_mha", 2 * e * rows * Cc + 2 * 4 * Cc * Cc, proj + 4.0 * rows * T * Cc)
                plan.cost(n + ".a_mha", 2 * e * rows * Cc + e * krows * Cc + e * rows * oa.C + 2 * Cc * (4 * Cc + oa.C),
                          proj + 4.0 * rows * nq * Cc + 2.0 * rows * Cc * oa.C)
            else:
                # within-instance MHA over the T tokens of a query (transformer.py:403-406)
                self._conv(plan, n + ".w_qkv", src_f, L["within_qkv"], qkv_f)
                plan._op(n + ".w_attn", lib.dp_attention, qkv.data_ptr(), 3 * Cc, qkv.data_ptr() + Cc * e,
                         qkv.data_ptr() + 2 * Cc * e, 3 * Cc, att.ptr, Cc, B * nq, 1, T, 0, 1, T, nh, Cc // nh, self.code)
                plan.cost(n + ".w_attn", 4 * e * rows * Cc, 4.0 * rows * T * Cc)
                if fused:
                    wn, fr = L["within_norm"], L["frag"]
                    plan._op(n + ".w_out_ln", lib.dp_linear_layernorm, dst.data_ptr(), cr(Cc), att.ptr, cr(Cc), Cc,
                             *lin(L["within_out"], fr["within_out"], Cc), src.data_ptr(), cr(Cc), wn[0].data_ptr(),
                             wn[1].data_ptr(), eps, rows, Cc, None, rowmap(group=1), 1, 0)
                    plan.cost(n + ".w_out_ln", 3 * e * rows * Cc + e * Cc * Cc, 2.0 * rows * Cc * Cc + 8.0 * rows * Cc)
                else:
                    self._conv(plan, n + ".w_out", att, L["within_out"], ao)
                    self._ln(plan, n + ".w_norm", dst.data_ptr(), contiguous_rows(Cc), src.data_ptr(), contiguous_rows(Cc),
                             ao.ptr, contiguous_rows(Cc), L["within_norm"], rows, Cc)
                    plan.cost(n + ".w_norm", 3 * e * rows * Cc, 8.0 * rows * Cc)
                # across-instance MHA over the nq queries of a token slot (transformer.py:409-419)
                self._conv(plan, n + ".a_qkv", dst_f, L["across_qkv"], qkv_f)
                plan._op(n + ".a_attn", lib.dp_attention, qkv.data_ptr(), 3 * Cc, qkv.data_ptr() + Cc * e,
                         qkv.data_ptr() + 2 * Cc * e, 3 * Cc, att.ptr, Cc, B, T, nq * T, 1, T, nq, nh, Cc // nh,
                         self.code)
                plan.cost(n + ".a_attn", 4 * e * rows * Cc, 4.0 * rows * nq * Cc)
                # out_proj + LN + second in-place pos add -> x1 = gx[:, :C]   (transformer.py:419-422)
                if fused:
                    an, fr = L["across_norm"], L["frag"]
                    plan._op(n + ".a_out_ln", lib.dp_linear_layernorm, gx.data_ptr(), cr(2 * Cc), att.ptr, cr(Cc), Cc,
                             *lin(L["across_out"], fr["across_out"], Cc), dst.data_ptr(), cr(Cc), an[0].data_ptr(),
                             an[1].data_ptr(), eps, rows, Cc, pos.ptr, cr(Cc), T, 1)
                    plan.cost(n + ".a_out_ln", 3 * e * rows * Cc + e * krows * Cc + e * Cc * Cc,
                              2.0 * rows * Cc * Cc + 8.0 * rows * Cc)
                else:
                    self._conv(plan, n + ".a_out", att, L["across_out"], ao)
                    self._ln(plan, n + ".a_norm", gx.data_ptr(), contiguous_rows(2 * Cc), dst.data_ptr(),
                             contiguous_rows(Cc), ao.ptr, contiguous_rows(Cc), L["across_norm"], rows, Cc,
                             post=(pos.ptr, contiguous_rows(Cc)), post_group=T, post_skip=1)
                    plan.cost(n + ".a_norm", 3 * e * rows * Cc + e * krows * Cc, 8.0 * rows * Cc)
            # MSDA (ms_deform_attn.py:384-444) -> gx[:, C:]
            if not mha:
                self._conv(plan, n + ".offattn", gx_f.ch(0, Cc), L["offattn"], oa)
            plan._op(n + ".msda", lib.dp_msda, memory.data_ptr(), B, S, lvl_hw, len(shapes), oa.ptr, ref.data_ptr(),
                     gx.data_ptr() + Cc * e, 2 * Cc, nq * T, nh, Cc // nh, npnt, self.code)
            # SURVEY.md §8d algorithmic bytes: value once + offsets/logits + ref + output;
            # FLOPs: 4 corners x (bilinear weight FMA) per channel per sampling point + softmax
            plan.cost(n + ".msda", e * (B * S * Cc + rows * oa.C + rows * Cc) + 4 * rows * 2,
                      10.0 * rows * nh * nl_ * npnt * (Cc // nh))
            # Gate (transformer.py:222-235), FFN (transformer.py:380-385)
            if fused:
                gn, n2, fr = L["gate_norm"], L["norm2"], L["frag"]
                plan._op(n + ".gate_ln", lib.dp_gate_linear_layernorm, dst.data_ptr(), cr(Cc), gx.data_ptr(),
                         cr(2 * Cc), *lin(L["gate"], fr["gate"], 2 * Cc), gn[0].data_ptr(), gn[1].data_ptr(), eps,
                         rows, Cc)
                plan.cost(n + ".gate_ln", 3 * e * rows * Cc + e * 4 * Cc * Cc, 2.0 * rows * 4 * Cc * Cc + 12.0 * rows * Cc)
                fd = tr.dim_feedforward
                plan._op(n + ".ffn_ln", lib.dp_ffn_layernorm, dst.data_ptr(), cr(Cc), dst.data_ptr(), cr(Cc),
                         *lin(L["ffn1"], fr["ffn1"], Cc), fd, *lin(L["ffn2"], fr["ffn2"], fd), n2[0].data_ptr(),
                         n2[1].data_ptr(), eps, rows, Cc)
                plan.cost(n + ".ffn_ln", 2 * e * rows * Cc + e * 2 * Cc * fd, 4.0 * rows * Cc * fd + 8.0 * rows * Cc)
                last_op = n + ".ffn_ln"
            else:
                self._conv(plan, n + ".gate", gx_f, L["gate"], gt)
                plan._op(n + ".gate_ln", lib.dp_gate_layernorm, dst.data_ptr(), Cc, gt.ptr, gx.data_ptr(),
                         L["gate_norm"][0].data_ptr(), L["gate_norm"][1].data_ptr(), C.c_float(1e-5), rows, Cc,
                         self.code)
                plan.cost(n + ".gate_ln", 5 * e * rows * Cc, 12.0 * rows * Cc)
                self._conv(plan, n + ".ffn1", dst_f, L["ffn1"], f1)
                self._conv(plan, n + ".ffn2", f1, L["ffn2"], f2)
                self._ln(plan, n + ".norm2", dst.data_ptr(), contiguous_rows(Cc), dst.data_ptr(), contiguous_rows(Cc),
                         f2.ptr, contiguous_rows(Cc), L["norm2"], rows, Cc)
                plan.cost(n + ".norm2", 3 * e * rows * Cc, 8.0 * rows * Cc)
                last_op = n + ".norm2"
            plan.bufs["layers"].append(dst)
            # ---- heads (transformer.py:701-728)
            pose_f = FMap(dst, Cc, B * nq, 1, K, Cc, Cc, T * Cc)       # output[:, :, 1:]
            if l == 0:
                pp = P["pre_pose"]
                self._conv(plan, n + ".pre0", pose_f, pp[0], ph1)
                self._conv(plan, n + ".pre1", ph1, pp[1], ph2)
                self._conv(plan, n + ".pre2", ph2, pp[2], FMap(pre, 0, 1, 1, krows, 2, 2, pre.numel()), out_f32=True)
                plan._op(n + ".pre_pose", lib.dp_pre_pose, pre.data_ptr(), ref.data_ptr(), B * nq, K,
                         ref_init.data_ptr())
                plan.cost(n + ".pre_pose", 4 * krows * 2 * 2 + 8 * B * nq * T, 10.0 * krows * 2)
                if aux:
                    # pre_scores = class_head[0](output_instance) (transformer.py:708)
                    c0 = P["layers"][0]["cls"]
                    plan._op(n + ".pre_cls", lib.dp_linear_small, dst.data_ptr(), rowmap(0, 1, T * Cc, 0), self.code,
                             B * nq, c0.k, c0.wt.data_ptr(), c0.b.data_ptr(), c0.n, c0.n, 0, None,
                             pre_logits.data_ptr())
                    plan.cost(n + ".pre_cls", e * B * nq * Cc + 4 * B * nq * c0.n, 2.0 * B * nq * Cc * c0.n)
            ph = L["pose"]
            cur, prev = corners[l % ncorn], corners[(l - 1) % ncorn]
            if fused:
                # pred_corners = pose_head(output_pose [+ output_pose_detach]) [+ pred_corners_undetach]
                # (transformer.py:712): src keypoint rows hold the previous output_pose + this layer's
                # pos (in-place aliasing, transformer.py:369/716/922)
                pw = [v for i in range(3) for v in lin(ph[i], L["frag"]["pose"][i], Cc)]
                plan._op(n + ".pose", lib.dp_pose_mlp, dst.data_ptr(), kp_map, src.data_ptr() if l > 0 else None,
                         kp_map, krows, *pw, nb, prev.data_ptr() if l > 0 else None, cur.data_ptr(), Cc)
                plan.cost(n + ".pose", e * krows * Cc * (1 + (l > 0)) + 4 * krows * nb * (1 + (l > 0))
                          + e * Cc * (2 * Cc + nb), 2.0 * krows * Cc * (2 * Cc + nb))
                plan.bufs["layer_ops"].append((last_op, n + ".pose"))
            else:
                if l == 0:
                    x_in = pose_f
                else:
                    # pose_head(output_pose + output_pose_detach): src keypoint rows hold the previous
                    # output_pose + this layer's pos (in-place aliasing, transformer.py:369/716/922)
                    plan._op(n + ".pin", lib.dp_add_rows, pin.ptr, contiguous_rows(Cc), dst.data_ptr(), kp_map,
                             src.data_ptr(), kp_map, krows, Cc, self.code)
                    plan.cost(n + ".pin", 3 * e * krows * Cc, krows * Cc)
                    x_in = pin
                self._conv(plan, n + ".pose0", x_in, ph[0], ph1)
                self._conv(plan, n + ".pose1", ph1, ph[1], ph2)
                # pred_corners = pose_head(...) + pred_corners_undetach (transformer.py:712), f32 out + f32 residual
                self._conv(plan, n + ".pose2", ph2, ph[2], FMap(cur, 0, 1, 1, krows, nb, nb, cur.numel()),
                           res=FMap(prev, 0, 1, 1, krows, nb, nb, prev.numel()) if l > 0 else None, out_f32=True)
                plan.bufs["layer_ops"].append((last_op, n + ".pose2"))
            plan._op(n + ".refine", lib.dp_pose_refine, cur.data_ptr(), P["project"].data_ptr(), tr.reg_max,
                     ref_init.data_ptr(), C.c_float(P["reg_scale"]), B * nq, K, layer_kps[l].data_ptr(), ref.data_ptr())
            plan.cost(n + ".refine", 4 * krows * (nb + 2 + 2) + 8 * B * nq * T, 5.0 * krows * nb)
            if l == nlayers - 1 or aux:
                class_lqe(n, L, dst.data_ptr(), layer_kps[l], layer_logits[l])
            if l == nlayers - 1:
                plan.outputs = {"pred_logits": layer_logits[l], "pred_keypoints": kps}
            src, dst = dst, src
        plan.bufs["ref"] = ref
        if aux:
            plan.aux_outputs = {"logits": layer_logits, "keypoints": layer_kps,
                                "corners": [corners[l % ncorn].view(B, nq, K, nb) for l in range(nlayers)],
                                "ref_init": ref_init.view(B, nq, K, 2), "pre_logits": pre_logits,
                                "interm_logits": interm_logits, "interm_ref": interm_ref}
