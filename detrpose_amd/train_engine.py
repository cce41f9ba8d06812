"""The transformer's training step on the HIP kernels: training-mode forward with OKS-denoising
queries, the criterion (matching + losses + their gradients), and the backward through every
transformer parameter — a fixed tape of C-ABI launches, like the inference Plan.

Reference: Transformer.forward in training mode
(src/models/detrpose/transformer.py:1219-1385), TransformerDecoder.forward training branch
(558-603, 701-728, 903-916), DeformableTransformerDecoderLayer.forward (387-442), prepare_for_cdn
(dn_component.py:39-183), Criterion.forward incl. the dn_* losses (criterion.py:285-435), then
loss.backward() (src/solver/engine.py:55-60). The reference runs this through torch autograd;
here every forward op that the backward needs saves its inputs / statistics into buffers of the
step's arena, and the backward is written out op by op in reverse:

  nn.Linear            dp_gemm forward / dgrad (dy W) / wgrad (dy^T x, split-K f32 atomics)
                       + dp_colsum bias grads; ReLU backward is the dgrad GEMM's gate
  nn.LayerNorm         dp_ln_fwd (saves the pre-norm sum and mean / rstd) / dp_ln_bwd
  MultiheadAttention   in_proj / out_proj GEMMs + dp_attn_fwd (saves P) / dp_attn_bwd, with the
                       DN attn_mask in the across attention
  MSDeformAttn         dp_msda (f32 offsets) / dp_msda_bwd_sorted (offsets / logits / value gradients)
  Gate                 dp_gate_fwd / dp_gate_bwd + its Linear
  heads                pose / pre / class / LQE MLPs as GEMMs, dp_pose_refine(_bwd),
                       dp_pre_pose + dp_sigmoid_bwd, dp_lqe_stats(_bwd)
  query construction   dp_query_build(_bwd) (tgt_embed, keypoint / instance embeddings, DN
                       label_enc / pose_enc rows)
  two-stage            enc_output + LN + class + top-k forward over all rows; the backward
                       recomputes enc_output + LN on the selected rows only (the only rows
                       with a gradient)

Scope of this tape: the transformer. Its encoder-memory input is differentiated (d memory,
accumulated by the MSDA value gradient and the two-stage rows) and handed to the encoder tape
(encoder_train.EncoderTrainPlan), whose backward feeds the backbone tape
(backbone_train.BackboneTrainPlan): train.Trainer chains the three. BatchNorm is not on this
tape. Parameter gradients accumulate into one f32 buffer (`TrainEngine.grads`, reference names).
"""
from __future__ import annotations

import ctypes as C
import os
import math

import numpy as np
import torch

from . import _lib
from ._lib import DP_BF16, DP_F32, ConvDesc, GemmDesc, contiguous_rows, rowmap
from .criterion import COCO_SIGMAS, CROWDPOSE_SIGMAS, pack_targets
from .transformer import weighting_function

DT = {"bf16": (torch.bfloat16, DP_BF16), "fp32": (torch.float32, DP_F32)}
T_ = "transformer."


def dn_match(sizes, pad_size, num_group):
    """criterion.py:385-399: DN slot g*single_pad + t <-> target t of its image (positives)."""
    single = pad_size // num_group
    m = np.full((len(sizes), pad_size), -1, np.int32)
    for b, n in enumerate(sizes):
        for g in range(num_group):
            m[b, g * single: g * single + n] = np.arange(n)
    return m


class Tape:
    """Recorded launches with their descriptors kept alive.

    use_graph: after one eager run, the launches are captured once into hipGraphs
    (torch.cuda.CUDAGraph) and later runs replay them (one launch instead of one ctypes call per
    op). Every op's arguments are fixed buffers and descriptors, so a replay is the eager run. A
    tape holding host ops (the SyncBN collectives of world > 1) is cut at them into segments:
    each run of device ops between two host ops is its own graph, and the host ops run between
    the replays in stream order (graph -> collective -> graph), so world > 1 keeps the replay."""

    def __init__(self, lib, device):
        self.lib = lib
        self.device = device
        self.ops = []
        self.keep = []
        self.use_graph = False
        self.runs = 0
        self._graph = None   # [("graph", CUDAGraph) | ("host", fn)] once captured
        # a forward tape: its GEMMs never split K (float atomics would make the forward differ
        # run to run; the reference's forward is deterministic, tests/test_gpu_train_graphs.py)
        self.deterministic = False

    def op(self, name, fn, *args):
        self.ops.append((name, fn, args))
        self._graph = None

    @property
    def n_host(self):
        """Host ops on the tape (each one a cut between two graph segments)."""
        return sum(1 for _, fn, _ in self.ops if getattr(fn, "host", False))

    @property
    def n_graphs(self):
        """Graph segments of the captured tape (0 before capture)."""
        return sum(1 for k, _ in self._graph if k == "graph") if self._graph else 0

    def _launch(self, stream, debug, ops=None):
        s = C.c_void_p(stream if stream is not None else torch.cuda.current_stream(self.device).cuda_stream)
        for name, fn, args in (self.ops if ops is None else ops):
            rc = fn(*args, s)
            if rc:
                _lib.check(rc, name)
            if debug is not None:
                torch.cuda.synchronize()
                debug(name)

    def batch_packs(self):
        """Replace the tape's weight packs (dp_conv_pack calls, and the dp_convert_rows f32 ->
        dtype copies of whole weights) by ONE dp_conv_pack_batch launch over a device table of
        their descriptors. Every pack writes its own output from the f32 master, so their order is
        free; the tape's other ops keep theirs, after the batch."""
        lib = self.lib
        rows, rest = [], []
        for name, fn, args in self.ops:
            if fn is lib.dp_conv_pack:
                w, cout, cin, kh, kw, out, kpad, kc, mode, scale, dt = args
                rows.append((w, out, scale, cout, cin, kh, kw, kpad, kc, mode, dt))
            elif (fn is lib.dp_convert_rows and len(args) == 10 and args[1] == _lib.DP_F32 and args[6] == 1 and
                  args[2] == args[5] == args[7] and not args[9] and getattr(args[8], "value", args[8]) == 1.0):
                # dp_convert_rows(src, F32, n, dst, code, n, 1, n, 1.0, 0): a whole-weight copy
                rows.append((args[0], args[3], None, args[2], 1, 1, 1, 0, 0, 5, args[4]))
            else:
                rest.append((name, fn, args))
        if len(rows) < 2:
            return
        n = len(rows)
        tab = (_lib.PackDesc * n)()
        for i, (w, out, scale, cout, cin, kh, kw, kpad, kc, mode, dt) in enumerate(rows):
            tab[i] = _lib.PackDesc(w, out, scale, cout, cin, kh, kw, kpad, kc, mode, dt)
        _lib.check(lib.dp_conv_pack_check(tab, n), "pack table")
        dev = torch.frombuffer(bytearray(bytes(tab)), dtype=torch.uint8).to(self.device)
        self.keep.append(dev)
        self.ops = [("pack.batch", lib.dp_conv_pack_batch, (_p(dev), n, 64))] + rest
        self._graph = None

    @staticmethod
    def segments(ops):
        """The tape cut at its host ops: [("device", [ops...]) | ("host", op)] in tape order, no
        empty device runs."""
        segs, run = [], []
        for op in ops:
            if getattr(op[1], "host", False):
                if run:
                    segs.append(("device", run))
                    run = []
                segs.append(("host", op))
            else:
                run.append(op)
        if run:
            segs.append(("device", run))
        return segs

    def _capture(self):
        out = []
        for kind, x in self.segments(self.ops):
            if kind == "device":
                g = torch.cuda.CUDAGraph()
                with torch.cuda.graph(g):
                    self._launch(None, None, x)
                out.append(("graph", g))
            else:
                out.append(("host", x))
        return out

    def run(self, stream=None, debug=None):
        if self.use_graph and stream is None and debug is None and self.runs > 0:
            if self._graph is None:
                self._graph = self._capture()
            for kind, x in self._graph:
                if kind == "graph":
                    x.replay()
                else:
                    self._launch(None, None, [x])
        else:
            self._launch(stream, debug)
        self.runs += 1


def _p(t, off=0):
    return t.data_ptr() + off * t.element_size()


class TrainEngine:
    """Transformer training step for a DETRPose module (reference parameter names).

    dtype 'fp32' (parity mode) or 'bf16' (bf16 activations and activation gradients, f32
    accumulation, f32 LayerNorm statistics, f32 heads and parameter gradients)."""

    def __init__(self, model, dtype="fp32", device="cuda", train_encoder=False, train_backbone=False):
        self.lib = _lib.load()
        self.train_encoder = train_encoder = train_encoder or train_backbone
        self.train_backbone = train_backbone
        self.model = model
        self.tr = tr = model.transformer
        self.dtype_name = dtype
        self.tdtype, self.code = DT[dtype]
        self.device = torch.device(device)
        self.C = tr.hidden_dim
        self.nh = tr.nhead
        self.nq = tr.num_queries
        self.K = tr.num_body_points
        self.T = self.K + 1
        self.L = tr.num_decoder_layers
        self.nlev = tr.num_feature_levels
        self.npnt = tr.dec_n_points
        self.F = tr.dim_feedforward
        self.reg_max = tr.reg_max
        self.nb = 2 * (tr.reg_max + 1)
        self.ncls = tr.num_classes
        # parameters: one f32 master buffer (the optimizer's), gradients and AdamW moments of
        # the same layout, views under the reference names
        # the transformer's parameters; with train_encoder also the HybridEncoder's
        # (detrpose_amd/encoder_train.py), whose BatchNorm running statistics live in `running`
        pref = (T_, "encoder.") if train_encoder else (T_,)
        if train_backbone:   # (detrpose_amd/backbone_train.py)
            pref = pref + ("backbone.",)
        self.pnames = [n for n, p in model.named_parameters() if n.startswith(pref) and p.requires_grad]
        shapes = {n: tuple(p.shape) for n, p in model.named_parameters()}
        # each parameter starts on a 256-byte boundary (16-byte vector loads of any view)
        sizes = [(int(np.prod(shapes[n])) + 63) // 64 * 64 for n in self.pnames]
        total = sum(sizes)
        dev = self.device
        self.master = torch.zeros(total, dtype=torch.float32, device=dev)
        self.grad_flat = torch.zeros(total, dtype=torch.float32, device=dev)
        self.exp_avg = torch.zeros(total, dtype=torch.float32, device=dev)
        self.exp_avg_sq = torch.zeros(total, dtype=torch.float32, device=dev)
        self.sqnorm = torch.zeros(1, dtype=torch.float32, device=dev)   # ||g||^2 (dp_grad_sqnorm)
        self.sqnorm_ws = torch.zeros(max(1, self.lib.dp_grad_sqnorm_ws_floats(total)), dtype=torch.float32, device=dev)
        self.bad = torch.zeros(1, dtype=torch.float32, device=dev)   # step guard (dp_finite_guard)
        self.grad_acc = None   # gradient-accumulation buffer (accumulate_grads)
        self.opt_step = 0
        self.grads, self.params = {}, {}
        o = 0
        self.offsets = {}
        for n, sz in zip(self.pnames, sizes):
            k = int(np.prod(shapes[n]))
            self.grads[n] = self.grad_flat[o:o + k].view(shapes[n])
            self.params[n] = self.master[o:o + k].view(shapes[n])
            self.offsets[n] = (o, o + sz)
            o += sz
        # the backbone's parameters are one leading range of the flat buffers (module order):
        # its own AdamW learning rate (configs/detrpose/detrpose_hgnetv2_*.py: '^(?=.*backbone).*$')
        bbn = [n for n in self.pnames if n.startswith("backbone.")]
        self.bb_end = self.offsets[bbn[-1]][1] if bbn else 0
        nbb = len(bbn)
        assert self.pnames[:nbb] == bbn, "backbone parameters must lead the flat buffer"
        assert all(self.offsets[n][0] >= self.bb_end for n in self.pnames[nbb:]), \
            "a non-backbone parameter inside the backbone learning-rate range"
        self.ema = None
        self.ema_updates = 0
        # the encoder's BatchNorm running statistics: views of ONE flat f32 buffer, so ModelEMA's
        # update of all of them is one launch (was one per tensor: 178 per L step)
        self.running = {}
        self.running_flat = None
        if train_encoder:
            rb = [(n, b) for n, b in model.named_buffers()
                  if n.startswith("encoder.") and (n.endswith(".running_mean") or n.endswith(".running_var"))]
            rsz = [(b.numel() + 63) // 64 * 64 for _, b in rb]
            self.running_flat = torch.zeros(max(sum(rsz), 1), dtype=torch.float32, device=dev)
            ro = 0
            for (n, b), sz in zip(rb, rsz):
                v = self.running_flat[ro:ro + b.numel()].view(b.shape)
                v.copy_(b.detach().to(dev, torch.float32))
                self.running[n] = v
                ro += sz
        self.load_weights()
        self.plans = {}          # TrainPlan per (batch, DN pad, shapes, ...), LRU order
        self.max_plans = 6
        self.enc_plans = {}

    # ------------------------------------------------------------------ weights
    def load_weights(self):
        """Copy the module's parameters into the f32 master and pack: dtype copies for the
        GEMMs, f32 biases / norms / embeddings / the LQE MLP (f32 inputs). Later calls update
        every packed buffer IN PLACE (recorded tapes hold their pointers)."""
        sd = {k: v.detach() for k, v in self.model.state_dict().items()}
        dev = self.device
        with torch.no_grad():
            for n in self.pnames:
                self.params[n].copy_(sd[n].to(dev, torch.float32))
        if getattr(self, "sd32", None) is not None:
            with torch.no_grad():
                for k, v in sd.items():
                    if k.startswith(T_) and k not in self.params and k in self.sd32:
                        self.sd32[k].copy_(v.to(dev, torch.float32))
            self.refresh()
            return
        self.sd32 = {}
        for k, v in sd.items():
            if not k.startswith(T_):
                continue
            self.sd32[k] = self.params[k] if k in self.params else v.to(dev, torch.float32).contiguous()
        self.w = {}
        for k, v in self.sd32.items():
            if k.endswith("weight") and v.dim() == 2:
                self.w[k] = v if self.tdtype == torch.float32 else v.to(self.tdtype).contiguous()
        for l in range(self.L):
            ca = f"{T_}decoder.layers.{l}.cross_attn."
            self.w[ca + "offattn.weight"] = torch.cat([self.sd32[ca + "sampling_offsets.weight"],
                                                       self.sd32[ca + "attention_weights.weight"]], 0).to(
                self.tdtype).contiguous()
            self.sd32[ca + "offattn.bias"] = torch.cat([self.sd32[ca + "sampling_offsets.bias"],
                                                        self.sd32[ca + "attention_weights.bias"]], 0).contiguous()
            # the f32 concatenation too (the fp32 mode's GEMM weight itself), so the input gradient
            # packs its W^T from it and runs on the 1x1 conv kernel (TrainEngine.dgrad) instead of
            # dp_gemm's 64 x 64 tiles (K = 288 output columns: 48 -> ~15 us per layer)
            wc = self.w[ca + "offattn.weight"]
            self.sd32[ca + "offattn.weight"] = wc if wc.dtype == torch.float32 else torch.cat(
                [self.sd32[ca + "sampling_offsets.weight"], self.sd32[ca + "attention_weights.weight"]], 0).contiguous()
        self._derived(sd)

    def _derived(self, sd):
        """Constants computed from the parameters (the masked-row LN value) and buffers."""
        dev = self.device
        g, b = self.sd32[T_ + "enc_output_norm.weight"].double(), self.sd32[T_ + "enc_output_norm.bias"].double()
        bias = self.sd32[T_ + "enc_output.bias"].double()
        mr = (bias - bias.mean()) / torch.sqrt(bias.var(unbiased=False) + 1e-5) * g + b
        if getattr(self, "masked_row", None) is None:
            self.masked_row = mr.float().contiguous()
        else:
            self.masked_row.copy_(mr.float())
        self.mask_u8 = sd[T_ + "valid_mask"].reshape(-1).to(dev, torch.uint8).contiguous()
        self.anchors = sd[T_ + "anchors"].reshape(-1, 2).to(dev, torch.float32).contiguous()
        tr = self.tr
        self.project = weighting_function(tr.reg_max, float(sd[T_ + "up"]), float(sd[T_ + "reg_scale"])).to(
            dev, torch.float32).contiguous()
        self.reg_scale = abs(float(sd[T_ + "reg_scale"]))
        self.dim_t = sd[T_ + "decoder.dim_t"].to(dev, torch.float32).contiguous()

    def refresh(self, stream=None):
        """After an optimizer step on the master: the dtype GEMM copies (bf16 mode), the fused
        offsets | logits weights and the masked-row constant follow the new values (in place:
        the recorded tapes keep their pointers)."""
        with torch.no_grad():
            copies = []   # (f32 source, destination): every copy of this refresh
            if self.tdtype != torch.float32:
                # (the offsets | logits concatenations: from the masters below, never through the f32
                # concatenation, whose own copy runs in the same unordered batch)
                copies += [(v, self.w[k]) for k, v in self.sd32.items()
                           if k in self.w and self.w[k] is not v and not k.endswith("offattn.weight")]
            for l in range(self.L):
                ca = f"{T_}decoder.layers.{l}.cross_attn."
                no = self.sd32[ca + "sampling_offsets.weight"].shape[0]
                if self.sd32[ca + "offattn.weight"] is not self.w[ca + "offattn.weight"]:
                    copies += [(self.sd32[ca + "sampling_offsets.weight"], self.sd32[ca + "offattn.weight"][:no]),
                               (self.sd32[ca + "attention_weights.weight"], self.sd32[ca + "offattn.weight"][no:])]
                copies += [(self.sd32[ca + "sampling_offsets.weight"], self.w[ca + "offattn.weight"][:no]),
                           (self.sd32[ca + "attention_weights.weight"], self.w[ca + "offattn.weight"][no:]),
                           (self.sd32[ca + "sampling_offsets.bias"], self.sd32[ca + "offattn.bias"][:no]),
                           (self.sd32[ca + "attention_weights.bias"], self.sd32[ca + "offattn.bias"][no:])]
            self._refresh_copies(copies, stream)
            g, b = self.sd32[T_ + "enc_output_norm.weight"].double(), self.sd32[T_ + "enc_output_norm.bias"].double()
            bias = self.sd32[T_ + "enc_output.bias"].double()
            self.masked_row.copy_(((bias - bias.mean()) / torch.sqrt(bias.var(unbiased=False) + 1e-5) * g + b).float())
        for p in self.plans.values():
            p.refresh_constants()

    def _refresh_copies(self, copies, stream=None):
        """The refresh's weight copies: on the GPU one dp_conv_pack_batch launch (mode 5: a plain
        f32 -> dtype copy per table entry; the table is built once, the tensors never move), else
        torch copies."""
        if self.device.type != "cuda" or os.environ.get("DETRPOSE_PACK_BATCH", "1") == "0":
            for src, dst in copies:
                dst.copy_(src)
            return
        if getattr(self, "_refresh_tab", None) is None:
            n = len(copies)
            tab = (_lib.PackDesc * n)()
            for i, (src, dst) in enumerate(copies):
                assert src.dtype == torch.float32 and src.is_contiguous() and dst.is_contiguous()
                assert src.numel() == dst.numel() < 2 ** 31
                code = DP_F32 if dst.dtype == torch.float32 else self.code
                tab[i] = _lib.PackDesc(_p(src), _p(dst), None, src.numel(), 1, 1, 1, 0, 0, 5, code)
            _lib.check(self.lib.dp_conv_pack_check(tab, n), "refresh table")
            dev = torch.frombuffer(bytearray(bytes(tab)), dtype=torch.uint8).to(self.device)
            self._refresh_tab = (dev, n, [(src.data_ptr(), dst.data_ptr()) for src, dst in copies])
        dev, n, ptrs = self._refresh_tab
        assert ptrs == [(src.data_ptr(), dst.data_ptr()) for src, dst in copies], "refresh tensors moved"
        s = stream if stream is not None else C.c_void_p(torch.cuda.current_stream(self.device).cuda_stream)
        _lib.check(self.lib.dp_conv_pack_batch(_p(dev), n, 64, s), "refresh copies")

    def optimizer_step(self, lr=1e-4, betas=(0.9, 0.999), eps=1e-8, weight_decay=1e-4, max_norm=0.1,
                       backbone_lr=1e-5):
        """clip_grad_norm_(max_norm) over every trained parameter + AdamW (src/solver/
        engine.py:78-89, configs: AdamW lr 1e-4 (backbone 1e-5), wd 1e-4, clip 0.1) on the flat
        buffers: one norm launch, one AdamW launch per learning-rate range, no host
        synchronisation."""
        lib = self.lib
        s = C.c_void_p(torch.cuda.current_stream(self.device).cuda_stream)
        n = self.master.numel()
        # host counters (AdamW bias correction here, the EMA warm-up in ema_update): a step the
        # device guard skips still advances them. The reference never continues past a
        # non-finite loss (engine.py:62-66 exits), so no reference behaviour is matched or broken
        # by it; keeping them host-side keeps the update free of host synchronisation.
        self.opt_step += 1
        if max_norm and max_norm > 0:
            _lib.check(lib.dp_grad_sqnorm(_p(self.grad_flat), n, _p(self.sqnorm), _p(self.sqnorm_ws),
                                              self.sqnorm_ws.numel(), s), "dp_grad_sqnorm")
            _lib.check(lib.dp_finite_guard(_p(self.sqnorm), 1, _p(self.bad), s), "dp_finite_guard")
        for o0, o1, lr_ in ((0, self.bb_end, backbone_lr), (self.bb_end, n, lr)):
            if o1 > o0:
                _lib.check(lib.dp_adamw(_p(self.master, o0), _p(self.grad_flat, o0), _p(self.exp_avg, o0),
                                        _p(self.exp_avg_sq, o0), o1 - o0, lr_, betas[0], betas[1], eps, weight_decay,
                                        self.opt_step, max_norm if max_norm else 0.0, _p(self.sqnorm), _p(self.bad),
                                        s), "dp_adamw")
        self.refresh()

    def step_ok_reset(self):
        """Clear the step guard (dp_finite_guard sets it; dp_adamw / dp_ema skip while set)."""
        s = C.c_void_p(torch.cuda.current_stream(self.device).cuda_stream)
        _lib.check(self.lib.dp_zero(_p(self.bad), 4, s), "guard reset")

    def check_finite(self, vals):
        """Set the step guard when any of the device losses `vals` is not finite."""
        s = C.c_void_p(torch.cuda.current_stream(self.device).cuda_stream)
        _lib.check(self.lib.dp_finite_guard(_p(vals), vals.numel(), _p(self.bad), s), "dp_finite_guard")

    def step_skipped(self) -> bool:
        """Whether the last optimizer step was skipped by the guard (synchronises)."""
        return float(self.bad) != 0.0

    def accumulate_grads(self, first: bool, last: bool, lo: int = 0, hi: int = None):
        """Gradient accumulation over sub-batches (engine.py:43-59: .grad sums over the loop's
        backward calls): every backward overwrites grad_flat, so sub-batch j's gradient is added
        into grad_acc, and the last one's grad_flat receives the sum (2 passes over the flat
        buffer per step for 2 sub-batches). [lo, hi): one range of the flat buffer (a DDP bucket)."""
        if first and last:
            return
        s = C.c_void_p(torch.cuda.current_stream(self.device).cuda_stream)
        hi = self.grad_flat.numel() if hi is None else hi
        n = hi - lo
        if self.grad_acc is None:
            self.grad_acc = torch.empty_like(self.grad_flat)
        src, dst, acc = (self.grad_acc, self.grad_flat, 1) if last else (self.grad_flat, self.grad_acc, 0 if first else 1)
        _lib.check(self.lib.dp_convert_rows(_p(src, lo), DP_F32, n, _p(dst, lo), DP_F32, n, 1, n, C.c_float(1.0), acc,
                                            s), "grad accumulate")

    def grad_buckets(self):
        """DDP buckets of the flat gradient in the order the backward finishes them: [(part, lo,
        hi)] for the transformer, the encoder, the backbone (each part's parameters are one range
        of the flat buffer, module order backbone | encoder | transformer)."""
        out = []
        for pre in ("transformer.", "encoder.", "backbone."):
            ns = [n for n in self.pnames if n.startswith(pre)]
            if not ns:
                continue
            i0 = self.pnames.index(ns[0])
            assert self.pnames[i0:i0 + len(ns)] == ns, f"{pre} parameters are not one range of the flat buffer"
            out.append((pre[:-1], self.offsets[ns[0]][0], self.offsets[ns[-1]][1]))
        assert sum(h - l for _, l, h in out) == sum(b - a for a, b in self.offsets.values())
        return out

    def ema_init(self):
        self.ema = self.master.clone()
        self.ema_running_flat = self.running_flat.clone() if self.running_flat is not None else None
        self.ema_running = {}
        for k, v in self.running.items():   # same offsets as the running views
            o = (v.data_ptr() - self.running_flat.data_ptr()) // 4
            self.ema_running[k] = self.ema_running_flat[o:o + v.numel()].view(v.shape)
        self.ema_updates = 0

    def ema_update(self, decay=0.9999, warmups=2000):
        """ModelEMA.update (src/nn/optimizer/ema.py:55-70) over the trained parameters and the
        BatchNorm running statistics: v = d v + (1 - d) p, d = decay (1 - exp(-updates / warmups)),
        from the copy ema_init() took (ModelEMA deep-copies the model when it is built)."""
        lib = self.lib
        s = C.c_void_p(torch.cuda.current_stream(self.device).cuda_stream)
        if self.ema is None:
            self.ema_init()
        self.ema_updates += 1
        d = decay * (1 - math.exp(-self.ema_updates / warmups)) if warmups else decay
        pairs = [(self.ema, self.master)]
        if self.running:   # every running statistic in one launch (the pads are zero in both)
            pairs.append((self.ema_running_flat, self.running_flat))
        for e, p in pairs:
            _lib.check(lib.dp_ema(_p(e), _p(p), e.numel(), C.c_float(d), _p(self.bad), s), "dp_ema")

    def state_dict_update(self, module=None):
        """Write the master parameters back into the module (reference names)."""
        module = module or self.model
        with torch.no_grad():
            for n, p in module.named_parameters():
                if n in self.params:
                    p.copy_(self.params[n].to(p.device, p.dtype))
            for n, b in module.named_buffers():
                if n in self.running:
                    b.copy_(self.running[n].to(b.device, b.dtype))

    # ------------------------------------------------------------------ launch helpers
    def _gemm(self, tape, name, a, a_rs, a_ks, b, b_ks, b_ns, c, c_rs, m, n, k, in_code, out_code, bias=None,
              alpha=1.0, beta=0.0, act=0, gate=None, gate_rs=0, gate_code=None, batch=1, a_bs=0, b_bs=0, c_bs=0,
              gate_bs=0, colsum=None):
        d = GemmDesc()
        d.a, d.a_bs, d.a_rs, d.a_ks = a, a_bs, a_rs, a_ks
        d.b, d.b_bs, d.b_ks, d.b_ns = b, b_bs, b_ks, b_ns
        d.c, d.c_bs, d.c_rs = c, c_bs, c_rs
        d.batch, d.m, d.n, d.k = batch, m, n, k
        d.in_dtype, d.out_dtype = in_code, out_code
        d.bias = bias
        d.alpha, d.beta, d.act = alpha, beta, act
        d.gate, d.gate_bs, d.gate_rs = gate, gate_bs, gate_rs
        d.gate_dtype = self.code if gate_code is None else gate_code
        d.split_k = 1 if tape.deterministic else 0
        d.colsum = colsum
        tape.keep.append(d)
        tape.op(name, self.lib.dp_gemm, C.byref(d))
        self.cur.cost(name, 2.0 * batch * m * n * k)

    @staticmethod
    def _rows_ok(ptr, ld):
        """A bf16 row operand the 1x1 conv kernel takes: 16-byte aligned rows."""
        return ptr % 16 == 0 and ld % 8 == 0

    def _conv1x1(self, tape, name, x, ldx, rows, w, kpad, cin, cout, out, ldo, bias, act, res=False):
        """out = act(x W^T + bias) [+ out] on the 1x1 conv kernel (conv_stream: weight-stationary
        MFMA tiles streaming the rows), W packed [cout][kpad] bf16; the rows are one image of
        1 x rows pixels. ~10x dp_gemm's rate on the decoder's linears (scripts/gemm_bench.py)."""
        d = ConvDesc()
        d.in_, d.in_bstride, d.in_pstride, d.in_h, d.in_w, d.cin = x, rows * ldx, ldx, 1, rows, cin
        d.weight, d.kpad, d.bias = w, kpad, bias
        d.kh, d.kw, d.stride, d.pad_t, d.pad_l = 1, 1, 1, 0, 0
        d.out, d.out_bstride, d.out_pstride, d.out_h, d.out_w, d.cout = out, rows * ldo, ldo, 1, rows, cout
        if res:   # out += ...: the residual read and the store are the same element of the same thread
            d.res, d.res_bstride, d.res_pstride = out, rows * ldo, ldo
        d.batch, d.act, d.dtype = 1, act, DP_BF16
        tape.keep.append(d)
        tape.op(name, self.lib.dp_conv2d, C.byref(d))
        self.cur.cost(name, 2.0 * rows * cin * cout)

    def _wt_pack(self, wkey):
        """W^T of a linear's weight packed [K][pad64(N)] bf16 (dp_conv_pack mode 1 of the f32
        master): the input-gradient conv's weights, re-packed by an op on the current plan's pack
        tape (run before the first forward after every update; Tape.batch_packs merges the
        plan's packs into one launch)."""
        if not hasattr(self, "_wts"):
            self._wts, self._wt_ops = {}, set()
        N, K = self.sd32[wkey].shape
        if wkey not in self._wts:
            kpad = (N + 63) // 64 * 64
            self._wts[wkey] = (torch.zeros(K, kpad, dtype=torch.bfloat16, device=self.device), kpad)
        t, kpad = self._wts[wkey]
        if (id(self.cur), wkey) not in self._wt_ops:
            self._wt_ops.add((id(self.cur), wkey))
            self.cur.pk.op(f"pack.{wkey}.T", self.lib.dp_conv_pack, _p(self.sd32[wkey]), N, K, 1, 1, _p(t), kpad, N, 1,
                           None, DP_BF16)
        return t, kpad

    def _wt_f32(self, wkey):
        """W^T of a linear's weight as f32 [K][N] (dp_conv_pack mode 4 of the f32 master, kpad = N):
        dp_linear_small's weight layout, re-packed on the current plan's pack tape as _wt_pack."""
        if not hasattr(self, "_wtf"):
            self._wtf, self._wtf_ops = {}, set()
        N, K = self.sd32[wkey].shape
        if wkey not in self._wtf:
            self._wtf[wkey] = torch.zeros(K, N, dtype=torch.float32, device=self.device)
        t = self._wtf[wkey]
        if (id(self.cur), wkey) not in self._wtf_ops:
            self._wtf_ops.add((id(self.cur), wkey))
            self.cur.pk.op(f"pack.{wkey}.Tf", self.lib.dp_conv_pack, _p(self.sd32[wkey]), N, K, 1, 1, _p(t), N, 0, 4,
                           None, DP_F32)
        return t

    def lin(self, tape, name, x, ldx, rows, wkey, out, ldo, act=0, out_code=None, bias=True, beta=0.0, wt=None,
            in_code=None):
        """out = act(x W^T + b): nn.Linear forward."""
        W = self.w[wkey] if wt is None else wt
        N, K = W.shape
        bk = wkey[:-len("weight")] + "bias"
        b = self.sd32.get(bk) if bias else None
        ic = self.code if in_code is None else in_code
        oc = self.code if out_code is None else out_code
        if (tape.deterministic and self.code == DP_BF16 and ic == oc == DP_F32 and N <= 128 and rows <= 4096 and ldo == N and act in (0, 1) and
                beta in (0.0, 1.0) and wkey in self.sd32 and os.environ.get("DETRPOSE_TRAIN_LINEAR_SMALL", "1") != "0"):
            # the all-f32 heads of a bf16 forward tape (the LQE Linears over <= 4096 rows; f32 input
            # and f32 weights, as the GEMM had them): one wave per row (dp_linear_small, the inference heads' kernel) instead of a GEMM of a few
            # 64-row tiles whose K-steps each wait a full load latency (the GEMM may not split K here:
            # the forward stays deterministic). The fp32 parity mode keeps the GEMM's summation order
            wT = _p(self.sd32[wkey]) if N == 1 else _p(self._wt_f32(wkey))
            tape.op(name, self.lib.dp_linear_small, x, contiguous_rows(ldx), ic, rows, K, wT,
                    _p(b) if b is not None else None, N, N, act, out if beta == 1.0 else None, out)
            self.cur.cost(name, 2.0 * rows * N * K)
            return
        if (ic == oc == DP_BF16 and K % 64 == 0 and W.is_contiguous() and self._rows_ok(x, ldx) and
                self._rows_ok(out, ldo) and act in (0, 1) and (beta == 0.0 or (beta == 1.0 and act == 0))):
            self._conv1x1(tape, name, x, ldx, rows, _p(W), K, K, N, out, ldo,
                          _p(b) if b is not None else None, act, res=beta == 1.0)
            return
        self._gemm(tape, name, x, ldx, 1, _p(W), 1, K, out, ldo, rows, N, K, self.code if in_code is None else in_code,
                   self.code if out_code is None else out_code, bias=_p(b) if b is not None else None, beta=beta,
                   act=act)

    def dgrad(self, tape, name, dy, ldy, rows, wkey, dx, ldx, beta=0.0, gate=None, ld_gate=0, wt=None, in_code=None,
              gate_code=None):
        """dx (+)= (dy W) [* relu'(gate)]: nn.Linear input gradient."""
        W = self.w[wkey] if wt is None else wt
        N, K = W.shape
        code = self.code if in_code is None else in_code
        gc = self.code if gate_code is None else gate_code
        # (N % 8 != 0: dy's rows are padded to 16 bytes with zeros -- to_dt -- and the kernel reads
        # their last 16-byte chunk whole against zero-padded packed weights)
        if (code == DP_BF16 and wt is None and wkey in self.sd32 and self._rows_ok(dy, ldy) and self._rows_ok(dx, ldx) and
                (beta == 0.0 or (beta == 1.0 and gate is None)) and (gate is None or gc == DP_BF16)):
            Wt, kpad = self._wt_pack(wkey)
            # K of the conv = N rounded up to 8: dy's pad columns are zeros (to_dt) against zero weights
            self._conv1x1(tape, name, dy, ldy, rows, _p(Wt), kpad, -(-N // 8) * 8, K, dx, ldx, None, 0, res=beta == 1.0)
            if gate is not None:   # relu'(gate): the mask applied in place
                tape.op(name + ".mask", self.lib.dp_act_bwd, gate, ld_gate, dx, ldx, dx, ldx, rows, K, 1, code)
            return
        self._gemm(tape, name, dy, ldy, 1, _p(W), K, 1, dx, ldx, rows, K, N, code, code, beta=beta, gate=gate,
                   gate_rs=ld_gate, gate_code=gate_code)

    def wgrad(self, tape, name, dy, ldy, rows, wkey, x, ldx, gkey=None, in_code=None, dy32=None, ld32=None):
        """dW += dy^T x and db += colsum(dy): nn.Linear parameter gradients."""
        gkey = gkey or wkey
        G = self.grads[gkey]
        N, K = G.shape
        code = self.code if in_code is None else in_code
        bk = gkey[:-len("weight")] + "bias"
        fuse = bk in self.grads and dy32 is None   # db += colsum(dy) inside the dW GEMM, which streams dy
        self._gemm(tape, name + ".dW", dy, 1, ldy, x, ldx, 1, _p(G), K, N, K, rows, code, DP_F32, beta=1.0,
                   colsum=_p(self.grads[bk]) if fuse else None)
        if bk in self.grads and not fuse:
            tape.op(name + ".db", self.lib.dp_colsum, dy32, ld32, rows, N, _p(self.grads[bk]), 1, DP_F32)
            self.cur.cost(name + ".db", 4.0 * rows * N)

    # ------------------------------------------------------------------ plan
    def plan(self, batch: int, pad: int, shapes, memory=None, d_memory=None, cut_location_grads=False) -> "TrainPlan":
        """memory: an existing (B, S, C) device buffer of dtype the plan reads the encoder memory
        from (e.g. the inference plan's), instead of its own input buffer. d_memory: a (B, S, C)
        f32 buffer the backward writes d loss / d memory into (the encoder's training step).
        cut_location_grads: a parity-analysis variant whose backward drops the gradient through
        the bilinear sampling locations (MSDA's sampling offsets, the LQE's keypoints) — the
        function's discontinuous part, so precision can be compared per parameter; never for
        training (tests/test_gpu_full_train_step_l.py)."""
        key = (batch, pad, tuple(tuple(s) for s in shapes), memory.data_ptr() if memory is not None else None,
               d_memory.data_ptr() if d_memory is not None else None, bool(cut_location_grads))
        if key in self.plans:
            self.plans[key] = self.plans.pop(key)   # most recently used last
            return self.plans[key]
        # the DN pad (2 x the batch's largest person count x groups) varies from batch to batch on
        # real data: keep the max_plans most recently used plans, drop the rest (their arenas
        # return to the caching allocator)
        while len(self.plans) >= self.max_plans:
            old_key = next(iter(self.plans))
            old = self.plans.pop(old_key)
            if hasattr(self, "_wt_ops"):
                self._wt_ops = {k for k in self._wt_ops if k[0] != id(old)}
            old.arena.clear()
        self.plans[key] = TrainPlan(self, batch, pad, [tuple(s) for s in shapes], memory, d_memory,
                                    cut_location_grads)
        return self.plans[key]

    def encoder_plan(self, batch: int, feat_shapes, feats=None, feats_plan=None):
        """The HybridEncoder's training forward / backward (encoder_train.EncoderTrainPlan);
        feats: the backbone plan's output maps (its input), or None (own input buffers)."""
        assert self.train_encoder, "TrainEngine(train_encoder=True) trains the encoder"
        from .encoder_train import EncoderTrainPlan
        key = (batch, tuple(tuple(s) for s in feat_shapes), id(feats[0].buf) if feats else None)
        if key not in self.enc_plans:
            self.enc_plans[key] = EncoderTrainPlan(self, batch, feat_shapes, feats, feats_plan)
        return self.enc_plans[key]

    def backbone_plan(self, batch: int, h: int, w: int):
        """The HGNetv2 backbone's training forward / backward (backbone_train.BackboneTrainPlan)."""
        assert self.train_backbone, "TrainEngine(train_backbone=True) trains the backbone"
        from .backbone_train import BackboneTrainPlan
        key = ("bb", batch, h, w)
        if key not in self.enc_plans:
            self.enc_plans[key] = BackboneTrainPlan(self, batch, h, w)
        return self.enc_plans[key]


class TrainPlan:
    """Buffers and tapes for one (batch, DN pad size, feature shapes)."""

    def __init__(self, eng: TrainEngine, B: int, P: int, shapes, memory=None, d_memory=None, cut_location_grads=False):
        self.eng = eng
        self.d_memory = d_memory
        self.cut_loc = cut_location_grads
        eng.cur = self
        self.B, self.P, self.shapes = B, P, shapes
        self.op_flops = {}
        self.arena = []
        self._derived = []   # (buffer, parameter) pairs derived from parameters (refresh_constants)
        lib = eng.lib
        Cc, nh, nq, K, T, L, F = eng.C, eng.nh, eng.nq, eng.K, eng.T, eng.L, eng.F
        dt, code = eng.tdtype, eng.code
        e = dt.itemsize
        Qt = P + nq
        self.Qt = Qt
        S = sum(h * w for h, w in shapes)
        self.S = S
        rows, krows, qrows = B * Qt * T, B * Qt * K, B * Qt
        self.rows, self.krows, self.qrows = rows, krows, qrows
        nb, ncol = eng.nb, nh * eng.nlev * eng.npnt * 3
        sd = eng.sd32
        dev = eng.device

        def buf(*shape, dtype=None):
            t = torch.empty(*shape, dtype=dtype or dt, device=dev)
            self.arena.append(t)
            return t

        def f32(*shape):
            return buf(*shape, dtype=torch.float32)

        # ---------------- inputs
        if memory is not None:
            assert memory.dtype == dt and memory.numel() == B * S * Cc and memory.is_contiguous()
            self.memory = memory.view(B, S, Cc)
        else:
            self.memory = buf(B, S, Cc)
        self.dn_label = torch.full((B, max(P, 1)), -1, dtype=torch.int32, device=dev)
        self.dn_ref = f32(B, max(P, 1), T, 2)
        self.mask = torch.zeros(Qt, Qt, dtype=torch.uint8, device=dev)
        self.lvl_hw = (C.c_int32 * (2 * len(shapes)))(*[v for hw in shapes for v in hw])
        # dp_msda_bwd_sorted's workspace (shared by the layers: their backward ops run in order on one
        # stream); None where the shape is outside the sort's range (dp_msda_bwd's atomics then)
        nws = int(lib.dp_msda_bwd_ws_bytes(B, S, self.lvl_hw, len(shapes), Qt * T, nh, eng.npnt))
        sort_ok = nws > 0 and Cc // nh in (8, 16, 32, 64) and os.environ.get("DETRPOSE_MSDA_BWD", "sorted") == "sorted"
        self.msda_ws = buf(nws, dtype=torch.uint8) if sort_ok else None
        fw = Tape(lib, dev)
        fw.deterministic = True
        bw = Tape(lib, dev)
        self.fw, self.bw = fw, bw
        self.pk = Tape(lib, dev)   # weight packs: run once per optimizer step (TrainEngine._wt_pack)
        cr = contiguous_rows
        kp_map = rowmap(Cc, K, T * Cc, Cc)   # keypoint token rows of a [rows][Cc] tensor

        # ================= forward: two-stage selection (transformer.py:1219-1250)
        mrows = B * S
        eo = buf(mrows, Cc)
        eng.lin(fw, "ts.enc_output", _p(self.memory), Cc, mrows, T_ + "enc_output.weight", _p(eo), Cc)
        om = buf(mrows, Cc)
        g_, b_ = sd[T_ + "enc_output_norm.weight"], sd[T_ + "enc_output_norm.bias"]
        fw.op("ts.enc_norm", lib.dp_layernorm, _p(om), cr(Cc), _p(eo), cr(Cc), None, cr(Cc), _p(g_), _p(b_),
              C.c_float(1e-5), mrows, Cc, None, rowmap(group=1), 1, 0, _p(eng.mask_u8), S, _p(eng.masked_row), code)
        score = f32(mrows)
        wc, bc = sd[T_ + "enc_out_class_embed.weight"], sd[T_ + "enc_out_class_embed.bias"]
        fw.op("ts.class_max", lib.dp_class_max, _p(om), mrows, Cc, _p(wc), _p(bc), wc.shape[0], _p(score), code)
        self.topv = f32(B, nq)
        self.topi = torch.empty(B, nq, dtype=torch.int64, device=dev)
        self.arena.append(self.topi)
        fw.op("ts.topk", lib.dp_topk, _p(score), B, S, S, nq, _p(self.topv), _p(self.topi))
        tm = buf(B * nq, Cc)
        fw.op("ts.gather", lib.dp_gather_rows, _p(om), S * Cc, _p(self.topi), B, nq, Cc, _p(tm), code)
        self.interm_logits = f32(B, nq, eng.ncls)
        eng.lin(fw, "ts.interm_cls", _p(tm), Cc, B * nq, T_ + "enc_out_class_embed.weight", _p(self.interm_logits),
                eng.ncls, out_code=DP_F32)
        ep = [buf(B * nq, eng.w[f"{T_}enc_pose_embed.layers.{i}.weight"].shape[0]) for i in range(3)]
        x, ldx = _p(tm), Cc
        for i in range(3):
            eng.lin(fw, f"ts.enc_pose{i}", x, ldx, B * nq, f"{T_}enc_pose_embed.layers.{i}.weight", _p(ep[i]),
                    ep[i].shape[1], act=1)
            x, ldx = _p(ep[i]), ep[i].shape[1]
        delta = f32(B * nq, 2 * K)
        eng.lin(fw, "ts.enc_pose3", x, ldx, B * nq, f"{T_}enc_pose_embed.layers.3.weight", _p(delta), 2 * K,
                out_code=DP_F32)
        self.ref0 = f32(B, nq, T, 2)
        fw.op("ts.refpoints", lib.dp_refpoint_init, _p(delta), _p(eng.anchors), _p(self.topi), B, nq, K, _p(self.ref0))

        # ================= queries (transformer.py:1253-1279, dn_component.py:132-153)
        tgt0 = buf(B, Qt, T, Cc)
        fw.op("q.build", lib.dp_query_build, _p(sd[T_ + "tgt_embed.weight"]), _p(sd[T_ + "keypoint_embedding.weight"]),
              _p(sd[T_ + "instance_embedding.weight"]), _p(sd[T_ + "label_enc.weight"]),
              _p(sd[T_ + "pose_enc.weight"]), _p(self.dn_label), B, P, nq, K, Cc, _p(tgt0), code)
        refs = [f32(B, Qt, T, 2) for _ in range(L + 1)]
        if P:
            fw.op("q.dn_ref", lib.dp_convert_rows, _p(self.dn_ref), DP_F32, P * T * 2, _p(refs[0]), DP_F32,
                  Qt * T * 2, B, P * T * 2, C.c_float(1.0), 0)
        fw.op("q.ref", lib.dp_convert_rows, _p(self.ref0), DP_F32, nq * T * 2, _p(refs[0], P * T * 2), DP_F32,
              Qt * T * 2, B, nq * T * 2, C.c_float(1.0), 0)
        self.refs = refs

        # ================= decoder layers (transformer.py:588-602, 387-442) + heads (701-728)
        lv0 = shapes[0]
        self.L_ = []
        corners = [f32(krows, nb) for _ in range(L)]
        kps = [f32(B, Qt, K, 2) for _ in range(L)]
        logits = [f32(B, Qt, eng.ncls) for _ in range(L)]
        self.pre_out = f32(B, Qt, K, 2)
        self.pre_logits = f32(B, Qt, eng.ncls)
        nhid = eng.sd32[f"{T_}lqe_embed.0.reg_conf.layers.0.weight"].shape[0]
        prev_y = tgt0
        for l in range(L):
            n = f"dec{l}"
            lp = f"{T_}decoder.layers.{l}."
            S_ = {}
            se = buf(krows, Cc)
            fw.op(n + ".sine", lib.dp_sine_embed, _p(refs[l]), qrows, K, Cc, _p(eng.dim_t), _p(se), code)
            ph = buf(krows, Cc)
            pos = buf(krows, Cc)
            hp = f"{T_}decoder.half_pose_ref_point_head.layers."
            eng.lin(fw, n + ".pos0", _p(se), Cc, krows, hp + "0.weight", _p(ph), Cc, act=1)
            eng.lin(fw, n + ".pos1", _p(ph), Cc, krows, hp + "1.weight", _p(pos), Cc)
            x0 = buf(rows, Cc)
            fw.op(n + ".x0", lib.dp_convert_rows, _p(prev_y), code, Cc, _p(x0), code, Cc, rows, Cc, C.c_float(1.0), 0)
            fw.op(n + ".x0pos", lib.dp_add_rows, _p(x0), kp_map, _p(x0), kp_map, _p(pos), cr(Cc), krows, Cc, code)
            # within-instance attention over the T tokens of a query
            qkv_w = buf(rows, 3 * Cc)
            eng.lin(fw, n + ".w_qkv", _p(x0), Cc, rows, lp + "within_attn.in_proj_weight", _p(qkv_w), 3 * Cc)
            att_w = buf(rows, Cc)
            P_w = f32(qrows * nh * T * T)
            fw.op(n + ".w_attn", lib.dp_attn_fwd, _p(qkv_w), 3 * Cc, _p(qkv_w, Cc), _p(qkv_w, 2 * Cc), 3 * Cc, _p(att_w),
                  Cc, _p(P_w), None, qrows, 1, T, 0, 1, T, nh, Cc // nh, code)
            ao_w = buf(rows, Cc)
            eng.lin(fw, n + ".w_out", _p(att_w), Cc, rows, lp + "within_attn.out_proj.weight", _p(ao_w), Cc)
            x1, s_w, st_w = buf(rows, Cc), buf(rows, Cc), f32(rows, 2)
            fw.op(n + ".w_norm", lib.dp_ln_fwd, _p(x1), Cc, _p(x0), _p(ao_w), _p(s_w), _p(st_w),
                  _p(sd[lp + "within_norm.weight"]), _p(sd[lp + "within_norm.bias"]), C.c_float(1e-5), rows, Cc, None,
                  1, 0, code)
            # across-instance attention over the Qt queries of a token slot, DN attn_mask
            qkv_a = buf(rows, 3 * Cc)
            eng.lin(fw, n + ".a_qkv", _p(x1), Cc, rows, lp + "across_attn.in_proj_weight", _p(qkv_a), 3 * Cc)
            att_a = buf(rows, Cc)
            P_a = f32(B * T * nh * Qt * Qt)
            fw.op(n + ".a_attn", lib.dp_attn_fwd, _p(qkv_a), 3 * Cc, _p(qkv_a, Cc), _p(qkv_a, 2 * Cc), 3 * Cc, _p(att_a),
                  Cc, _p(P_a), _p(self.mask) if P else None, B, T, Qt * T, 1, T, Qt, nh, Cc // nh, code)
            ao_a = buf(rows, Cc)
            eng.lin(fw, n + ".a_out", _p(att_a), Cc, rows, lp + "across_attn.out_proj.weight", _p(ao_a), Cc)
            xcat, s_a, st_a = buf(rows, 2 * Cc), buf(rows, Cc), f32(rows, 2)
            # LN + the second in-place pos add (transformer.py:419-422) -> x3 = xcat[:, :Cc]
            fw.op(n + ".a_norm", lib.dp_ln_fwd, _p(xcat), 2 * Cc, _p(x1), _p(ao_a), _p(s_a), _p(st_a),
                  _p(sd[lp + "across_norm.weight"]), _p(sd[lp + "across_norm.bias"]), C.c_float(1e-5), rows, Cc,
                  _p(pos), T, 1, code)
            # MSDA (ms_deform_attn.py:384-444): offsets / logits in f32, output -> xcat[:, Cc:]
            oa = f32(rows, ncol)
            eng.lin(fw, n + ".offattn", _p(xcat), 2 * Cc, rows, lp + "cross_attn.offattn.weight", _p(oa), ncol,
                    out_code=DP_F32)
            fw.op(n + ".msda", lib.dp_msda, _p(self.memory), B, S, self.lvl_hw, len(shapes), _p(oa), _p(refs[l]),
                  _p(xcat, Cc), 2 * Cc, Qt * T, nh, Cc // nh, eng.npnt, code | _lib.DP_MSDA_OFFATTN_F32)
            # Gate (transformer.py:222-235)
            G, gs, z = buf(rows, 2 * Cc), buf(rows, 2 * Cc), buf(rows, Cc)
            eng.lin(fw, n + ".gate", _p(xcat), 2 * Cc, rows, lp + "gateway.gate.weight", _p(G), 2 * Cc)
            fw.op(n + ".gate_fn", lib.dp_gate_fwd, _p(G), _p(xcat), _p(gs), _p(z), rows, Cc, code)
            yg, s_g, st_g = buf(rows, Cc), buf(rows, Cc), f32(rows, 2)
            fw.op(n + ".g_norm", lib.dp_ln_fwd, _p(yg), Cc, _p(z), None, _p(s_g), _p(st_g),
                  _p(sd[lp + "gateway.norm.weight"]), _p(sd[lp + "gateway.norm.bias"]), C.c_float(1e-5), rows, Cc,
                  None, 1, 0, code)
            # FFN (transformer.py:371-385)
            h, f = buf(rows, F), buf(rows, Cc)
            eng.lin(fw, n + ".ffn1", _p(yg), Cc, rows, lp + "linear1.weight", _p(h), F, act=1)
            eng.lin(fw, n + ".ffn2", _p(h), F, rows, lp + "linear2.weight", _p(f), Cc)
            y, s_2, st_2 = buf(rows, Cc), buf(rows, Cc), f32(rows, 2)
            fw.op(n + ".norm2", lib.dp_ln_fwd, _p(y), Cc, _p(yg), _p(f), _p(s_2), _p(st_2), _p(sd[lp + "norm2.weight"]),
                  _p(sd[lp + "norm2.bias"]), C.c_float(1e-5), rows, Cc, None, 1, 0, code)
            # ---- heads. u = output_pose (+ output_pose_detach: the previous output + this layer's
            # pos, i.e. x0's keypoint rows: transformer.py:369/712/913 aliasing)
            u = buf(krows, Cc)
            fw.op(n + ".u", lib.dp_add_rows, _p(u), cr(Cc), _p(y), kp_map, _p(x0) if l > 0 else None, kp_map, krows, Cc,
                  code)
            if l == 0:
                pp = f"{T_}pre_pose_embed.layers."
                pre0, pre1 = buf(krows, Cc), buf(krows, Cc)
                pre = f32(krows, 2)
                eng.lin(fw, "pre0", _p(u), Cc, krows, pp + "0.weight", _p(pre0), Cc, act=1)
                eng.lin(fw, "pre1", _p(pre0), Cc, krows, pp + "1.weight", _p(pre1), Cc, act=1)
                eng.lin(fw, "pre2", _p(pre1), Cc, krows, pp + "2.weight", _p(pre), 2, out_code=DP_F32)
                fw.op("pre_pose", lib.dp_pre_pose, _p(pre), _p(refs[0]), qrows, K, _p(self.pre_out))
                eng.lin(fw, "pre_cls", _p(y), T * Cc, qrows, f"{T_}class_embed.0.weight", _p(self.pre_logits),
                        eng.ncls, out_code=DP_F32)
                S_.update(pre0=pre0, pre1=pre1)
            pe = f"{T_}pose_embed.{l}.layers."
            c0, c1 = buf(krows, Cc), buf(krows, Cc)
            eng.lin(fw, n + ".pose0", _p(u), Cc, krows, pe + "0.weight", _p(c0), Cc, act=1)
            eng.lin(fw, n + ".pose1", _p(c0), Cc, krows, pe + "1.weight", _p(c1), Cc, act=1)
            if l > 0:   # + pred_corners_undetach (transformer.py:712)
                fw.op(n + ".corners_prev", lib.dp_convert_rows, _p(corners[l - 1]), DP_F32, nb, _p(corners[l]), DP_F32,
                      nb, krows, nb, C.c_float(1.0), 0)
            eng.lin(fw, n + ".pose2", _p(c1), Cc, krows, pe + "2.weight", _p(corners[l]), nb, out_code=DP_F32,
                    beta=1.0 if l > 0 else 0.0)
            fw.op(n + ".refine", lib.dp_pose_refine, _p(corners[l]), _p(eng.project), eng.reg_max, _p(self.pre_out),
                  C.c_float(eng.reg_scale), qrows, K, _p(kps[l]), _p(refs[l + 1]))
            eng.lin(fw, n + ".cls", _p(y), T * Cc, qrows, f"{T_}class_embed.{l}.weight", _p(logits[l]), eng.ncls,
                    out_code=DP_F32)
            stt = f32(qrows, K * 5)
            fw.op(n + ".lqe_stats", lib.dp_lqe_stats, _p(self.memory), S * Cc, lv0[0], lv0[1], Cc, _p(kps[l]), B, Qt, K,
                  _p(stt), code)
            hq = f32(qrows, nhid)
            qe = f"{T_}lqe_embed.{l}.reg_conf.layers."
            eng.lin(fw, n + ".lqe0", _p(stt), K * 5, qrows, qe + "0.weight", _p(hq), nhid, act=1, out_code=DP_F32,
                    wt=sd[qe + "0.weight"], in_code=DP_F32)
            # quality score (B, Q, 1) added to every class logit (transformer.py:288 broadcasts): the
            # one output row of reg_conf's last layer read for each of the ncls columns (b_ns = 0)
            w1 = sd[qe + "1.weight"]
            b2 = sd[qe + "1.bias"].repeat(eng.ncls).contiguous()
            self.arena.append(b2)
            self._derived.append((b2, qe + "1.bias"))
            if code == DP_BF16 and os.environ.get("DETRPOSE_TRAIN_LINEAR_SMALL", "1") != "0":
                # w1 [1][nhid] is its own transpose: nw = 1 broadcasts the one output to the ncls columns
                fw.op(n + ".lqe1", lib.dp_linear_small, _p(hq), contiguous_rows(nhid), DP_F32, qrows, nhid, _p(w1),
                      _p(sd[qe + "1.bias"]), 1, eng.ncls, 0, _p(logits[l]), _p(logits[l]))
                self.cost(n + ".lqe1", 2.0 * qrows * eng.ncls * nhid)
            else:
                eng._gemm(fw, n + ".lqe1", _p(hq), nhid, 1, _p(w1), 1, 0, _p(logits[l]), eng.ncls, qrows, eng.ncls,
                          nhid, DP_F32, DP_F32, bias=_p(b2), beta=1.0)
            S_.update(se=se, ph=ph, pos=pos, x0=x0, qkv_w=qkv_w, att_w=att_w, P_w=P_w, x1=x1, s_w=s_w, st_w=st_w,
                      qkv_a=qkv_a, att_a=att_a, P_a=P_a, xcat=xcat, s_a=s_a, st_a=st_a, oa=oa, gs=gs, yg=yg, s_g=s_g,
                      st_g=st_g, h=h, y=y, s_2=s_2, st_2=st_2, u=u, c0=c0, c1=c1, stt=stt, hq=hq)
            self.L_.append(S_)
            prev_y = y
        self.corners, self.kps, self.logits = corners, kps, logits

        # ================= criterion (criterion.py:285-435) -> gradients of the head outputs
        self._criterion_buffers()
        # ================= backward
        self._record_backward(tm, ep, delta)
        if os.environ.get("DETRPOSE_PACK_BATCH", "1") != "0":
            self.pk.batch_packs()

    # ------------------------------------------------------------------ criterion
    def _criterion_buffers(self):
        eng, B, P, nq, K, L = self.eng, self.B, self.P, self.eng.nq, self.eng.K, self.eng.L
        dev = eng.device
        ncls = eng.ncls
        H = L + 2
        self.H = H
        self.hl = torch.empty(H, B, nq, ncls, dtype=torch.float32, device=dev)   # packed heads (match layout)
        self.hk = torch.empty(H, B, nq, 2 * K, dtype=torch.float32, device=dev)
        self.g_lg = torch.empty(H, B, nq, ncls, dtype=torch.float32, device=dev)
        self.g_l1 = torch.empty(H, B, nq, 2 * K, dtype=torch.float32, device=dev)
        self.g_oks = torch.empty(H, B, nq, 2 * K, dtype=torch.float32, device=dev)
        self.losses = torch.empty(H, 3, dtype=torch.float32, device=dev)
        self.match = torch.empty(H, B, nq, dtype=torch.int32, device=dev)
        self.go = torch.empty(B, nq, dtype=torch.int32, device=dev)
        self.n_go = torch.empty(1, dtype=torch.float32, device=dev)
        self.n_boxes = torch.empty(1, dtype=torch.float32, device=dev)
        if P:
            Hd = L + 1
            self.Hd = Hd
            self.dl = torch.empty(Hd, B, P, ncls, dtype=torch.float32, device=dev)
            self.dk = torch.empty(Hd, B, P, 2 * K, dtype=torch.float32, device=dev)
            self.dg_lg = torch.empty(Hd, B, P, ncls, dtype=torch.float32, device=dev)
            self.dg_l1 = torch.empty(Hd, B, P, 2 * K, dtype=torch.float32, device=dev)
            self.dg_oks = torch.empty(Hd, B, P, 2 * K, dtype=torch.float32, device=dev)
            self.dn_losses = torch.empty(Hd, 3, dtype=torch.float32, device=dev)
            self.dn_m = torch.empty(B, P, dtype=torch.int32, device=dev)
            self.n_dn = torch.empty(1, dtype=torch.float32, device=dev)
        # gradients of the head outputs, assembled from the loss kernels
        self.d_logits = [torch.zeros_like(t) for t in self.logits]
        self.d_kps = [torch.zeros_like(t) for t in self.kps]
        self.d_pre_logits = torch.zeros_like(self.pre_logits)
        self.d_pre_out = torch.zeros_like(self.pre_out)
        self.d_interm_logits = torch.zeros_like(self.interm_logits)
        self.d_interm_kps = torch.empty(B, nq, 2 * K, dtype=torch.float32, device=dev)

    def _copy_rows(self, key, entries, s):
        """The f32 row copies `entries` [(dst, ld_dst, src0, ld_src0, src1 | None, ld_src1, rows, n)]
        (pointers) in ONE dp_copy_rows_batch launch; the device table is built once per key (the
        plan's buffers never move) and rebuilt if the pointers change."""
        lib = self.eng.lib
        cache = self.__dict__.setdefault("_row_copies", {})
        ent = tuple(entries)
        got = cache.get(key)
        if got is None or got[2] != ent:
            n = len(ent)
            tab = (_lib.RowCopyDesc * n)()
            for i, (dst, ldd, s0, ld0, s1, ld1, rows, cols) in enumerate(ent):
                tab[i] = _lib.RowCopyDesc(s0, s1, dst, ld0, ld1 if s1 else 0, ldd, rows, cols)
            _lib.check(lib.dp_copy_rows_check(tab, n), "row-copy table " + key)
            dev = torch.frombuffer(bytearray(bytes(tab)), dtype=torch.uint8).to(self.eng.device)
            bpe = max(1, min(64, -(-max(r * c for *_, r, c in ent) // 512)))
            got = cache[key] = (dev, n, ent, bpe)
        dev, n, _, bpe = got
        _lib.check(lib.dp_copy_rows_batch(_p(dev), n, bpe, s), "dp_copy_rows_batch " + key)

    def heads_pack(self):
        """The H heads in the reference's matching order (final, aux 0..L-2, pre, interm) as
        contiguous (B, nq, .) f32 blocks (their matching rows; DN rows separately): one launch."""
        eng = self.eng
        B, P, nq, K, L, Qt, T = self.B, self.P, eng.nq, eng.K, eng.L, self.Qt, eng.T
        ncls = eng.ncls
        s = C.c_void_p(torch.cuda.current_stream(eng.device).cuda_stream)
        order = [L - 1] + list(range(L - 1))
        e = []

        def cp(dst, ldd, src, lds, rows, n):
            e.append((dst, ldd, src, lds, None, 0, rows, n))

        for h, l in enumerate(order):
            cp(_p(self.hl[h]), nq * ncls, _p(self.logits[l], P * ncls), Qt * ncls, B, nq * ncls)
            cp(_p(self.hk[h]), nq * 2 * K, _p(self.kps[l], P * 2 * K), Qt * 2 * K, B, nq * 2 * K)
        cp(_p(self.hl[L]), nq * ncls, _p(self.pre_logits, P * ncls), Qt * ncls, B, nq * ncls)
        cp(_p(self.hk[L]), nq * 2 * K, _p(self.pre_out, P * 2 * K), Qt * 2 * K, B, nq * 2 * K)
        cp(_p(self.hl[L + 1]), nq * ncls, _p(self.interm_logits), nq * ncls, B, nq * ncls)
        # interm keypoints = enc_outputs_pose_coord[:, :, 1:] (skip the centre)
        cp(_p(self.hk[L + 1]), 2 * K, _p(self.ref0, 2), T * 2, B * nq, 2 * K)
        if P:
            for l in range(L):
                cp(_p(self.dl[l]), P * ncls, _p(self.logits[l]), Qt * ncls, B, P * ncls)
                cp(_p(self.dk[l]), P * 2 * K, _p(self.kps[l]), Qt * 2 * K, B, P * 2 * K)
            cp(_p(self.dl[L]), P * ncls, _p(self.pre_logits), Qt * ncls, B, P * ncls)
            cp(_p(self.dk[L]), P * 2 * K, _p(self.pre_out), Qt * 2 * K, B, P * 2 * K)
        self._copy_rows("heads", e, s)

    def criterion(self, packed, sizes, num_group, weights=(2.0, 10.0, 4.0), cost=(2.0, 10.0, 4.0), alpha=0.25,
                  gamma=2.0):
        """Matching + losses + loss gradients (criterion.py:285-435) on the kernels of
        detrpose_amd/criterion.py, then the hand-off into the head-output gradient buffers.
        Returns (loss names, device loss values)."""
        eng, lib = self.eng, self.eng.lib
        B, P, nq, K, L, Qt, H = self.B, self.P, eng.nq, eng.K, eng.L, self.Qt, self.H
        ncls = eng.ncls
        dev = eng.device
        s = C.c_void_p(torch.cuda.current_stream(dev).cuda_stream)
        chk = _lib.check
        self.heads_pack()
        if getattr(self, "_sig", None) is None:
            self._sig = torch.tensor(COCO_SIGMAS if K == 17 else CROWDPOSE_SIGMAS, device=dev)
        sig = self._sig
        max_t = max([int(v) for v in sizes] + [1])
        chk(lib.dp_hungarian_match(_p(self.hl), B * nq * ncls, nq * ncls, ncls, ncls, _p(self.hk), B * nq * 2 * K,
                                   nq * 2 * K, 2 * K, K, _p(packed.off), _p(packed.label), _p(packed.kps),
                                   _p(packed.area), H, B, nq, max_t, cost[0], cost[1], cost[2], alpha, _p(sig),
                                   _p(self.match), None, s), "dp_hungarian_match")
        chk(lib.dp_match_union(_p(self.match), H, B, nq, _p(self.go), _p(self.n_go), s), "dp_match_union")
        self.n_boxes.fill_(float(max(sum(sizes), 0)))
        world = 1
        if torch.distributed.is_available() and torch.distributed.is_initialized():
            # criterion.py:306-323: num_boxes / num_boxes_go summed over the ranks
            from .encoder_train import all_reduce
            all_reduce(self.n_boxes)
            all_reduce(self.n_go)
            world = torch.distributed.get_world_size()
        heads = (_lib.LossHead * H)()
        for h in range(H):
            heads[h] = _lib.LossHead(_p(self.hl[h]), nq * ncls, ncls, _p(self.hk[h]), nq * 2 * K, 2 * K,
                                     _p(self.match[h]))
        chk(lib.dp_pose_loss(heads, H, B, nq, ncls, K, _p(self.go), _p(packed.off), _p(packed.label), _p(packed.kps),
                             _p(packed.area), _p(sig), alpha, gamma, _p(self.n_boxes), _p(self.n_go), float(world),
                             weights[0],
                             weights[1], weights[2], _p(self.losses), _p(self.g_lg), _p(self.g_l1), _p(self.g_oks), s),
            "dp_pose_loss")
        names = ["", *[f"_{i}" for i in range(L - 1)], "_pre", "_enc_0"]
        if P:
            Hd = self.Hd
            # pinned + non-blocking: a pageable copy would make the host wait for the queued forward
            self.dn_m.copy_(torch.from_numpy(dn_match(sizes, P, num_group)).pin_memory(), non_blocking=True)
            # num_boxes (all-reduced, / world, clamped to >= 1: criterion.py:316-322) * num_dn_group
            # (criterion.py:406); dp_pose_loss divides by `world` again, so pass it pre-multiplied
            self.n_dn.copy_(torch.clamp(self.n_boxes / world, min=1.0) * num_group * world)
            dheads = (_lib.LossHead * Hd)()
            for h in range(Hd):
                dheads[h] = _lib.LossHead(_p(self.dl[h]), P * ncls, ncls, _p(self.dk[h]), P * 2 * K, 2 * K,
                                          _p(self.dn_m))
            chk(lib.dp_pose_loss(dheads, Hd, B, P, ncls, K, _p(self.dn_m), _p(packed.off), _p(packed.label),
                                 _p(packed.kps), _p(packed.area), _p(sig), alpha, gamma, _p(self.n_dn), _p(self.n_dn),
                                 float(world), weights[0], weights[1], weights[2], _p(self.dn_losses), _p(self.dg_lg),
                                 _p(self.dg_l1), _p(self.dg_oks), s), "dp_pose_loss(dn)")
        # ---- hand-off: d loss_total / d head outputs
        order = [L - 1] + list(range(L - 1))

        # one launch; keypoint gradients = the L1 part + the OKS part (dst = src0 + src1)
        e = []

        def put(dst, dst_off, ld_dst, src, n, src1=None):
            e.append((_p(dst, dst_off), ld_dst, _p(src), n, _p(src1) if src1 is not None else None, n, B, n))

        for h, l in enumerate(order):
            put(self.d_logits[l], P * ncls, Qt * ncls, self.g_lg[h], nq * ncls)
            put(self.d_kps[l], P * 2 * K, Qt * 2 * K, self.g_l1[h], nq * 2 * K, self.g_oks[h])
        put(self.d_pre_logits, P * ncls, Qt * ncls, self.g_lg[L], nq * ncls)
        put(self.d_pre_out, P * 2 * K, Qt * 2 * K, self.g_l1[L], nq * 2 * K, self.g_oks[L])
        put(self.d_interm_logits, 0, nq * ncls, self.g_lg[L + 1], nq * ncls)
        put(self.d_interm_kps, 0, nq * 2 * K, self.g_l1[L + 1], nq * 2 * K, self.g_oks[L + 1])
        if P:
            for l in range(L):
                put(self.d_logits[l], 0, Qt * ncls, self.dg_lg[l], P * ncls)
                put(self.d_kps[l], 0, Qt * 2 * K, self.dg_l1[l], P * 2 * K, self.dg_oks[l])
            put(self.d_pre_logits, 0, Qt * ncls, self.dg_lg[L], P * ncls)
            put(self.d_pre_out, 0, Qt * 2 * K, self.dg_l1[L], P * 2 * K, self.dg_oks[L])
        self._copy_rows("hand-off", e, s)
        keys = []
        for n in names:
            keys += ["loss_vfl" + n, "loss_keypoints" + n, "loss_oks" + n]
        vals = [self.losses.reshape(-1)]
        if P:
            for n in [*[f"_dn_{i}" for i in range(L)], "_dn_pre"]:
                keys += ["loss_vfl" + n, "loss_keypoints" + n, "loss_oks" + n]
            vals.append(self.dn_losses.reshape(-1))
        return keys, torch.cat(vals)

    # ------------------------------------------------------------------ backward
    def _record_backward(self, tm, ep, delta):
        eng, lib = self.eng, self.eng.lib
        bw = self.bw
        B, P, nq, K, T, L, F, Qt = self.B, self.P, eng.nq, eng.K, eng.T, eng.L, eng.F, self.Qt
        C_, nh = eng.C, eng.nh
        Cc = C_
        code = eng.code
        dt = eng.tdtype
        e = dt.itemsize
        rows, krows, qrows = self.rows, self.krows, self.qrows
        nb, ncol, ncls = eng.nb, nh * eng.nlev * eng.npnt * 3, eng.ncls
        dev = eng.device
        sd = eng.sd32
        cr = contiguous_rows
        kp_map = rowmap(Cc, K, T * Cc, Cc)
        lv0 = self.shapes[0]
        conv = code != DP_F32   # f32 gradients must be converted to dtype for the GEMMs

        def buf(*shape, dtype=None):
            t = torch.empty(*shape, dtype=dtype or dt, device=dev)
            self.arena.append(t)
            return t

        def f32(*shape):
            return buf(*shape, dtype=torch.float32)

        def to_dt(name, src, rows_, n, ld=None):
            """f32 gradient rows as the GEMM dtype (a copy in bf16 mode, the buffer itself in fp32)."""
            if not conv:
                return src, (ld or n)
            # rows padded to a 16-byte multiple: the GEMMs then load whole 16-byte row chunks (the
            # pose head's 66 columns otherwise took dp_gemm's per-element path)
            ldp = -(-n // 8) * 8
            d = buf(rows_, ldp)
            if ldp != n:
                d.zero_()   # the pad columns stay zero (the convert writes the first n)
            bw.op(name, lib.dp_convert_rows, _p(src), DP_F32, ld or n, _p(d), code, ldp, rows_, n, C.c_float(1.0), 0)
            return d, ldp

        def mlp_bwd(name, dout_dt, ld_out, dout32, ld32, rows_, layers, ins, wkeys):
            """Backward of an MLP chain: layers[i] output i (ReLU between); ins[i] input of layer i.
            dout: gradient of the last layer's output. Returns the gradient of ins[0] (a buffer)."""
            d, ldd, d32, l32 = dout_dt, ld_out, dout32, ld32
            for i in range(len(wkeys) - 1, -1, -1):
                x, ldx = ins[i]
                eng.wgrad(bw, f"{name}.l{i}", _p(d), ldd, rows_, wkeys[i], _p(x), ldx, dy32=_p(d32) if d32 is not None
                          else None, ld32=l32)
                W = eng.w[wkeys[i]]
                din = buf(rows_, W.shape[1])
                gate = ins[i][0] if i > 0 else None
                eng.dgrad(bw, f"{name}.l{i}.dx", _p(d), ldd, rows_, wkeys[i], _p(din), W.shape[1],
                          gate=_p(gate) if gate is not None else None, ld_gate=ins[i][1] if i > 0 else 0)
                d, ldd, d32, l32 = din, W.shape[1], None, None
            return d

        self.ones = torch.ones(ncls, dtype=torch.float32, device=dev)
        bw.op("bw.zero", lib.dp_zero, _p(eng.grad_flat), eng.grad_flat.numel() * 4)
        dm = self.d_memory   # d loss / d memory (f32): MSDA value, LQE feats[0], two-stage rows
        if dm is not None:
            assert dm.dtype == torch.float32 and dm.numel() == B * self.S * Cc
            bw.op("bw.zero_dmem", lib.dp_zero, _p(dm), dm.numel() * 4)
        dY = buf(rows, Cc)
        bw.op("bw.dY0", lib.dp_zero, _p(dY), rows * Cc * e)
        dcorn = f32(krows, nb)
        dpos = buf(krows, Cc)
        for l in range(L - 1, -1, -1):
            n = f"bw{l}"
            lp = f"{T_}decoder.layers.{l}."
            S_ = self.L_[l]
            y = S_["y"]
            # ---------------- heads of layer l
            # LQE: logits = score + MLP(stats) (transformer.py:728, 275-288)
            qe = f"{T_}lqe_embed.{l}.reg_conf.layers."
            dlg = self.d_logits[l]
            # d quality = sum over the class columns it was added to
            dq = f32(qrows, 1)
            eng._gemm(bw, n + ".lqe_dq", _p(dlg), ncls, 1, _p(self.ones), 1, 0, _p(dq), 1, qrows, 1, ncls, DP_F32,
                      DP_F32)
            eng.wgrad(bw, n + ".lqe1", _p(dq), 1, qrows, qe + "1.weight", _p(S_["hq"]), S_["hq"].shape[1],
                      in_code=DP_F32)
            nhid = S_["hq"].shape[1]
            dhq = f32(qrows, nhid)
            eng.dgrad(bw, n + ".lqe1.dx", _p(dq), 1, qrows, qe + "1.weight", _p(dhq), nhid, gate=_p(S_["hq"]),
                      ld_gate=nhid, wt=sd[qe + "1.weight"], in_code=DP_F32, gate_code=DP_F32)
            eng.wgrad(bw, n + ".lqe0", _p(dhq), nhid, qrows, qe + "0.weight", _p(S_["stt"]), K * 5, in_code=DP_F32)
            dst = f32(qrows, K * 5)
            eng.dgrad(bw, n + ".lqe0.dx", _p(dhq), nhid, qrows, qe + "0.weight", _p(dst), K * 5, wt=sd[qe + "0.weight"],
                      in_code=DP_F32)
            dkps_lqe = self.d_kps[l]
            if self.cut_loc:   # parity-analysis variant: no gradient through the sampling keypoints
                dkps_lqe = f32(B * Qt * K * 2)
            bw.op(n + ".lqe_stats_bwd", lib.dp_lqe_stats_bwd, _p(self.memory), self.S * Cc, lv0[0], lv0[1], Cc,
                  _p(self.kps[l]), _p(dst), B, Qt, K, _p(dkps_lqe), _p(dm) if dm is not None else None,
                  self.S * Cc, code)
            # class head on the instance token: score = class_embed[l](output[:, :, 0])
            ck = f"{T_}class_embed.{l}.weight"
            dlg_dt, ldl = to_dt(n + ".dlogits", dlg, qrows, ncls)
            eng.wgrad(bw, n + ".cls", _p(dlg_dt), ldl, qrows, ck, _p(y), T * Cc, dy32=_p(dlg), ld32=ncls)
            eng.dgrad(bw, n + ".cls.dx", _p(dlg_dt), ldl, qrows, ck, _p(dY), T * Cc, beta=1.0)
            # Integral + distance2pose, then pred_corners = pose_head(u) + corners_{l-1} (kept
            # undetached: d corners_{l-1} += d corners_l, carried in dcorn)
            bw.op(n + ".refine_bwd", lib.dp_pose_refine_bwd, _p(self.corners[l]), _p(eng.project), eng.reg_max,
                  C.c_float(eng.reg_scale), _p(self.d_kps[l]), qrows, K, _p(dcorn), 1 if l < L - 1 else 0)
            dc_dt, ldc = to_dt(n + ".dcorn", dcorn, krows, nb)
            pe = f"{T_}pose_embed.{l}.layers."
            du = mlp_bwd(n + ".pose", dc_dt, ldc, dcorn, nb, krows, 3,
                         [(S_["u"], Cc), (S_["c0"], Cc), (S_["c1"], Cc)], [pe + "0.weight", pe + "1.weight",
                                                                         pe + "2.weight"])
            bw.op(n + ".du", lib.dp_add_rows, _p(dY), kp_map, _p(dY), kp_map, _p(du), cr(Cc), krows, Cc, code)
            if l == 0:
                # pre head: pre_poses = sigmoid(MLP(output_pose) + inverse_sigmoid(ref)) (transformer.py:707)
                dpre = f32(krows, 2)
                bw.op("bw.pre_sig", lib.dp_sigmoid_bwd, _p(self.pre_out), _p(self.d_pre_out), _p(dpre), krows, 2, 2, 2,
                      2)
                dpre_dt, ldp = to_dt("bw.dpre", dpre, krows, 2)
                pp = f"{T_}pre_pose_embed.layers."
                du0 = mlp_bwd("bw.pre", dpre_dt, ldp, dpre, 2, krows, 3,
                              [(S_["u"], Cc), (S_["pre0"], Cc), (S_["pre1"], Cc)],
                              [pp + "0.weight", pp + "1.weight", pp + "2.weight"])
                bw.op("bw.pre.du", lib.dp_add_rows, _p(dY), kp_map, _p(dY), kp_map, _p(du0), cr(Cc), krows, Cc, code)
                dpl_dt, ldq = to_dt("bw.dpre_logits", self.d_pre_logits, qrows, ncls)
                c0k = f"{T_}class_embed.0.weight"
                eng.wgrad(bw, "bw.pre_cls", _p(dpl_dt), ldq, qrows, c0k, _p(y), T * Cc, dy32=_p(self.d_pre_logits),
                          ld32=ncls)
                eng.dgrad(bw, "bw.pre_cls.dx", _p(dpl_dt), ldq, qrows, c0k, _p(dY), T * Cc, beta=1.0)
            # ---------------- the layer (transformer.py:387-442) in reverse
            # FFN + norm2
            ds2 = buf(rows, Cc)
            bw.op(n + ".norm2", lib.dp_ln_bwd, _p(ds2), _p(dY), Cc, _p(S_["s_2"]), _p(S_["st_2"]),
                  _p(sd[lp + "norm2.weight"]), rows, Cc, _p(eng.grads[lp + "norm2.weight"]),
                  _p(eng.grads[lp + "norm2.bias"]), 0, code)
            eng.wgrad(bw, n + ".ffn2", _p(ds2), Cc, rows, lp + "linear2.weight", _p(S_["h"]), F)
            dh = buf(rows, F)
            eng.dgrad(bw, n + ".ffn2.dx", _p(ds2), Cc, rows, lp + "linear2.weight", _p(dh), F, gate=_p(S_["h"]),
                      ld_gate=F)
            eng.wgrad(bw, n + ".ffn1", _p(dh), F, rows, lp + "linear1.weight", _p(S_["yg"]), Cc)
            eng.dgrad(bw, n + ".ffn1.dx", _p(dh), F, rows, lp + "linear1.weight", _p(ds2), Cc, beta=1.0)   # d yg
            # Gate + its norm
            dz = buf(rows, Cc)
            bw.op(n + ".g_norm", lib.dp_ln_bwd, _p(dz), _p(ds2), Cc, _p(S_["s_g"]), _p(S_["st_g"]),
                  _p(sd[lp + "gateway.norm.weight"]), rows, Cc, _p(eng.grads[lp + "gateway.norm.weight"]),
                  _p(eng.grads[lp + "gateway.norm.bias"]), 0, code)
            dG, dx = buf(rows, 2 * Cc), buf(rows, 2 * Cc)
            bw.op(n + ".gate_fn", lib.dp_gate_bwd, _p(dz), _p(S_["gs"]), _p(S_["xcat"]), _p(dG), _p(dx), rows, Cc, code)
            eng.wgrad(bw, n + ".gate", _p(dG), 2 * Cc, rows, lp + "gateway.gate.weight", _p(S_["xcat"]), 2 * Cc)
            eng.dgrad(bw, n + ".gate.dx", _p(dG), 2 * Cc, rows, lp + "gateway.gate.weight", _p(dx), 2 * Cc, beta=1.0)
            # MSDA: d offsets / logits (dp_msda_bwd), then the offattn Linear
            doa = f32(rows, ncol)
            msda_args = (_p(self.memory), B, self.S, self.lvl_hw, len(self.shapes), _p(S_["oa"]), _p(self.refs[l]),
                         _p(dx, Cc), 2 * Cc, Qt * T, nh, Cc // nh, eng.npnt, _p(dm) if dm is not None else None, 1,
                         _p(doa), None)
            if dm is not None and self.msda_ws is not None:   # value gradient by the per-pixel sort
                bw.op(n + ".msda_bwd", lib.dp_msda_bwd_sorted, *msda_args, _p(self.msda_ws), self.msda_ws.numel(),
                      code)
            else:
                bw.op(n + ".msda_bwd", lib.dp_msda_bwd, *msda_args, code)
            if self.cut_loc:   # parity-analysis variant: d sampling offsets = 0 (the location columns)
                nof = eng.nh * eng.nlev * eng.npnt * 2
                bw.op(n + ".cut_loc", lib.dp_convert_rows, _p(doa), DP_F32, ncol, _p(doa), DP_F32, ncol, rows, nof,
                      C.c_float(0.0), 0)
            doa_dt, ldo = to_dt(n + ".doa", doa, rows, ncol)
            ok = lp + "cross_attn.offattn.weight"
            self._wgrad_offattn(bw, n, doa_dt, ldo, doa, rows, ok, S_["xcat"], lp)
            eng.dgrad(bw, n + ".offattn.dx", _p(doa_dt), ldo, rows, ok, _p(dx), 2 * Cc, beta=1.0)
            # x3 = LN_a(...) + pos on the keypoint rows (transformer.py:422): d pos
            dx3_kp = rowmap(2 * Cc, K, T * 2 * Cc, 2 * Cc)
            bw.op(n + ".dpos", lib.dp_add_rows, _p(dpos), cr(Cc), _p(dx), dx3_kp, None, cr(Cc), krows, Cc, code)
            # across attention + its norm
            da = buf(rows, Cc)
            bw.op(n + ".a_norm", lib.dp_ln_bwd, _p(da), _p(dx), 2 * Cc, _p(S_["s_a"]), _p(S_["st_a"]),
                  _p(sd[lp + "across_norm.weight"]), rows, Cc, _p(eng.grads[lp + "across_norm.weight"]),
                  _p(eng.grads[lp + "across_norm.bias"]), 0, code)
            self._mha_bwd(bw, n + ".a", lp + "across_attn.", da, S_["att_a"], S_["qkv_a"], S_["P_a"], S_["x1"],
                          B, T, Qt * T, 1, T, Qt)
            # within attention + its norm (da now holds d x1)
            dw = buf(rows, Cc)
            bw.op(n + ".w_norm", lib.dp_ln_bwd, _p(dw), _p(da), Cc, _p(S_["s_w"]), _p(S_["st_w"]),
                  _p(sd[lp + "within_norm.weight"]), rows, Cc, _p(eng.grads[lp + "within_norm.weight"]),
                  _p(eng.grads[lp + "within_norm.bias"]), 0, code)
            self._mha_bwd(bw, n + ".w", lp + "within_attn.", dw, S_["att_w"], S_["qkv_w"], S_["P_w"], S_["x0"],
                          qrows, 1, T, 0, 1, T)
            # dw = d x0: x0 = y_{l-1} + pos on the keypoint rows (transformer.py:369)
            bw.op(n + ".dpos2", lib.dp_add_rows, _p(dpos), cr(Cc), _p(dpos), cr(Cc), _p(dw), kp_map, krows, Cc, code)
            hp = f"{T_}decoder.half_pose_ref_point_head.layers."
            eng.wgrad(bw, n + ".pos1", _p(dpos), Cc, krows, hp + "1.weight", _p(S_["ph"]), Cc)
            dph = buf(krows, Cc)
            eng.dgrad(bw, n + ".pos1.dx", _p(dpos), Cc, krows, hp + "1.weight", _p(dph), Cc, gate=_p(S_["ph"]),
                      ld_gate=Cc)
            eng.wgrad(bw, n + ".pos0", _p(dph), Cc, krows, hp + "0.weight", _p(S_["se"]), Cc)
            # the next (earlier) layer's output gradient starts as d x0
            dY = dw
        self.d_tgt0 = dY
        bw.op("bw.query", lib.dp_query_build_bwd, _p(dY), _p(self.dn_label), B, P, nq, K, Cc,
              _p(eng.grads[T_ + "tgt_embed.weight"]), _p(eng.grads[T_ + "keypoint_embedding.weight"]),
              _p(eng.grads[T_ + "instance_embedding.weight"]), _p(eng.grads[T_ + "label_enc.weight"]),
              eng.grads[T_ + "label_enc.weight"].shape[0], _p(eng.grads[T_ + "pose_enc.weight"]), code)
        # ---------------- two-stage (transformer.py:1227-1250), selected rows only
        ddelta = f32(B * nq, 2 * K)
        bw.op("bw.ts.sig", lib.dp_sigmoid_bwd, _p(self.ref0, 2), _p(self.d_interm_kps), _p(ddelta), B * nq, 2 * K,
              T * 2, 2 * K, 2 * K)
        ddelta_dt, ldd = to_dt("bw.ts.ddelta", ddelta, B * nq, 2 * K)
        epk = [f"{T_}enc_pose_embed.layers.{i}.weight" for i in range(4)]
        dtm = mlp_bwd("bw.ts.pose", ddelta_dt, ldd, ddelta, 2 * K, B * nq, 4,
                      [(tm, Cc)] + [(t, t.shape[1]) for t in ep], epk)
        dil_dt, ldi = to_dt("bw.ts.dinterm", self.d_interm_logits, B * nq, ncls)
        ck = f"{T_}enc_out_class_embed.weight"
        eng.wgrad(bw, "bw.ts.cls", _p(dil_dt), ldi, B * nq, ck, _p(tm), Cc, dy32=_p(self.d_interm_logits), ld32=ncls)
        eng.dgrad(bw, "bw.ts.cls.dx", _p(dil_dt), ldi, B * nq, ck, _p(dtm), Cc, beta=1.0)
        xs = buf(B * nq, Cc)
        bw.op("bw.ts.gather", lib.dp_gather_rows_masked, _p(self.memory), self.S * Cc, _p(self.topi), _p(eng.mask_u8),
              self.S, B, nq, Cc, _p(xs), code)
        ssel = buf(B * nq, Cc)
        eng.lin(bw, "bw.ts.enc_output", _p(xs), Cc, B * nq, T_ + "enc_output.weight", _p(ssel), Cc)
        ysel, stsel = buf(B * nq, Cc), f32(B * nq, 2)
        bw.op("bw.ts.enc_norm_fwd", lib.dp_ln_fwd, _p(ysel), Cc, _p(ssel), None, None, _p(stsel),
              _p(sd[T_ + "enc_output_norm.weight"]), _p(sd[T_ + "enc_output_norm.bias"]), C.c_float(1e-5), B * nq, Cc,
              None, 1, 0, code)
        dsel = buf(B * nq, Cc)
        bw.op("bw.ts.enc_norm", lib.dp_ln_bwd, _p(dsel), _p(dtm), Cc, _p(ssel), _p(stsel),
              _p(sd[T_ + "enc_output_norm.weight"]), B * nq, Cc, _p(eng.grads[T_ + "enc_output_norm.weight"]),
              _p(eng.grads[T_ + "enc_output_norm.bias"]), 0, code)
        eng.wgrad(bw, "bw.ts.enc_output", _p(dsel), Cc, B * nq, T_ + "enc_output.weight", _p(xs), Cc)
        if dm is not None:
            # d memory on the selected rows (memory.masked_fill(~valid_mask, 0): none to masked rows)
            dxs = f32(B * nq, Cc)
            W = eng.w[T_ + "enc_output.weight"]
            eng._gemm(bw, "bw.ts.enc_output.dx", _p(dsel), Cc, 1, _p(W), Cc, 1, _p(dxs), Cc, B * nq, Cc, Cc, code,
                      DP_F32)
            bw.op("bw.ts.dmem", lib.dp_scatter_rows, _p(dxs), Cc, _p(self.topi), _p(eng.mask_u8), self.S, B, nq, Cc,
                  _p(dm), self.S * Cc, Cc, 1, DP_F32)

    def _wgrad_offattn(self, bw, n, doa_dt, ldo, doa32, rows, okey, xcat, lp):
        """The fused offsets | logits Linear's weight / bias gradients, written into the two
        reference parameters (sampling_offsets, attention_weights)."""
        eng, lib = self.eng, self.eng.lib
        Cc = eng.C
        no = eng.grads[lp + "cross_attn.sampling_offsets.weight"].shape[0]
        na = eng.grads[lp + "cross_attn.attention_weights.weight"].shape[0]
        for key, c0, nn in (("sampling_offsets", 0, no), ("attention_weights", no, na)):
            G = eng.grads[lp + f"cross_attn.{key}.weight"]
            eng._gemm(bw, f"{n}.{key}.dW", _p(doa_dt, c0), 1, ldo, _p(xcat), 2 * Cc, 1, _p(G), Cc, nn, Cc, rows,
                      eng.code, DP_F32, beta=1.0)
            bw.op(f"{n}.{key}.db", lib.dp_colsum, _p(doa32, c0), doa32.shape[1], rows, nn,
                  _p(eng.grads[lp + f"cross_attn.{key}.bias"]), 1, DP_F32)

    def _mha_bwd(self, bw, n, ap, dsum, att, qkv, Pbuf, xin, n_outer, n_inner, so, si, st, L):
        """nn.MultiheadAttention backward (q = k = v = xin): dsum (the LN backward's output, d of
        the residual sum) is the out_proj gradient; on return dsum holds d xin."""
        eng, lib = self.eng, self.eng.lib
        Cc, nh, code = eng.C, eng.nh, eng.code
        rows = self.rows
        eng.wgrad(bw, n + ".out", _p(dsum), Cc, rows, ap + "out_proj.weight", _p(att), Cc)
        datt = self._scratch(("datt", rows, Cc), rows, Cc)
        eng.dgrad(bw, n + ".out.dx", _p(dsum), Cc, rows, ap + "out_proj.weight", _p(datt), Cc)
        dqkv = self._scratch(("dqkv", rows, 3 * Cc), rows, 3 * Cc)
        bw.op(n + ".attn_bwd", lib.dp_attn_bwd, _p(qkv), 3 * Cc, _p(qkv, Cc), _p(qkv, 2 * Cc), 3 * Cc, _p(Pbuf),
              _p(datt), _p(att), Cc, _p(dqkv), 3 * Cc, _p(dqkv, Cc), _p(dqkv, 2 * Cc), 3 * Cc, n_outer, n_inner, so, si, st, L,
              nh, Cc // nh, code)
        eng.wgrad(bw, n + ".in", _p(dqkv), 3 * Cc, rows, ap + "in_proj_weight", _p(xin), Cc)
        eng.dgrad(bw, n + ".in.dx", _p(dqkv), 3 * Cc, rows, ap + "in_proj_weight", _p(dsum), Cc, beta=1.0)

    def _scratch(self, key, *shape):
        if not hasattr(self, "_scr"):
            self._scr = {}
        if key not in self._scr:
            t = torch.empty(*shape, dtype=self.eng.tdtype, device=self.eng.device)
            self.arena.append(t)
            self._scr[key] = t
        return self._scr[key]

    def cost(self, name, flops):
        self.op_flops[name] = self.op_flops.get(name, 0.0) + flops

    # ------------------------------------------------------------------ inputs / run
    def set_inputs(self, memory, dn=None):
        """memory (B, S, C) (encoder output levels flattened, any float dtype, on the device);
        dn: {'label' (B, pad) int (-1 = padding), 'pose_unsig' (B, pad, 1+K, 2), 'attn_mask'
        (pad+nq, pad+nq) bool} or None (pad must be 0)."""
        self.memory.copy_(memory.to(self.memory.dtype))
        if self.P:
            self.dn_label.copy_(torch.as_tensor(dn["label"], dtype=torch.int32))
            self.dn_ref.copy_(torch.sigmoid(torch.as_tensor(dn["pose_unsig"], dtype=torch.float32)))
            self.mask.copy_(torch.as_tensor(dn["attn_mask"]).to(torch.uint8))

    def set_dn(self, dn_label, dn_ref, mask):
        """DN draws already on the device (dp_cdn_build): dn_label (B, pad) int32, dn_ref
        (B, pad, 1+K, 2) f32 reference points, mask (Qt, Qt) uint8."""
        if self.P:
            self.dn_label.copy_(dn_label)
            self.dn_ref.copy_(dn_ref)
            self.mask.copy_(mask)

    def refresh_constants(self):
        with torch.no_grad():
            for buf_, key in self._derived:
                buf_.copy_(self.eng.sd32[key].repeat(buf_.numel() // self.eng.sd32[key].numel()))

    def forward(self, debug=None, pack=True):
        """pack=False: the weight packs of an earlier sub-batch of the same step are current."""
        if pack:
            self.pk.run(debug=debug)
        self.fw.run(debug=debug)

    def backward(self, debug=None):
        self.bw.run(debug=debug)


def encoder_memory(eng_inf, images):
    """The encoder output (B, S, C) of the inference engine's backbone + encoder for images:
    the training transformer's input (frozen BN, detached)."""
    plan = eng_inf.plan(images.shape[0])
    plan.input.copy_(images)
    plan.run()
    return plan.bufs["memory"].view(images.shape[0], -1, eng_inf.tr.hidden_dim)
