"""One DETRPose training step on the HIP kernels (BASELINE config 5):

    images -> backbone forward (backbone_train: FrozenBatchNorm2d folded per step)
           -> encoder training forward (encoder_train: BatchNorm on batch statistics, SyncBN)
           -> OKS-denoising draws (dp_cdn_build)  -> transformer training forward (TrainPlan)
           -> Hungarian matching + losses + their gradients (incl. dn_*)
           -> transformer backward (+ d memory) -> encoder backward -> backbone backward
           -> gradient all-reduce over RCCL (DDP's mean, when initialised)
           -> clip_grad_norm_(0.1) + AdamW (backbone lr 1e-5, the rest 1e-4) -> ModelEMA update

Reference: src/solver/engine.py:34-95 (train_one_epoch: model(samples, targets), criterion,
sum of the loss dict, backward, clip_grad_norm_, optimizer.step, ema.update), the DN construction
of src/models/detrpose/dn_component.py:39-183, the optimizer / EMA of
configs/detrpose/detrpose_hgnetv2_*.py, DDP and SyncBN (src/misc/dist_utils.py:111-133).
scope="transformer" keeps the earlier variant: backbone + encoder frozen (the inference plan's
launches up to the memory, BatchNorm in eval mode), only the transformer trained.
"""
from __future__ import annotations

import ctypes as C
import os

import numpy as np
import torch

from . import _lib
from .criterion import COCO_SIGMAS, CROWDPOSE_SIGMAS, pack_targets
from .encoder_train import all_reduce
from .train_engine import TrainEngine, _p


def dn_meta(sizes, dn_number=20):
    """dn_component.py:54-63, 113-114: (pad_size, num_dn_group, single_pad) or None."""
    known = max([int(s) for s in sizes] + [0])
    if known == 0:
        return None
    groups = max((dn_number * 2) // (known * 2), 1)
    return known * 2 * groups, groups, known


def dn_attn_mask(pad, groups, single, nq):
    """dn_component.py:155-167, the same loop (True = may not attend)."""
    m = np.zeros((pad + nq, pad + nq), bool)
    m[pad:, :pad] = True
    for i in range(groups):
        r = slice(single * 2 * i, single * 2 * (i + 1))
        if i == 0:
            m[r, single * 2 * (i + 1):pad] = True
        if i == groups - 1:
            m[r, :single * i * 2] = True
        else:
            m[r, single * 2 * (i + 1):pad] = True
            m[r, :single * 2 * i] = True
    return m


_SIZE_OF_BACKBONE = {"B0": "n", "B4": "l", "B5": "x"}


def model_size(model):
    """'n' | 'l' | 'x' from the backbone arch (configs: B0 / B4 / B5), or None."""
    return _SIZE_OF_BACKBONE.get(getattr(model.backbone, "name", None))


class Trainer:
    """The training step for a DETRPose module (reference parameter names), dtype 'bf16' or
    'fp32'. Optimizer: AdamW(lr, betas, weight_decay) + clip_grad_norm_(max_norm), the backbone's
    own learning rate, ModelEMA and the gradient accumulation of train_one_epoch: each argument
    left None takes the model size's config value (detrpose_amd.configs.training_params:
    configs/detrpose/detrpose_hgnetv2_*.py, include/detrpose_hgnetv2.py)."""

    def __init__(self, model, dtype="bf16", device="cuda", lr=None, betas=None, weight_decay=None,
                 max_norm=None, dn_number=20, label_noise_ratio=0.5, weights=(2.0, 10.0, 4.0), seed=0,
                 scope="full", backbone_lr=None, ema=True, ema_decay=None, ema_warmups=None, grad_accum_steps=None,
                 graphs=None):
        from .configs import training_params
        assert scope in ("full", "transformer"), scope
        size = model_size(model)
        cfg = training_params(size) if size else training_params("l")

        def pick(v, k):
            return cfg[k] if v is None else v

        self.model = model
        self.device = torch.device(device)
        self.scope = scope
        model.set_dtype(dtype)
        if scope == "transformer":
            self.inf = model.engine(self.device)
        self.eng = TrainEngine(model, dtype, self.device, train_backbone=scope == "full")
        self.opt = dict(lr=pick(lr, "lr"), betas=tuple(pick(betas, "betas")),
                        weight_decay=pick(weight_decay, "weight_decay"), max_norm=pick(max_norm, "max_norm"),
                        backbone_lr=pick(backbone_lr, "backbone_lr"))
        self.ema = dict(decay=pick(ema_decay, "ema_decay"), warmups=pick(ema_warmups, "ema_warmups")) if ema else None
        if ema:
            self.eng.ema_init()
        self.grad_accum_steps = int(pick(grad_accum_steps, "grad_accum_steps"))
        # tapes replayed from hipGraphs after their first (eager) run, at every world size (at
        # world > 1 the SyncBN collectives are host ops that cut the encoder's tapes into graph
        # segments: graph -> collective -> graph, train_engine.Tape)
        if graphs is None:
            graphs = os.environ.get("DETRPOSE_TRAIN_GRAPHS", "1") != "0"
        self.graphs = bool(graphs)
        self.dn_number, self.label_noise_ratio = dn_number, label_noise_ratio
        self.weights = weights
        self.seed = seed
        self.steps = 0
        self.draws = 0
        K = self.eng.K
        sig = COCO_SIGMAS if K == 17 else CROWDPOSE_SIGMAS
        self.dn_sigmas = torch.tensor(np.concatenate([[0.1], sig]).astype(np.float32), device=self.device)

    def _memory(self, images):
        """The encoder memory of images and its shapes: scope 'full' runs the backbone and encoder
        training forwards (their plans kept in self.bb / self.ep for the backward); 'transformer'
        the frozen inference plan's launches up to the memory."""
        B = images.shape[0]
        if self.scope == "full":
            bb = self.eng.backbone_plan(B, images.shape[2], images.shape[3])
            bb.set_image(images)
            shapes = [(v.H, v.W) for v in bb.outs]
            ep = self.eng.encoder_plan(B, shapes, feats=bb.outs, feats_plan=bb)
            bb.forward(pack=self._pack_due(bb))
            ep.forward(pack=self._pack_due(ep))
            self.bb, self.ep = bb, ep
            return ep.memory, shapes
        plan = self.inf.plan(B)
        if images.data_ptr() != plan.input.data_ptr():
            plan.input.copy_(images.to(torch.float32))
        if not hasattr(plan, "encoder_ops"):
            first = next(i for i, (n, _, _) in enumerate(plan.ops) if n.startswith("ts."))
            plan.encoder_ops = plan.ops[:first]
        s = C.c_void_p(torch.cuda.current_stream(self.device).cuda_stream)
        for name, fn, args in plan.encoder_ops:
            rc = fn(*args, s)
            if rc:
                _lib.check(rc, name)
        shapes = [(f.H, f.W) for f in plan.bufs["encoder"]]
        return plan.bufs["memory"], shapes

    def _draw_dn(self, plan, packed, images, pad, groups, single):
        """The step's OKS-denoising draws into the plan (dp_cdn_build) and its attention mask."""
        if not pad:
            return
        eng, lib = self.eng, self.eng.lib
        if packed.boxes is None:
            raise ValueError("targets need 'boxes' (xyxy) for the denoising queries (dn_component.py:94-95)")
        s = C.c_void_p(torch.cuda.current_stream(self.device).cuda_stream)
        h, w = images.shape[-2:]
        _lib.check(lib.dp_cdn_build(_p(packed.off), _p(packed.label), _p(packed.kps), _p(packed.area),
                                    _p(packed.boxes), _p(self.dn_sigmas), images.shape[0], pad, single, eng.K,
                                    self.label_noise_ratio, 80, float(h), float(w),
                                    (self.seed * 1000003 + self.draws) & 0xFFFFFFFFFFFF, _p(plan.dn_label),
                                    _p(plan.dn_ref), s), "dp_cdn_build")
        self.draws += 1
        if getattr(plan, "_mask_key", None) != (pad, groups, single):
            plan.mask.copy_(torch.from_numpy(dn_attn_mask(pad, groups, single, eng.nq).astype(np.uint8)))
            plan._mask_key = (pad, groups, single)

    def _pack_due(self, p):
        """Whether plan p's weight-pack tape must run: once per optimizer step (the master weights
        change only in the update), so the later grad_accum sub-batches reuse the packs."""
        if getattr(p, "_packed_at", None) == self.steps:
            return False
        p._packed_at = self.steps
        return True

    def _set_graphs(self, *plans):
        """Graph replay for the plans' tapes when self.graphs. A backbone with LearnableAffineBlocks
        (DETRPose-N's B0) keeps both its tapes eager: sync_lab writes the scalars' current values
        into conv descriptors that its forward and backward launches read by value."""
        only = os.environ.get("DETRPOSE_GRAPH_TAPES")   # debugging: a comma list of tape names to graph
        for p in plans:
            on = self.graphs and not getattr(p, "labs", None)
            kind = "bb" if p is getattr(self, "bb", None) else "ep" if p is getattr(self, "ep", None) else "tr"
            tapes = [(p.fw, kind + ".fw"), (p.bw, kind + ".bw")]
            if getattr(p, "pk", None) is not None:
                tapes.append((p.pk, kind + ".pk"))
            for t, nm in tapes:
                t.use_graph = on and (only is None or nm in only.split(","))

    def sub_step(self, images, targets, after=None):
        """Forward + criterion + backward of one sub-batch (engine.py:44-59): the gradients of
        its summed losses in eng.grad_flat (overwritten). after(part): called as each part's
        backward finishes ('transformer', 'encoder', 'backbone'; the DDP buckets). Returns (loss
        names, device losses)."""
        after = after or (lambda part: None)
        eng = self.eng
        B = images.shape[0]
        if self.scope == "full" and getattr(self, "bb", None) is not None:
            self._set_graphs(self.bb, self.ep)   # before their forwards run (the plans are cached per shape)
        memory, shapes = self._memory(images)
        packed = pack_targets(targets, eng.K, self.device)
        sizes = packed.sizes
        meta = dn_meta(sizes, self.dn_number)
        pad, groups, single = meta if meta else (0, 1, 1)
        full = self.scope == "full"
        plan = eng.plan(B, pad, shapes, memory=memory, d_memory=self.ep.d_memory if full else None)
        self.plan = plan
        self._set_graphs(plan, *((self.bb, self.ep) if full else ()))
        self._draw_dn(plan, packed, images, pad, groups, single)
        plan.forward(pack=self._pack_due(plan))
        keys, vals = plan.criterion(packed, sizes, groups, weights=self.weights)
        plan.backward()
        after("transformer")
        if full:
            self.ep.backward()
            after("encoder")
            self.bb.backward()
            after("backbone")
        return keys, vals

    def step(self, images, targets, update=True):
        """One step of train_one_epoch (src/solver/engine.py:41-89): the batch split into
        grad_accum_steps consecutive sub-batches, each with its own forward (DN draws, BatchNorm
        batch statistics), criterion (matching, num_boxes) and backward, the gradients summed;
        then DDP's gradient mean, clip_grad_norm_ + AdamW and the EMA update — skipped on the
        device when the summed losses or the gradient norm are not finite (the reference stops
        before optimizer.step on a non-finite loss, engine.py:62-66). Returns (loss names, device
        tensor of the last sub-batch's losses), like the loss_dict the reference logs."""
        eng, lib = self.eng, self.eng.lib
        B = images.shape[0]
        n = self.grad_accum_steps
        if B % n:
            raise ValueError(f"batch {B} is not divisible by grad_accum_steps {n}")
        sub = B // n
        s = C.c_void_p(torch.cuda.current_stream(self.device).cuda_stream)
        eng.step_ok_reset()
        world = torch.distributed.get_world_size() if (torch.distributed.is_available() and
                                                       torch.distributed.is_initialized()) else 1
        buckets = {p: (lo, hi) for p, lo, hi in eng.grad_buckets()}
        works = []
        if world > 1 and getattr(self, "_ddp_group", None) is None:
            # the buckets' own communicator (every rank creates it at its first step): on one
            # communicator RCCL runs collectives in issue order, and the encoder backward's SyncBN
            # reductions would queue behind the transformer bucket instead of overlapping it
            self._ddp_group = torch.distributed.new_group(list(range(world)))

        def bucket_done(first):
            # DDP's bucketed all-reduce overlapped with the backward (dist_utils.py:111-133 wraps
            # the model in DDP, whose hooks reduce each bucket as its gradients are ready): as a
            # part's backward of the LAST sub-batch finishes, its range gets the accumulated
            # sub-batch sum and its all-reduce starts (RCCL: async on the collective stream, while
            # the next part's backward runs; gloo: host-staged, in order)
            def hook(part):
                lo, hi = buckets[part]
                eng.accumulate_grads(first=first, last=True, lo=lo, hi=hi)
                works.append(all_reduce(eng.grad_flat[lo:hi], async_op=True, group=self._ddp_group))
            return hook

        for j in range(n):
            last = j == n - 1
            ddp = world > 1 and last
            keys, vals = self.sub_step(images[j * sub:(j + 1) * sub], targets[j * sub:(j + 1) * sub],
                                       after=bucket_done(j == 0) if ddp else None)
            eng.check_finite(vals)
            if not ddp:
                eng.accumulate_grads(first=j == 0, last=last)
        if world > 1:
            # the step guard over every rank's losses (4 bytes): the reference checks the
            # rank-reduced loss (engine.py:63-71), so all ranks skip or update together and the
            # replicas stay identical
            all_reduce(eng.bad)
            for w in works:
                if w is not None:
                    w.wait()
            # DDP: the mean of the ranks' gradients
            _lib.check(lib.dp_convert_rows(_p(eng.grad_flat), 0, eng.grad_flat.numel(), _p(eng.grad_flat), 0,
                                           eng.grad_flat.numel(), 1, eng.grad_flat.numel(), 1.0 / world, 0, s),
                       "grad mean")
        if update:
            eng.optimizer_step(**self.opt)
            if self.ema is not None:
                eng.ema_update(**self.ema)
        self.steps += 1
        return keys, vals


class _TransformerStep(torch.autograd.Function):
    """The TrainPlan's forward / backward as one autograd node: inputs are the transformer's
    parameters (so `loss.backward()` lands their gradients in param.grad, as the reference's
    autograd does), outputs the head tensors of every layer. The backward takes the gradients
    autograd hands the outputs, runs the recorded backward tape and returns the parameter
    gradients (copies: the engine's buffer is reused by the next step)."""

    @staticmethod
    def forward(ctx, trainer, plan, *params):
        plan.forward()
        ctx.trainer, ctx.plan = trainer, plan
        outs = [t.clone() for t in plan.logits] + [t.clone() for t in plan.kps]
        outs += [plan.pre_logits.clone(), plan.pre_out.clone(), plan.interm_logits.clone(),
                 plan.ref0[:, :, 1:].clone().flatten(-2)]
        return tuple(outs)

    @staticmethod
    def backward(ctx, *grads):
        plan, eng = ctx.plan, ctx.trainer.eng
        L = eng.L
        dsts = plan.d_logits + plan.d_kps + [plan.d_pre_logits, plan.d_pre_out, plan.d_interm_logits,
                                             plan.d_interm_kps]
        with torch.no_grad():
            for d, g in zip(dsts, grads):
                if g is None:
                    d.zero_()
                else:
                    d.copy_(g.reshape(d.shape))
        plan.backward()
        if ctx.trainer.scope == "full":
            ctx.trainer.ep.backward()
            ctx.trainer.bb.backward()
        return (None, None, *[eng.grads[n].clone() for n in eng.pnames])


def train_forward(trainer, images, targets):
    """DETRPose.forward(samples, targets) in training mode (transformer.py:1219-1387): the
    reference's output dict (final head, aux_outputs, aux_pre_outputs, aux_interm_outputs,
    dn_aux_outputs, dn_aux_pre_outputs, dn_meta), differentiable w.r.t. every trained parameter
    (scope 'full': backbone + encoder + transformer; 'transformer': the transformer's) through
    _TransformerStep. The encoder's BatchNorm running statistics are updated in the module, as
    the reference's train-mode BatchNorm does."""
    eng = trainer.eng
    model = trainer.model
    eng.load_weights()          # the module's current parameter values (the user's optimizer owns them)
    for p in eng.plans.values():
        p.refresh_constants()
    B = images.shape[0]
    K, nq, L = eng.K, eng.nq, eng.L
    memory, shapes = trainer._memory(images)
    packed = pack_targets(targets, K, trainer.device)
    meta = dn_meta(packed.sizes, trainer.dn_number)
    pad, groups, single = meta if meta else (0, 1, 1)
    full = trainer.scope == "full"
    plan = eng.plan(B, pad, shapes, memory=memory, d_memory=trainer.ep.d_memory if full else None)
    trainer._draw_dn(plan, packed, images, pad, groups, single)
    if full:
        with torch.no_grad():
            for n, b in model.named_buffers():
                if n in eng.running:
                    b.copy_(eng.running[n].to(b.device, b.dtype))
    params = [p for n, p in model.named_parameters() if n in eng.params]
    assert len(params) == len(eng.pnames)
    outs = _TransformerStep.apply(trainer, plan, *params)
    logits, kps = outs[:L], outs[L:2 * L]
    pre_lg, pre_kp, int_lg, int_kp = outs[2 * L:]
    tr = model.transformer

    def head(t_lg, t_kp, sl):
        return {"pred_logits": t_lg[:, sl], "pred_keypoints": t_kp[:, sl].flatten(-2)}

    m = slice(pad, None)
    corners = [c.detach().view(B, pad + nq, K, -1) for c in plan.corners]
    out = {**head(logits[-1], kps[-1], m), "pred_corners": corners[-1][:, m], "ref_points": plan.pre_out[:, m].detach(),
           "up": tr.up, "reg_scale": tr.reg_scale, "reg_max": tr.reg_max}
    out["aux_outputs"] = [{**head(logits[l], kps[l], m), "pred_corners": corners[l][:, m],
                           "ref_points": plan.pre_out[:, m].detach(), "teacher_corners": corners[-1][:, m],
                           "teacher_logits": logits[-1][:, m].detach()} for l in range(L - 1)]
    out["aux_interm_outputs"] = [{"pred_logits": int_lg, "pred_keypoints": int_kp}]
    out["aux_pre_outputs"] = head(pre_lg, pre_kp, m)
    if pad:
        d = slice(0, pad)
        out["dn_aux_outputs"] = [{**head(logits[l], kps[l], d), "pred_corners": corners[l][:, d],
                                  "ref_points": plan.pre_out[:, d].detach()} for l in range(L)]
        out["dn_aux_pre_outputs"] = head(pre_lg, pre_kp, d)
        out["dn_meta"] = {"pad_size": pad, "num_dn_group": groups}
    return out
