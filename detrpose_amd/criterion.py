"""Training criterion on the HIP kernels: `HungarianMatcher` and `Criterion`
with the reference's constructors, call signatures and loss-dict keys
(/root/reference/src/models/detrpose/matcher.py:21-112, criterion.py:10-435).

What differs is where the work runs. The reference builds each cost matrix with torch ops,
copies it to the host (one device->host sync per matched head, matcher.py:88/93) and runs
scipy's `linear_sum_assignment`; here one launch matches every head of the step on the GPU
(`dp_hungarian_match`: cost block in LDS + scipy's shortest augmenting path in f64, one wave
per (head, image)), one launch forms the union matching (`dp_match_union`), and one launch
computes vfl + keypoint L1 + OKS losses of every head together with their gradients
(`dp_pose_loss`). `num_boxes` / `num_boxes_go` stay device scalars (all-reduced over RCCL when
torch.distributed is initialised, criterion.py:306-323), so a criterion call never
synchronises with the host.

Scope: the losses of the shipped configs, `['vfl', 'keypoints']` with weight_dict
{loss_vfl, loss_keypoints, loss_oks} (configs/detrpose/include/detrpose_hgnetv2.py), for the
matched heads and the denoising heads (dn_aux_outputs / dn_aux_pre_outputs with their fixed
positive matching, criterion.py:385-435). The 'labels', 'mal', 'local' and 'matching' losses
raise NotImplementedError. There is no CPU path.

Two deliberate departures from matcher.py: (1) the reference drops the keypoint costs of a head
whose keypoints sum to <= 0 (matcher.py:70-93) and matches on the class cost alone; keypoints
come out of a sigmoid or of the refinement around sigmoid anchors, so that branch never runs
and the keypoint costs are always added here. (2) NaN / inf costs make scipy raise; here the
image's queries get match -2 and dp_pose_loss returns a NaN loss_vfl for the head, so a
diverged step shows in the loss instead of silently training on a partial matching.
"""
from __future__ import annotations

import ctypes as C
from dataclasses import dataclass

import numpy as np
import torch
from torch import nn

from . import _lib

COCO_SIGMAS = np.array([.26, .25, .25, .35, .35, .79, .79, .72, .72, .62, .62, 1.07, 1.07, .87, .87, .89, .89],
                       dtype=np.float32) / 10.0
CROWDPOSE_SIGMAS = np.array([.79, .79, .72, .72, .62, .62, 1.07, 1.07, .87, .87, .89, .89, .79, .79],
                            dtype=np.float32) / 10.0


def keypoint_sigmas(num_body_points: int) -> np.ndarray:
    """matcher.py:32-44 / keypoint_loss.py:48-60."""
    if num_body_points == 17:
        return COCO_SIGMAS
    if num_body_points == 14:
        return CROWDPOSE_SIGMAS
    raise NotImplementedError(f"{num_body_points} body points (17 or 14)")


def _stream(dev):
    return C.c_void_p(torch.cuda.current_stream(dev).cuda_stream)


@dataclass
class PackedTargets:
    """The targets of one batch packed for the kernels (sizes are host ints: no sync)."""
    off: torch.Tensor      # (B+1,) int32 prefix offsets
    label: torch.Tensor    # (T,) int32
    kps: torch.Tensor      # (T, 3K) f32: K (x, y) pairs, then K visibilities
    area: torch.Tensor     # (T,) f32
    sizes: list
    max_t: int
    boxes: torch.Tensor = None   # (T, 4) f32 xyxy (the DN queries' centre points) when given


def to_device_async(x: torch.Tensor, device, dtype=None) -> torch.Tensor:
    """x on `device` (as dtype) without a host synchronisation: a host tensor goes through pinned
    memory with a non-blocking copy (a pageable host -> GPU copy synchronises the stream, which made
    the training step's host wait for the forward already queued before the targets were packed)."""
    if dtype is not None and x.dtype != dtype:
        x = x.to(dtype)
    device = torch.device(device)
    if x.device == device or device.type != "cuda" or x.device.type != "cpu":
        return x.to(device)
    return x.contiguous().pin_memory().to(device, non_blocking=True)


def pack_targets(targets, num_body_points: int, device) -> PackedTargets:
    sizes = [int(t["labels"].shape[0]) for t in targets]
    off = to_device_async(torch.from_numpy(np.concatenate([[0], np.cumsum(sizes)]).astype(np.int32)), device)
    K3 = 3 * num_body_points
    if sum(sizes):
        label = to_device_async(torch.cat([t["labels"].reshape(-1) for t in targets]), device, torch.int32)
        kps = to_device_async(torch.cat([t["keypoints"].reshape(-1, K3) for t in targets]), device, torch.float32)
        area = to_device_async(torch.cat([t["area"].reshape(-1) for t in targets]), device, torch.float32)
        boxes = (to_device_async(torch.cat([t["boxes"].reshape(-1, 4) for t in targets]), device, torch.float32)
                 if all("boxes" in t for t in targets) else None)
    else:
        label = torch.zeros(1, dtype=torch.int32, device=device)
        kps = torch.zeros(1, K3, dtype=torch.float32, device=device)
        area = torch.ones(1, dtype=torch.float32, device=device)
        boxes = torch.zeros(1, 4, dtype=torch.float32, device=device)
    return PackedTargets(off, label.contiguous(), kps.contiguous(), area.contiguous(), sizes, max(sizes or [0]),
                         boxes.contiguous() if boxes is not None else None)


def _f32_rows(x: torch.Tensor, last: int) -> torch.Tensor:
    """(B, Q, last) f32 view with unit stride in the last dim; a non-DN pre head's keypoints
    come as (B, Q, K, 2) (transformer.py:1373) and are flattened here."""
    if x.dim() == 4:
        x = x.flatten(-2)
    if x.dim() != 3 or x.shape[-1] != last:
        raise ValueError(f"expected (B, Q, {last}), got {tuple(x.shape)}")
    if not x.is_cuda:
        raise RuntimeError("criterion: outputs must be on the GPU (no CPU path)")
    x = x.float()
    return x if x.stride(-1) == 1 else x.contiguous()


def match_heads(logits, kps, packed: PackedTargets, num_body_points: int, cost_class: float, cost_keypoints: float,
                cost_oks: float, focal_alpha: float, cost_out: bool = False):
    """Match H heads at once. logits / kps: lists of (B, Q, ncls) / (B, Q, 2K) GPU tensors.
    Returns match (H, B, Q) int32 (image-local target index or -1) [, cost (H, B, Q, max_t)]."""
    H = len(logits)
    lg = torch.stack([_f32_rows(x, x.shape[-1]) for x in logits])
    kp = torch.stack([_f32_rows(x, 2 * num_body_points) for x in kps])
    _, B, Q, ncls = lg.shape
    dev = lg.device
    if packed.off.device != dev:
        raise RuntimeError(f"targets on {packed.off.device}, outputs on {dev}")
    if len(packed.sizes) != B:
        raise ValueError(f"{len(packed.sizes)} targets for a batch of {B}")
    sig = torch.tensor(keypoint_sigmas(num_body_points), device=dev)
    match = torch.empty(H, B, Q, dtype=torch.int32, device=dev)
    cost = torch.full((H, B, Q, max(packed.max_t, 1)), float("nan"), device=dev) if cost_out else None
    lib = _lib.load()
    _lib.check(lib.dp_hungarian_match(lg.data_ptr(), lg.stride(0), lg.stride(1), lg.stride(2), ncls, kp.data_ptr(),
                                      kp.stride(0), kp.stride(1), kp.stride(2), num_body_points, packed.off.data_ptr(),
                                      packed.label.data_ptr(), packed.kps.data_ptr(), packed.area.data_ptr(), H, B, Q,
                                      packed.max_t, float(cost_class), float(cost_keypoints), float(cost_oks),
                                      float(focal_alpha), sig.data_ptr(), match.data_ptr(),
                                      cost.data_ptr() if cost is not None else None, _stream(dev)),
               "dp_hungarian_match")
    return (match, cost) if cost_out else match


def match_to_indices(match_bq: torch.Tensor):
    """(B, Q) match -> the reference's [(query_idx, target_idx)] int64 list (host; syncs)."""
    m = match_bq.cpu().numpy()
    out = []
    for row in m:
        q = np.nonzero(row >= 0)[0]
        out.append((torch.as_tensor(q, dtype=torch.int64), torch.as_tensor(row[q], dtype=torch.int64)))
    return out


class HungarianMatcher(nn.Module):
    """matcher.py:21-112. `forward` returns the reference's list of (index_i, index_j) int64
    tensors per image (a host copy of the GPU matching); `match` keeps it on the device."""

    def __init__(self, cost_class: float = 1, focal_alpha=0.25, cost_keypoints=1.0, cost_oks=0.01,
                 num_body_points=17):
        super().__init__()
        self.cost_class = cost_class
        self.cost_keypoints = cost_keypoints
        self.cost_oks = cost_oks
        self.focal_alpha = focal_alpha
        self.num_body_points = num_body_points
        self.sigmas = keypoint_sigmas(num_body_points)

    def match(self, logits, kps, packed: PackedTargets, cost_out: bool = False):
        return match_heads(logits, kps, packed, self.num_body_points, self.cost_class, self.cost_keypoints,
                           self.cost_oks, self.focal_alpha, cost_out)

    @torch.no_grad()
    def forward(self, outputs, targets):
        lg = outputs["pred_logits"]
        packed = pack_targets(targets, self.num_body_points, lg.device)
        m = self.match([lg], [outputs["pred_keypoints"]], packed)
        return match_to_indices(m[0])


class _PoseLoss(torch.autograd.Function):
    """Losses (H, 3) of H heads; backward scales the kernel's per-loss gradients."""

    @staticmethod
    def forward(ctx, run, *tensors):
        losses, g_lg, g_l1, g_oks = run()
        ctx.save_for_backward(g_lg, g_l1, g_oks)
        ctx.H = len(tensors) // 2
        ctx.meta = [(t.shape, t.dtype) for t in tensors]
        return losses

    @staticmethod
    def backward(ctx, grad):
        g_lg, g_l1, g_oks = ctx.saved_tensors
        H = ctx.H
        d_lg = (grad[:, 0].view(H, 1, 1, 1) * g_lg).unbind(0)
        d_kp = (grad[:, 1].view(H, 1, 1, 1) * g_l1 + grad[:, 2].view(H, 1, 1, 1) * g_oks).unbind(0)
        grads = [d.reshape(s).to(dt) for d, (s, dt) in zip(d_lg + d_kp, ctx.meta)]
        return (None, *grads)


class Criterion(nn.Module):
    """criterion.py:10-435 for the losses ['vfl', 'keypoints'] (the shipped configs)."""

    SUPPORTED = ("vfl", "keypoints")

    def __init__(self, num_classes, matcher, weight_dict, losses, num_body_points, focal_alpha=0.25, mal_alpha=None,
                 gamma=2.0):
        super().__init__()
        bad = [l for l in losses if l not in self.SUPPORTED]
        if bad:
            raise NotImplementedError(f"losses {bad}: only {list(self.SUPPORTED)} (the shipped configs) are built")
        self.num_classes = num_classes
        self.matcher = matcher
        self.weight_dict = weight_dict
        self.losses = losses
        self.focal_alpha = focal_alpha
        self.mal_alpha = mal_alpha
        self.gamma = gamma
        self.num_body_points = num_body_points
        self.sigmas = keypoint_sigmas(num_body_points)
        self.last_match = None   # (match (H, B, Q), go (B, Q), head names) of the last call, for inspection

    def forward(self, outputs, targets):
        assert "aux_outputs" in outputs, ""   # criterion.py:313-314
        # heads in the reference's matching order (criterion.py:290-303)
        names = ["", *[f"_{i}" for i in range(len(outputs["aux_outputs"]))], "_pre",
                 *[f"_enc_{i}" for i in range(len(outputs["aux_interm_outputs"]))]]
        heads = [outputs, *outputs["aux_outputs"], outputs["aux_pre_outputs"], *outputs["aux_interm_outputs"]]
        K2 = 2 * self.num_body_points
        logits = [_f32_rows(h["pred_logits"], outputs["pred_logits"].shape[-1]) for h in heads]
        kps = [_f32_rows(h["pred_keypoints"], K2) for h in heads]
        H = len(heads)
        if H > 16:
            raise ValueError(f"{H} heads (at most 16)")
        B, Q, ncls = logits[0].shape
        dev = logits[0].device
        packed = pack_targets(targets, self.num_body_points, dev)
        m = self.matcher
        match = match_heads(logits, kps, packed, self.num_body_points, m.cost_class, m.cost_keypoints, m.cost_oks,
                            m.focal_alpha)
        lib = _lib.load()
        go = torch.empty(B, Q, dtype=torch.int32, device=dev)
        n_go = torch.empty(1, dtype=torch.float32, device=dev)
        _lib.check(lib.dp_match_union(match.data_ptr(), H, B, Q, go.data_ptr(), n_go.data_ptr(), _stream(dev)),
                   "dp_match_union")
        n_boxes = torch.full((1,), float(sum(packed.sizes)), dtype=torch.float32, device=dev)
        world = 1
        if torch.distributed.is_available() and torch.distributed.is_initialized():
            torch.distributed.all_reduce(n_boxes)
            torch.distributed.all_reduce(n_go)
            world = torch.distributed.get_world_size()
        self.last_match = (match, go, names)
        wd = self.weight_dict
        w_vfl, w_kp, w_oks = (float(wd.get(k, 1.0)) for k in ("loss_vfl", "loss_keypoints", "loss_oks"))
        sig = torch.tensor(self.sigmas, device=dev)

        def run():
            losses = torch.empty(H, 3, dtype=torch.float32, device=dev)
            g_lg = torch.empty(H, B, Q, ncls, dtype=torch.float32, device=dev)
            g_l1 = torch.empty(H, B, Q, K2, dtype=torch.float32, device=dev)
            g_oks = torch.empty(H, B, Q, K2, dtype=torch.float32, device=dev)
            hs = (_lib.LossHead * H)()
            for i in range(H):
                hs[i] = _lib.LossHead(logits[i].data_ptr(), logits[i].stride(0), logits[i].stride(1), kps[i].data_ptr(),
                                      kps[i].stride(0), kps[i].stride(1), match[i].data_ptr())
            _lib.check(lib.dp_pose_loss(hs, H, B, Q, ncls, self.num_body_points, go.data_ptr(), packed.off.data_ptr(),
                                        packed.label.data_ptr(), packed.kps.data_ptr(), packed.area.data_ptr(),
                                        sig.data_ptr(), float(self.focal_alpha), float(self.gamma),
                                        n_boxes.data_ptr(), n_go.data_ptr(), float(world), w_vfl, w_kp, w_oks,
                                        losses.data_ptr(), g_lg.data_ptr(), g_l1.data_ptr(), g_oks.data_ptr(),
                                        _stream(dev)), "dp_pose_loss")
            return losses, g_lg, g_l1, g_oks

        # the autograd inputs are the callers' tensors (logits/kps above may be f32 copies)
        src = [h["pred_logits"] for h in heads] + [h["pred_keypoints"] for h in heads]
        L = _PoseLoss.apply(run, *src)
        out = {}
        self._put(out, names, L)
        if "dn_aux_outputs" in outputs:
            self._dn_losses(outputs, packed, n_boxes, world, sig, dev, out)
        return dict(sorted(out.items()))

    def _put(self, out, names, L):
        wd = self.weight_dict
        for i, n in enumerate(names):
            if "vfl" in self.losses and "loss_vfl" in wd:
                out["loss_vfl" + n] = L[i, 0]
            if "keypoints" in self.losses:
                if "loss_keypoints" in wd:
                    out["loss_keypoints" + n] = L[i, 1]
                if "loss_oks" in wd:
                    out["loss_oks" + n] = L[i, 2]

    def _dn_losses(self, outputs, packed, n_boxes, world, sig, dev, out):
        """criterion.py:385-435: vfl + keypoints of every DN head with the fixed positive
        matching (DN slot g * single_pad + t <-> target t), normalised by num_boxes * groups."""
        from .train_engine import dn_match
        meta = outputs["dn_meta"]
        pad, groups = int(meta["pad_size"]), int(meta["num_dn_group"])
        heads = [*outputs["dn_aux_outputs"], outputs["dn_aux_pre_outputs"]]
        names = [*[f"_dn_{i}" for i in range(len(outputs["dn_aux_outputs"]))], "_dn_pre"]
        K2 = 2 * self.num_body_points
        logits = [_f32_rows(h["pred_logits"], outputs["pred_logits"].shape[-1]) for h in heads]
        kps = [_f32_rows(h["pred_keypoints"], K2) for h in heads]
        H = len(heads)
        B, Q, ncls = logits[0].shape
        assert Q == pad, (Q, pad)
        m = torch.from_numpy(dn_match(packed.sizes, pad, groups)).to(dev)
        # num_boxes (all-reduced, / world, >= 1) * groups; dp_pose_loss divides by world again
        n_dn = torch.clamp(n_boxes / world, min=1.0) * groups * world
        lib = _lib.load()
        wd = self.weight_dict
        w_vfl, w_kp, w_oks = (float(wd.get(k, 1.0)) for k in ("loss_vfl", "loss_keypoints", "loss_oks"))

        def run():
            losses = torch.empty(H, 3, dtype=torch.float32, device=dev)
            g_lg = torch.empty(H, B, Q, ncls, dtype=torch.float32, device=dev)
            g_l1 = torch.empty(H, B, Q, K2, dtype=torch.float32, device=dev)
            g_oks = torch.empty(H, B, Q, K2, dtype=torch.float32, device=dev)
            hs = (_lib.LossHead * H)()
            for i in range(H):
                hs[i] = _lib.LossHead(logits[i].data_ptr(), logits[i].stride(0), logits[i].stride(1), kps[i].data_ptr(),
                                      kps[i].stride(0), kps[i].stride(1), m.data_ptr())
            _lib.check(lib.dp_pose_loss(hs, H, B, Q, ncls, self.num_body_points, m.data_ptr(), packed.off.data_ptr(),
                                        packed.label.data_ptr(), packed.kps.data_ptr(), packed.area.data_ptr(),
                                        sig.data_ptr(), float(self.focal_alpha), float(self.gamma), n_dn.data_ptr(),
                                        n_dn.data_ptr(), float(world), w_vfl, w_kp, w_oks, losses.data_ptr(),
                                        g_lg.data_ptr(), g_l1.data_ptr(), g_oks.data_ptr(), _stream(dev)),
                       "dp_pose_loss(dn)")
            return losses, g_lg, g_l1, g_oks

        src = [h["pred_logits"] for h in heads] + [h["pred_keypoints"] for h in heads]
        self._put(out, names, _PoseLoss.apply(run, *src))
