"""TEST INFRASTRUCTURE ONLY (never imported by the product path).

CPU restatement of the reference's training criterion for the shipped loss set
['vfl', 'keypoints']: HungarianMatcher (src/models/detrpose/matcher.py:47-112), the union
matching Criterion._get_go_indices (criterion.py:247-268, with a stable order among tied
counts: tests/golden/make_train_golden.py explains why), loss_vfl (criterion.py:58-93),
loss_keypoints + loss_oks (criterion.py:200-229, OKS of src/misc/keypoint_loss.py:5-34) and
Criterion.forward's head loop / key naming / normalisers (criterion.py:285-383).
Pinned to the reference's own outputs by tests/golden/criterion_*.npz (tests/test_criterion.py).
Torch CPU ops so that autograd gives the reference gradients.
"""
from __future__ import annotations

import numpy as np
import torch
import torch.nn.functional as F

from oracle.lsap_cpu import lsap

SIGMAS = {17: np.array([.26, .25, .25, .35, .35, .79, .79, .72, .72, .62, .62, 1.07, 1.07, .87, .87, .89, .89],
                       dtype=np.float32) / 10.0,
          14: np.array([.79, .79, .72, .72, .62, .62, 1.07, 1.07, .87, .87, .89, .89, .79, .79],
                       dtype=np.float32) / 10.0}


def match_cost(logits, kps, tgt_labels, tgt_kps, tgt_area, K, cost_class=2.0, cost_kp=10.0, cost_oks=4.0,
               alpha=0.25):
    """matcher.py:51-87 for one image: (Q, ncls), (Q, 2K) vs its T targets -> C (Q, T)."""
    p = logits.sigmoid()
    neg = (1 - alpha) * (p ** 2.0) * (-(1 - p + 1e-8).log())
    pos = alpha * ((1 - p) ** 2.0) * (-(p + 1e-8).log())
    cc = pos[:, tgt_labels] - neg[:, tgt_labels]
    zp, zg, vg = kps[:, :2 * K], tgt_kps[:, :2 * K], tgt_kps[:, 2 * K:]
    var = (torch.from_numpy(SIGMAS[K]) * 2) ** 2
    kp_p, kp_g = zp.reshape(-1, K, 2), zg.reshape(-1, K, 2)
    d2 = (kp_p[:, None, :, 0] - kp_g[None, :, :, 0]) ** 2 + (kp_p[:, None, :, 1] - kp_g[None, :, :, 1]) ** 2
    d0 = d2 / (tgt_area[:, None] * var[None, :] * 2)
    oks = (torch.exp(-d0) * vg).sum(-1) / (vg.sum(-1) + 1e-6)
    oks = oks.clamp(min=1e-6)
    l1 = (torch.abs(zp[:, None, :] - zg[None]) * vg.repeat_interleave(2, dim=1)[None]).sum(-1)
    return cost_class * cc + cost_kp * l1 + cost_oks * (1 - oks)


def match(logits, kps, sizes, tgt_labels, tgt_kps, tgt_area, K, **costs):
    """One head: (B, Q, ncls), (B, Q, 2K) -> match (B, Q) int64 (target index or -1)."""
    B, Q, _ = logits.shape
    out = np.full((B, Q), -1, np.int64)
    off = np.concatenate([[0], np.cumsum(sizes)])
    with torch.no_grad():
        for b in range(B):
            t0, t1 = off[b], off[b + 1]
            if t1 == t0:
                continue
            C = match_cost(logits[b], kps[b], tgt_labels[t0:t1], tgt_kps[t0:t1], tgt_area[t0:t1], K, **costs)
            I, J = lsap(C.numpy())
            out[b, I] = J
    return out


def union(matches):
    """_get_go_indices: matches (H, B, Q) -> go (B, Q): per query the target most heads chose,
    ties to the smaller target index."""
    H, B, Q = matches.shape
    go = np.full((B, Q), -1, np.int64)
    for b in range(B):
        for q in range(Q):
            ts = [int(t) for t in matches[:, b, q] if t >= 0]
            if ts:
                cnt = {t: ts.count(t) for t in ts}
                go[b, q] = min(cnt, key=lambda t: (-cnt[t], t))
    return go


def oks(zp, zg, vg, area, K):
    """keypoint_loss.py:5-34 (linear, eps 1e-6): per pair."""
    var = (torch.from_numpy(SIGMAS[K]) * 2) ** 2
    p, g = zp.reshape(-1, K, 2), zg.reshape(-1, K, 2)
    d2 = (p[:, :, 0] - g[:, :, 0]) ** 2 + (p[:, :, 1] - g[:, :, 1]) ** 2
    d0 = d2 / (area[:, None] * var[None, :] * 2)
    o = (torch.exp(-d0) * vg).sum(1) / (vg.sum(1) + 1e-6)
    return o.clamp(min=1e-6)


def _pairs(m):
    b, q = np.nonzero(m >= 0)
    return torch.as_tensor(b), torch.as_tensor(q), m[b, q]


def loss_vfl(logits, kps, m, sizes, tgt_labels, tgt_kps, tgt_area, K, num_boxes, ncls, alpha=0.25, gamma=2.0):
    off = np.concatenate([[0], np.cumsum(sizes)])
    b, q, t = _pairs(m)
    tg = torch.as_tensor(off[b.numpy()] + t)
    zp = kps[b, q][:, :2 * K]
    o = oks(zp, tgt_kps[tg, :2 * K], tgt_kps[tg, 2 * K:], tgt_area[tg], K).detach()
    tc = torch.full(logits.shape[:2], ncls, dtype=torch.int64)
    tc[b, q] = tgt_labels[tg]
    target = F.one_hot(tc, num_classes=ncls + 1)[..., :-1]
    ts_o = torch.zeros(logits.shape[:2], dtype=logits.dtype)
    ts_o[b, q] = o
    ts = ts_o.unsqueeze(-1) * target
    ps = logits.sigmoid().detach()
    w = alpha * ps.pow(gamma) * (1 - target) + ts
    loss = F.binary_cross_entropy_with_logits(logits, ts, weight=w, reduction="none")
    return loss.mean(1).sum() * logits.shape[1] / num_boxes


def loss_keypoints(kps, go, sizes, tgt_kps, tgt_area, K, num_boxes_go):
    off = np.concatenate([[0], np.cumsum(sizes)])
    b, q, t = _pairs(go)
    if len(b) == 0:
        z = kps.sum() * 0
        return z, z
    tg = torch.as_tensor(off[b.numpy()] + t)
    zp = kps[b, q][:, :2 * K]
    zg, vg = tgt_kps[tg, :2 * K], tgt_kps[tg, 2 * K:]
    oks_loss = 1 - oks(zp, zg, vg, tgt_area[tg], K)
    pose = F.l1_loss(zp, zg, reduction="none") * vg.repeat_interleave(2, dim=1)
    return pose.sum() / num_boxes_go, oks_loss.sum() / num_boxes_go


def criterion(heads, sizes, tgt_labels, tgt_kps, tgt_area, K, ncls, n_aux, weights=(2.0, 10.0, 4.0),
              force_match=None):
    """heads: [(logits, kps)] in the reference's order (final, aux 0..n_aux-1, pre, interm).
    force_match: (H, B, Q) matchings to use instead of the matcher's (a run whose near-tied costs
    another summation order resolves differently is compared on the same assignment).
    Returns (loss dict, matches (H, B, Q), go (B, Q))."""
    if force_match is not None:
        matches = np.asarray(force_match, np.int64)
    else:
        matches = np.stack([match(lg.detach(), kp.detach(), sizes, tgt_labels, tgt_kps, tgt_area, K)
                            for lg, kp in heads])
    go = union(matches)
    num_boxes = max(float(sum(sizes)), 1.0)
    num_go = max(float((go >= 0).sum()), 1.0)
    names = ["", *[f"_{i}" for i in range(n_aux)], "_pre", "_enc_0"]
    out = {}
    for (lg, kp), m, n in zip(heads, matches, names):
        out["loss_vfl" + n] = weights[0] * loss_vfl(lg, kp, m, sizes, tgt_labels, tgt_kps, tgt_area, K, num_boxes, ncls)
        l1, lo = loss_keypoints(kp, go, sizes, tgt_kps, tgt_area, K, num_go)
        out["loss_keypoints" + n] = weights[1] * l1
        out["loss_oks" + n] = weights[2] * lo
    return dict(sorted(out.items())), matches, go
