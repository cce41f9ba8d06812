"""PostProcess: the drop-in for src/models/detrpose/postprocesses.py.

Deploy mode (postprocesses.py:15-30) returns (scores, labels, keypoints) — here for
any batch size (the reference's deploy branch hard-codes batch 1, line 28); the
non-deploy mode returns the per-image dicts with the visibility column appended
(32-40). Both run the dp_postprocess HIP kernel (sigmoid, top-k over query x class,
keypoint gather, scale by [w, h]).
"""
from __future__ import annotations

import ctypes as C

import torch
from torch import nn

from . import _lib


class PostProcess(nn.Module):
    def __init__(self, num_select=60, num_body_points=17):
        super().__init__()
        self.num_select = num_select
        self.num_body_points = num_body_points
        self.deploy_mode = False

    def deploy(self):
        self.eval()
        self.deploy_mode = True
        return self

    @torch.no_grad()
    def forward(self, outputs, target_sizes):
        logits = outputs["pred_logits"].float().contiguous()
        kps = outputs["pred_keypoints"].float()
        B, Q, NC = logits.shape
        K = self.num_body_points
        kps = kps.reshape(B, Q, K, 2).contiguous()
        if not logits.is_cuda:
            raise RuntimeError("PostProcess (MI355X) runs on the GPU only")
        ts = target_sizes.to(logits.device, torch.float32).reshape(B, 2).contiguous()
        n = self.num_select
        scores = torch.empty(B, n, device=logits.device)
        labels = torch.empty(B, n, dtype=torch.int64, device=logits.device)
        out = torch.empty(B, n, K, 2, device=logits.device)
        lib = _lib.load()
        rc = lib.dp_postprocess(logits.data_ptr(), kps.data_ptr(), ts.data_ptr(), B, Q, NC, K, n, scores.data_ptr(),
                                labels.data_ptr(), out.data_ptr(),
                                C.c_void_p(torch.cuda.current_stream(logits.device).cuda_stream))
        _lib.check(rc, "dp_postprocess")
        if self.deploy_mode:
            return scores, labels, out
        kp = torch.cat([out, torch.ones_like(out[..., :1])], -1).flatten(-2)
        return [{"scores": s, "labels": l, "keypoints": k} for s, l, k in zip(scores, labels, kp)]
