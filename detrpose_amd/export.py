"""Deployment boundary: `Model(images, orig_target_sizes) -> (scores, labels, keypoints)`.

The reference wraps the deployed model and the deploy-mode PostProcess in a small
`Model` module for ONNX/TensorRT export and for its latency benchmark
(tools/deployment/export_onnx.py:46-56, tools/benchmark/torch_benchmark.py:82-91):
`outputs = model(images); return postprocessor(outputs, orig_target_sizes)` with input
names ('images', 'orig_target_sizes') and output names ('scores', 'labels', 'keypoints')
(export_onnx.py:78-79). `DeployModel` is that module on the HIP kernels: images
(N, 3, 640, 640) float in [0, 1] and orig_target_sizes (N, 2) as [w, h] on the GPU give
scores (N, 60) f32, labels (N, 60) int64 and keypoints (N, 60, 17, 2) f32 in pixels of
the original image. Unlike the reference's deploy PostProcess (postprocesses.py:28,
batch 1 only) any N works.

`DeployModel.replay(images, orig_target_sizes)` is the same computation as one hipGraph
launch of the recorded plan with PostProcess appended (what bench.py's latency mode
times); outputs alias the plan's buffers until the next replay of that batch size (an
eager `model(images)` forward does not touch them: the plan keeps PostProcess out of its
eager launch list).
ONNX export itself is out of scope (onnx is not in this image; the kernels are the
deployment artifact), so this module carries the contract, not an exporter.
"""
from __future__ import annotations

import torch
from torch import nn

INPUT_NAMES = ("images", "orig_target_sizes")
OUTPUT_NAMES = ("scores", "labels", "keypoints")


class DeployModel(nn.Module):
    def __init__(self, model, postprocessor):
        super().__init__()
        self.model = model.deploy()
        self.postprocessor = postprocessor.deploy()
        self._graphs = {}

    @torch.no_grad()
    def forward(self, images, orig_target_sizes):
        outputs = self.model(images)
        return self.postprocessor(outputs, orig_target_sizes)

    @torch.no_grad()
    def replay(self, images, orig_target_sizes):
        """One hipGraph launch: copy the batch in, forward + PostProcess, return the plan's
        (scores, labels, keypoints) buffers (valid until the next replay at this N)."""
        if not images.is_cuda:
            raise RuntimeError("DeployModel runs on the GPU only")
        hw = tuple(self.model.encoder.eval_spatial_size)
        if tuple(images.shape[1:]) != (3, *hw):
            raise ValueError(f"expected images (N, 3, {hw[0]}, {hw[1]}), got {tuple(images.shape)}")
        n = images.shape[0]
        eng = self.model.engine(images.device)
        ns = self.postprocessor.num_select
        key = (n, eng.device, ns)
        entry = self._graphs.get(key)
        if entry is None or entry[0] is not eng or entry[1].post is not entry[2]:
            plan = eng.plan(n)
            post = plan.add_postprocess(ns)     # rebuilt (and the graph recaptured) when num_select changed
            entry = (eng, plan, post, plan.graph())
            self._graphs[key] = entry
        _, plan, post, g = entry
        with torch.cuda.device(images.device):
            plan.input.copy_(images.to(torch.float32), non_blocking=True)
            post["target_sizes"].copy_(orig_target_sizes.to(torch.float32).reshape(n, 2), non_blocking=True)
            g.replay()
        return post["scores"], post["labels"], post["keypoints"]
