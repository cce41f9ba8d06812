"""DETRPose top level: the drop-in for src/models/detrpose/detrpose.py.

`DETRPose(backbone, encoder, transformer)` keeps the reference constructor and
state_dict layout (detrpose.py:15-67), `.deploy()` returns self (69-74) and
`forward(samples, targets=None) -> {'pred_logits', 'pred_keypoints'}` (76-81). As in
the reference, the keypoint layout depends on deploy mode: (B,Q,34) before `.deploy()`
(transformer.py:1320-1321 flattens the last two dims) and (B,Q,17,2) after it
(convert_to_deploy, transformer.py:1202-1207); logits are (B,Q,2) either way. In eval
`targets` is accepted and ignored, as the reference's evaluate() passes them
(src/solver/engine.py:133-134) and only the training forward reads them
(transformer.py:1265). The forward runs entirely on the HIP kernels of
libdetrpose_hip.so through detrpose_amd.engine; there is no eager-torch or CPU fallback.

`build_model(size)` is the constructor the north star names ("build_model"); the
reference has no such function (only LazyConfig + instantiate), so it reads the
N/L/X kwargs from detrpose_amd.configs.
"""
from __future__ import annotations

import torch
from torch import nn

from .configs import get_config
from .hgnetv2 import HGNetv2
from .hybrid_encoder import HybridEncoder
from .postprocesses import PostProcess
from .transformer import Transformer


class DETRPose(nn.Module):
    def __init__(self, backbone, encoder, transformer, is_trainable=True, trainable_energy=False, dtype="bf16"):
        super().__init__()
        self.backbone = backbone
        self.encoder = encoder
        self.transformer = transformer
        self.layer_loss = torch.zeros(1, dtype=torch.float32)
        self.compute_dtype = dtype
        self.deploy_mode = False
        self._engine = None

    # -- reference API
    def deploy(self):
        """detrpose.py:69-74: eval + convert_to_deploy (BN folding happens in the engine's
        packer for every mode; what deploy changes visibly is the (B,Q,17,2) layout)."""
        self.eval()
        self.deploy_mode = True
        return self

    def set_dtype(self, dtype: str):
        """'bf16' (default; bf16 storage, f32 accumulation) or 'fp32' (parity mode)."""
        if dtype != self.compute_dtype:
            self.compute_dtype = dtype
            self._engine = None
        return self

    def engine(self, device="cuda"):
        from .engine import Engine
        dev = torch.device(device)
        if dev.type == "cuda" and dev.index is None:
            dev = torch.device("cuda", torch.cuda.current_device())
        if self._engine is None or self._engine.device != dev:
            self._engine = Engine(self, self.compute_dtype, dev)
        return self._engine

    def _load_from_state_dict(self, *args, **kw):
        self._engine = None  # weights changed: repack on next forward
        super()._load_from_state_dict(*args, **kw)

    def forward(self, samples, targets=None):
        if self.training:
            return self._forward_train(samples, targets)
        with torch.no_grad():
            return self._forward_eval(samples)

    def _forward_eval(self, samples):
        if not samples.is_cuda:
            raise RuntimeError("DETRPose (MI355X) runs on the GPU only: move the images to a HIP device")
        hw = tuple(self.encoder.eval_spatial_size)
        if samples.dim() != 4 or tuple(samples.shape[1:]) != (3, *hw):
            raise ValueError(f"DETRPose expects images (B, 3, {hw[0]}, {hw[1]}) (the plan is built for "
                             f"eval_spatial_size {list(hw)}), got {tuple(samples.shape)}")
        eng = self.engine(samples.device)
        B = samples.shape[0]
        plan = eng.plan(B)
        with torch.cuda.device(samples.device):
            if samples.data_ptr() != plan.input.data_ptr():
                plan.input.copy_(samples.to(torch.float32), non_blocking=True)
            plan.run()
            out = {k: v.clone() for k, v in plan.outputs.items()}
        if not self.deploy_mode:
            out["pred_keypoints"] = out["pred_keypoints"].flatten(-2)
        return out

    def _check_input(self, samples):
        if not samples.is_cuda:
            raise RuntimeError("DETRPose (MI355X) runs on the GPU only: move the images to a HIP device")
        hw = tuple(self.encoder.eval_spatial_size)
        if samples.dim() != 4 or tuple(samples.shape[1:]) != (3, *hw):
            raise ValueError(f"DETRPose expects images (B, 3, {hw[0]}, {hw[1]}), got {tuple(samples.shape)}")

    def _forward_train(self, samples, targets):
        """The training-mode forward (transformer.py:1219-1387).

        With targets: the full training forward with OKS-denoising queries through the HIP
        training step (detrpose_amd.train.train_forward): the reference's output dict incl.
        dn_aux_outputs / dn_aux_pre_outputs / dn_meta, differentiable w.r.t. every parameter of
        the network (the backbone with FrozenBatchNorm2d, the encoder with its BatchNorm2d on
        batch statistics: SyncBatchNorm across ranks under torch.distributed), so
        `criterion(outputs, targets)` then `loss.backward()` fills every .grad
        (src/solver/engine.py:34-60). With the encoder's BatchNorm layers put in eval mode the
        backbone and encoder run frozen instead and only the transformer is trained.

        Without targets: every decoder layer's logits / keypoints / corners (aux_outputs), the
        first layer's pre head and the two-stage selection, values only (the reference's own
        non-DN training forward stops at transformer.py:1353); BatchNorm in eval mode."""
        bn = [n for n, m in self.named_modules() if isinstance(m, nn.modules.batchnorm._BatchNorm) and m.training]
        self._check_input(samples)
        if targets is not None:
            return self._forward_train_dn(samples, targets, "full" if bn else "transformer")
        if bn:
            raise NotImplementedError(f"the training forward without targets runs with BatchNorm in eval mode "
                                      f"({len(bn)} in train mode, e.g. {bn[0]})")
        eng = self.engine(samples.device)
        plan = eng.plan(samples.shape[0], aux=True)
        with torch.cuda.device(samples.device):
            if samples.data_ptr() != plan.input.data_ptr():
                plan.input.copy_(samples.to(torch.float32), non_blocking=True)
            plan.run()
            ao = plan.aux_outputs
            logits = [t.clone() for t in ao["logits"]]
            poses = [t.clone().flatten(-2) for t in ao["keypoints"]]
            corners = [t.clone() for t in ao["corners"]]
            refs = ao["ref_init"].clone()
            tr = self.transformer
            out = {"pred_logits": logits[-1], "pred_keypoints": poses[-1], "pred_corners": corners[-1],
                   "ref_points": refs, "up": tr.up, "reg_scale": tr.reg_scale, "reg_max": tr.reg_max}
            out["aux_outputs"] = [{"pred_logits": logits[l], "pred_keypoints": poses[l], "pred_corners": corners[l],
                                   "ref_points": refs, "teacher_corners": corners[-1], "teacher_logits": logits[-1]}
                                  for l in range(len(logits) - 1)]
            out["aux_interm_outputs"] = [{"pred_logits": ao["interm_logits"].clone(),
                                          "pred_keypoints": ao["interm_ref"][:, :, 1:].clone().flatten(-2)}]
            out["aux_pre_outputs"] = {"pred_logits": ao["pre_logits"].clone(), "pred_keypoints": refs.clone()}
        return out

    def _forward_train_dn(self, samples, targets, scope):
        from .train import Trainer, train_forward
        dev = samples.device
        tr = getattr(self, "_trainer", None)
        if tr is None or tr.device != dev or tr.eng.dtype_name != self.compute_dtype or tr.scope != scope:
            tr = Trainer(self, dtype=self.compute_dtype, device=dev, scope=scope, ema=False)
            object.__setattr__(self, "_trainer", tr)
        with torch.cuda.device(dev), torch.enable_grad():
            out = train_forward(tr, samples, targets)
        tr.steps += 1
        return out


def build_model(size: str = "l", dtype: str = "bf16", cfg: dict | None = None):
    """Build (DETRPose, PostProcess) for size 'n' | 'l' | 'x' with the reference kwargs."""
    cfg = cfg or get_config(size)
    model = DETRPose(HGNetv2(**cfg["backbone"]), HybridEncoder(**cfg["encoder"]),
                     Transformer(**cfg["transformer"]), dtype=dtype)
    return model, PostProcess(**cfg["postprocessor"])
