"""TEST INFRASTRUCTURE: the CPU oracle (oracle/detrpose_cpu.py) with the HIP path's bf16 storage
emulated (the rounding points of scripts/bf16_attrib.py as a context manager): every conv /
linear rounds its input activation and weight to bf16 (the kernels store activations and
weights in bf16 and accumulate in f32), attention rounds Q / K / V, the probabilities and its
output, LayerNorm outputs are rounded, the encoder's output maps (the MSDA memory / LQE
feats[0]) are stored bf16, MSDA outputs are rounded; the pose / pre-pose / two-stage heads'
last layers keep f32 outputs, as on the GPU.

    with bf16_emulation():
        out = OracleDETRPose(cfg, sd)(images, force_topk=idx)
"""
from __future__ import annotations

import contextlib
import math
import types

import torch
import torch.nn.functional as TF


def _r(x):
    return x.to(torch.bfloat16).to(torch.float32)


@contextlib.contextmanager
def bf16_emulation(offsets_bf16=True):
    """offsets_bf16: the MSDA sampling-offset / attention-logit Linear outputs stored bf16, as the
    inference path's dp_mha_layernorm writes them (False: f32, DP_MSDA_OFFATTN_F32's input)."""
    import oracle.detrpose_cpu as O
    saved = {n: getattr(O, n) for n in ("F", "encoder", "_mlp", "_mha", "msda_core", "_linear")}
    orig_enc, orig_msda, orig_lin = O.encoder, O.msda_core, O._linear

    def conv2d(x, w, b=None, *a, **k):
        return TF.conv2d(_r(x), _r(w), b, *a, **k)

    def linear(x, w, b=None):
        return TF.linear(_r(x), _r(w), b)

    def layer_norm(x, shape, w, b, eps):
        return _r(TF.layer_norm(x, shape, w, b, eps))

    F = types.SimpleNamespace(**{k: getattr(TF, k) for k in dir(TF) if not k.startswith("_")})
    F.conv2d, F.linear, F.layer_norm = conv2d, linear, layer_norm

    def mlp(x, sd, p, n):
        for i in range(n):
            x = O._linear(x, sd, f"{p}.layers.{i}")   # F.linear above: rounds input and weight
            if i < n - 1:
                x = _r(TF.relu(x))
        return x

    def mha(q, k, v, sd, p, nhead):
        W, b = sd[p + ".in_proj_weight"], sd[p + ".in_proj_bias"]
        C = q.shape[-1]
        Q, K, V = (_r(F.linear(t, W[i * C:(i + 1) * C], b[i * C:(i + 1) * C])) for i, t in enumerate((q, k, v)))
        B, L, _ = Q.shape
        dh = C // nhead
        Q = Q.reshape(B, L, nhead, dh).transpose(1, 2)
        K = K.reshape(B, -1, nhead, dh).transpose(1, 2)
        V = V.reshape(B, -1, nhead, dh).transpose(1, 2)
        a = _r(torch.softmax((Q / math.sqrt(dh)) @ K.transpose(-1, -2), dim=-1))
        o = _r((a @ V).transpose(1, 2).reshape(B, L, C))
        return _r(F.linear(o, sd[p + ".out_proj.weight"], sd[p + ".out_proj.bias"]))

    def encoder(feats, sd, cfg):
        return [_r(o) for o in orig_enc(feats, sd, cfg)]

    def msda(value, shapes, loc, attn):
        return _r(orig_msda(value, shapes, loc, attn))

    def lin(x, sd, p):
        y = orig_lin(x, sd, p)
        return _r(y) if offsets_bf16 and ("sampling_offsets" in p or "attention_weights" in p) else y

    O.F, O.encoder, O._mlp, O._mha, O.msda_core, O._linear = F, encoder, mlp, mha, msda, lin
    try:
        yield
    finally:
        for n, f in saved.items():
            setattr(O, n, f)
