"""Attribute the bf16 path's end-to-end error to stages, on the CPU (no GPU needed).

The CPU oracle (oracle/detrpose_cpu.py, test infrastructure) is run with bf16 storage
rounding switched on stage by stage: for a stage that is "bf16", every conv / linear
rounds its input activation and weight to bf16 (the HIP path stores every activation and
weight in bf16 and accumulates in f32), attention rounds Q/K/V and the probabilities, and
LayerNorm outputs (the decoder's residual stream) are rounded. Stages:

  bb     backbone (hgnetv2.py)              enc    hybrid encoder + the memory it writes
  ts     two-stage selection linears/LN     dec    decoder-layer GEMMs, attention, MSDA out
  resid  decoder residual stream (LN outs)  pos    query-pos MLP (half_pose_ref_point_head)
  head   pose / pre-pose MLP inputs+hidden  (their last layer writes f32, as on the GPU)

Every configuration is compared with the fp32 oracle on the SAME two-stage selection
(force_topk), so the numbers are the slot-by-slot error the GPU test measures.

    python scripts/bf16_attrib.py [--size l] [--batch 1]
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import types

import torch
import torch.nn.functional as TF

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)

import oracle.detrpose_cpu as O  # noqa: E402
from detrpose_amd.configs import get_config  # noqa: E402
from detrpose_amd.synthetic import synthetic_images, synthetic_state_dict  # noqa: E402

STAGES = ("bb", "enc", "ts", "dec", "resid", "pos", "head")
ON: set = set()
CUR = ["bb"]


def r(x):
    return x.to(torch.bfloat16).to(torch.float32) if CUR[0] in ON else x


def _conv2d(x, w, b=None, *a, **k):
    return TF.conv2d(r(x), r(w), b, *a, **k)


def _linear(x, w, b=None):
    return TF.linear(r(x), r(w), b)


def _layer_norm(x, shape, w, b, eps):
    y = TF.layer_norm(x, shape, w, b, eps)
    if CUR[0] == "dec":
        return y.to(torch.bfloat16).float() if "resid" in ON else y
    return r(y)


F = types.SimpleNamespace(**{k: getattr(TF, k) for k in dir(TF) if not k.startswith("_")})
F.conv2d, F.linear, F.layer_norm = _conv2d, _linear, _layer_norm
O.F = F

_orig = {n: getattr(O, n) for n in ("backbone", "encoder", "decoder_layer", "_mlp", "_mha", "msda_core", "lqe")}


def staged(name, fn):
    def w(*a, **k):
        prev = CUR[0]
        CUR[0] = name
        try:
            return fn(*a, **k)
        finally:
            CUR[0] = prev
    return w


def _mlp(x, sd, p, n):
    st = "ts" if "enc_pose_embed" in p else "pos" if "half_pose" in p else "head"
    prev = CUR[0]
    CUR[0] = st
    try:
        for i in range(n):
            last = i == n - 1
            # last layer of pose / pre-pose / enc_pose heads writes f32 on the GPU: round the input only
            x = O._linear(x, sd, f"{p}.layers.{i}")
            if not last:
                x = r(TF.relu(x))
        return x
    finally:
        CUR[0] = prev


def _mha(q, k, v, sd, p, nhead):
    import math
    W, b = sd[p + ".in_proj_weight"], sd[p + ".in_proj_bias"]
    C = q.shape[-1]
    Q, K, V = (r(F.linear(t, W[i * C:(i + 1) * C], b[i * C:(i + 1) * C])) for i, t in enumerate((q, k, v)))
    B, L, _ = Q.shape
    dh = C // nhead
    Q = Q.reshape(B, L, nhead, dh).transpose(1, 2)
    K = K.reshape(B, -1, nhead, dh).transpose(1, 2)
    V = V.reshape(B, -1, nhead, dh).transpose(1, 2)
    a = r(torch.softmax((Q / math.sqrt(dh)) @ K.transpose(-1, -2), dim=-1))
    o = r((a @ V).transpose(1, 2).reshape(B, L, C))
    return r(F.linear(o, sd[p + ".out_proj.weight"], sd[p + ".out_proj.bias"]))


def _msda(value, shapes, loc, attn):
    return r(_orig["msda_core"](value, shapes, loc, attn))


def _encoder(feats, sd, cfg):
    outs = staged("enc", _orig["encoder"])(feats, sd, cfg)
    CUR[0], prev = "enc", CUR[0]
    outs = [r(o) for o in outs]        # memory / feats[0] are stored bf16
    CUR[0] = prev
    return outs


O.backbone = staged("bb", _orig["backbone"])
O.encoder = _encoder
O.decoder_layer = staged("dec", _orig["decoder_layer"])
O._mlp = _mlp
O._mha = _mha
O.msda_core = _msda
O.lqe = staged("head", _orig["lqe"])


def run(orc, img, on, force):
    ON.clear()
    ON.update(on)
    CUR[0] = "ts"          # the transformer's top level (enc_output / LN / class linear)
    return orc(img, force_topk=force)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--size", default="l")
    ap.add_argument("--batch", type=int, default=1)
    ap.add_argument("--out", default="")
    a = ap.parse_args()
    torch.set_num_threads(min(8, len(os.sched_getaffinity(0))))
    g = __import__("numpy").load(os.path.join(REPO, "tests", "golden", f"detrpose_{a.size}_b{a.batch}.npz"))
    man = json.load(open(os.path.join(REPO, "tests", "golden", "manifest.json")))
    sd = synthetic_state_dict(man[a.size], seed=int(g["meta"][1]))
    from detrpose_amd import build_model
    m, _ = build_model(a.size)
    m.load_state_dict(sd, strict=False)
    orc = O.OracleDETRPose(get_config(a.size), m.state_dict())
    img = synthetic_images(a.batch, seed=int(g["meta"][2]))
    ref = run(orc, img, (), None)
    force = torch.from_numpy(g["topk_idx"])
    configs = [("all bf16", STAGES)] + [(f"only {s}", (s,)) for s in STAGES] + \
              [(f"all but {s}", tuple(x for x in STAGES if x != s)) for s in STAGES] + \
              [("all but dec+resid+head+pos", ("bb", "enc", "ts")),
               ("all but resid+head", ("bb", "enc", "ts", "dec", "pos"))]
    rows = []
    for name, on in configs:
        o = run(orc, img, on, force)
        dk = (o["pred_keypoints"] - ref["pred_keypoints"]).abs()
        dl = (o["pred_logits"] - ref["pred_logits"]).abs()
        row = {"config": name, "max_dkp": float(dk.max()), "mean_dkp": float(dk.mean()),
               "max_dlogit": float(dl.max()), "mean_dlogit": float(dl.mean())}
        rows.append(row)
        print(f"{name:32s} max|dkp| {row['max_dkp']:.2e} mean {row['mean_dkp']:.2e}   "
              f"max|dlogit| {row['max_dlogit']:.2e} mean {row['mean_dlogit']:.2e}", flush=True)
    if a.out:
        json.dump({"size": a.size, "batch": a.batch, "rows": rows}, open(a.out, "w"), indent=1)


if __name__ == "__main__":
    main()
