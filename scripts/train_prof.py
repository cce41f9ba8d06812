"""Per-op device times of the training step's tapes (DETRPose-L bf16 b16 by default): each recorded
launch of the backbone / encoder / transformer forward and backward timed with HIP events on the
launch stream, summed by op name pattern. Writes a JSON summary (top ops, per-tape totals).

    python scripts/train_prof.py [--size l] [--batch 16] [--out gpurun_out/train_ops.json]
"""
import argparse
import ctypes as C
import json
import os
import re
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def timed_run(tape, reps=2):
    """Per-op event times of one tape (median over reps)."""
    from detrpose_amd import _lib
    s = torch.cuda.current_stream()
    res = {}
    for _ in range(reps):
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(len(tape.ops) + 1)]
        ev[0].record()
        for i, (name, fn, args) in enumerate(tape.ops):
            rc = fn(*args, C.c_void_p(s.cuda_stream))
            if rc:
                _lib.check(rc, name)
            ev[i + 1].record()
        torch.cuda.synchronize()
        for i, (name, _, _) in enumerate(tape.ops):
            res.setdefault(i, []).append(ev[i].elapsed_time(ev[i + 1]))
    return [(tape.ops[i][0], sorted(v)[len(v) // 2]) for i, v in res.items()]


def family(name):
    n = re.sub(r"\d+", "#", name)
    return n


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--size", default="l")
    ap.add_argument("--batch", type=int, default=16)
    ap.add_argument("--dtype", default="bf16")
    ap.add_argument("--out", default="gpurun_out/train_ops.json")
    ap.add_argument("--accum", type=int, default=None, help="grad_accum_steps (default: the config's)")
    a = ap.parse_args()
    from bench import synthetic_targets
    from detrpose_amd import build_model
    from detrpose_amd.synthetic import load_synthetic, synthetic_images
    from detrpose_amd.train import Trainer
    dev = torch.device("cuda")
    model, _ = build_model(a.size, dtype=a.dtype)
    load_synthetic(model, 0)
    tr = Trainer(model, dtype=a.dtype, device=dev, grad_accum_steps=a.accum)
    images = synthetic_images(a.batch, seed=11).to(dev)
    ts = synthetic_targets(a.batch, dev=dev)
    for _ in range(2):
        tr.step(images, ts)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    tr.step(images, ts)
    torch.cuda.synchronize()
    step_ms = (time.perf_counter() - t0) * 1e3
    plan = tr.plan   # the last sub-batch's
    sub = a.batch // tr.grad_accum_steps
    tapes = {"backbone_fwd": tr.bb.fw, "encoder_fwd": tr.ep.fw, "transformer_fwd": plan.fw,
             "transformer_bwd": plan.bw, "encoder_bwd": tr.ep.bw, "backbone_bwd": tr.bb.bw}
    out = {"size": a.size, "batch": a.batch, "grad_accum_steps": tr.grad_accum_steps, "dtype": a.dtype,
           "step_ms": round(step_ms, 2), "tapes_of_one_sub_batch": sub, "tapes": {}}
    allops = []
    for tname, tape in tapes.items():
        if tname == "transformer_bwd":   # the backward reads the criterion's hand-off
            from detrpose_amd.criterion import pack_targets
            from detrpose_amd.train import dn_meta
            packed = pack_targets(ts[a.batch - sub:], 17, dev)
            plan.criterion(packed, packed.sizes, dn_meta(packed.sizes)[1])
        ops = timed_run(tape)
        fam = {}
        for n, ms in ops:
            fam[family(n)] = fam.get(family(n), 0.0) + ms
            allops.append((ms, tname, n))
        out["tapes"][tname] = {"ms": round(sum(ms for _, ms in ops), 3), "launches": len(ops),
                               "top_families": sorted(((round(v, 3), k) for k, v in fam.items()), reverse=True)[:15]}
        print(tname, out["tapes"][tname]["ms"], "ms", out["tapes"][tname]["top_families"][:6], flush=True)
    allops.sort(reverse=True)
    out["top_ops"] = [(round(ms, 3), t, n) for ms, t, n in allops[:40]]
    out["all_ops"] = [(round(ms, 4), t, n) for ms, t, n in allops]
    os.makedirs(os.path.dirname(a.out) or ".", exist_ok=True)
    with open(a.out, "w") as f:
        json.dump(out, f, indent=1)
    print(json.dumps(out["top_ops"][:25]))


if __name__ == "__main__":
    main()
