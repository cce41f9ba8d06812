"""Per-section device time of the DETRPose plan for two compute dtypes (development tool).

    python scripts/section_cost.py [--size l] [--batch 64] [--out file.json]

Profiles the bf16 and the fp32 plan op by op (HIP events, median of 3) and sums the ops
per section (backbone / encoder / two-stage / decoder+heads): the cost of running a
section in fp32 while the rest stays bf16 is read off these sums ("Where the
bf16 error comes from").
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from detrpose_amd import build_model  # noqa: E402
from detrpose_amd.synthetic import load_synthetic, synthetic_images  # noqa: E402


def section(name):
    if name.startswith("stem") or (name.startswith("s") and name[1:2].isdigit()):
        return "backbone"
    if name.startswith("enc."):
        return "encoder"
    if name.startswith("ts."):
        return "two_stage"
    return "decoder"


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--size", default="l")
    ap.add_argument("--batch", type=int, default=64)
    ap.add_argument("--out", default="")
    a = ap.parse_args()
    res = {}
    for dt in ("bf16", "fp32"):
        m, _ = build_model(a.size, dtype=dt)
        load_synthetic(m, 0)
        m.deploy()
        plan = m.engine().plan(a.batch)
        plan.input.copy_(synthetic_images(a.batch, 1).cuda())
        plan.run()
        torch.cuda.synchronize()
        ms = plan.profile(reps=3)
        sec = {}
        for n, t in ms.items():
            sec[section(n)] = sec.get(section(n), 0.0) + t
        res[dt] = {k: round(v, 3) for k, v in sec.items()}
        res[dt]["total"] = round(sum(ms.values()), 3)
        print(dt, res[dt], flush=True)
        del plan, m
        m = None
        torch.cuda.empty_cache()
    b, f = res["bf16"], res["fp32"]
    mixed = b["backbone"] + b["encoder"] + b["two_stage"] + f["decoder"]
    res["mixed_bf16_bb_enc_ts_fp32_decoder_ms"] = round(mixed, 3)
    res["img_per_s_kernel_time"] = {"bf16": round(a.batch / b["total"] * 1e3, 1),
                                    "fp32": round(a.batch / f["total"] * 1e3, 1),
                                    "mixed": round(a.batch / mixed * 1e3, 1)}
    print(json.dumps(res))
    if a.out:
        json.dump(res, open(a.out, "w"), indent=1)


if __name__ == "__main__":
    main()
