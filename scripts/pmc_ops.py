"""Map per-dispatch rocprofv3 PMC counters (sqlite rocpd output) to plan op names.

    python scripts/pmc_ops.py gpurun_out/pmc_sq/run_results.db [--size l --batch 64] [--top 40]

Each forward of the plan issues len(plan.ops) (+1 postprocess) dispatches in order; the
last complete forward in the trace is reported. Counters are summed over shader engines."""
import argparse
import collections
import os
import sqlite3
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("--size", default="l")
    ap.add_argument("--batch", type=int, default=64)
    ap.add_argument("--top", type=int, default=40)
    ap.add_argument("--sort", default="SQ_WAVE_CYCLES")
    a = ap.parse_args()
    from detrpose_amd import build_model
    from detrpose_amd.engine import Engine
    from detrpose_amd.synthetic import load_synthetic
    m, _ = build_model(a.size)
    load_synthetic(m, 0)
    plan = Engine(m, "bf16", device="cpu").plan(a.batch)
    names = [n for n, _, _ in plan.ops]
    c = sqlite3.connect(a.db)
    vals = collections.defaultdict(dict)
    kname, dur = {}, {}
    for did, kn, cn, v, d in c.execute(
            "select dispatch_id, kernel_name, counter_name, value, duration from counters_collection"):
        if "rocclr" in kn or "at::native" in kn or "elementwise" in kn:
            continue
        vals[did][cn] = vals[did].get(cn, 0.0) + v
        kname[did] = kn
        dur[did] = d
    ids = sorted(vals)
    per = len(names) + 1
    nf = len(ids) // per
    last = ids[(nf - 1) * per:(nf - 1) * per + len(names)]
    counters = sorted({k for d in last for k in vals[d]})
    rows = [(names[i], vals[d], dur[d], kname[d]) for i, d in enumerate(last)]
    rows.sort(key=lambda r: -r[1].get(a.sort, 0))
    print(f"{len(ids)} dispatches, {nf} forwards; counters: {counters}")
    hdr = f"{'op':26s} {'us':>7s} " + " ".join(f"{k[3:15]:>12s}" for k in counters)
    print(hdr)
    for n, v, d, kn in rows[:a.top]:
        print(f"{n:26s} {d / 1e3:7.1f} " + " ".join(f"{v.get(k, 0):12.3g}" for k in counters))


if __name__ == "__main__":
    main()
