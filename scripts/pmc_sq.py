"""Per-kernel-family SQ counters from one rocprofv3 --pmc pass (scripts/gpu_round.sh):
MFMA busy fraction, LDS bank-conflict fraction and wave-state split; plus the three conv
kernel instantiations with the most GPU time ("top3: <kernel name>").

    python scripts/pmc_sq.py <pmc_sq counter_collection.csv> [out.json]

mfma_busy  = SQ_VALU_MFMA_BUSY_CYCLES / (GRBM_GUI_ACTIVE / 8 XCDs x 1024 SIMDs)
             (MFMA-pipe cycles over all SIMD-cycles of the dispatch; MI355X_MICROARCH.md)
lds_conflict = SQ_LDS_BANK_CONFLICT / SQ_LDS_IDX_ACTIVE (extra LDS cycles over all)
wait_any / wait_inst / active = SQ_WAIT_ANY, SQ_WAIT_INST_ANY, rest, over SQ_WAVE_CYCLES
"""
import collections
import csv
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from pmc_traffic import family  # noqa: E402


def kfamily(name):
    for k in ("conv_stream_kernel", "conv_halo_kernel", "conv_gemm_kernel", "conv_direct_kernel"):
        if k in name:
            return k
    return family(name)


def main():
    per = collections.defaultdict(lambda: collections.defaultdict(float))
    disp, name = {}, {}
    for r in csv.DictReader(open(sys.argv[1])):
        key = r["Dispatch_Id"]
        disp[key] = kfamily(r["Kernel_Name"])
        name[key] = r["Kernel_Name"]
        per[key][r["Counter_Name"]] += float(r["Counter_Value"])
    fam = collections.defaultdict(lambda: collections.defaultdict(float))
    inst = collections.defaultdict(lambda: collections.defaultdict(float))   # per kernel instantiation
    for k, cs in per.items():
        for c, v in cs.items():
            fam[disp[k]][c] += v
            if disp[k].startswith("conv_"):
                inst[name[k]][c] += v
        fam[disp[k]]["dispatches"] += 1
        if disp[k].startswith("conv_"):
            inst[name[k]]["dispatches"] += 1
    out = {}
    # the three conv instantiations with the most GPU time get their own rows
    top = sorted(inst.items(), key=lambda kv: -kv[1]["GRBM_GUI_ACTIVE"])[:3]
    groups = sorted(fam.items(), key=lambda kv: -kv[1]["GRBM_GUI_ACTIVE"]) + [("top3: " + n, cs) for n, cs in top]
    for f, cs in groups:
        gui = cs["GRBM_GUI_ACTIVE"] / 8.0
        if gui <= 0 or f == "other":
            continue
        wc = max(cs["SQ_WAVE_CYCLES"], 1.0)
        row = {"dispatches": int(cs["dispatches"]),
               "mfma_busy": cs["SQ_VALU_MFMA_BUSY_CYCLES"] / (gui * 1024.0),
               "lds_conflict": cs["SQ_LDS_BANK_CONFLICT"] / max(cs["SQ_LDS_IDX_ACTIVE"], 1.0),
               "wait_any": cs["SQ_WAIT_ANY"] / wc, "wait_inst": cs["SQ_WAIT_INST_ANY"] / wc,
               "active": 1.0 - (cs["SQ_WAIT_ANY"] + cs["SQ_WAIT_INST_ANY"]) / wc}
        out[f] = row
        print(f"{f[:60]:22s} n={row['dispatches']:4d} mfma_busy {row['mfma_busy']:.3f} lds_conflict "
              f"{row['lds_conflict']:.4f} wait_any {row['wait_any']:.2f} wait_inst {row['wait_inst']:.2f} "
              f"active {row['active']:.2f}")
    if len(sys.argv) > 2:
        with open(sys.argv[2], "w") as fh:
            json.dump(out, fh, indent=1)


if __name__ == "__main__":
    main()
