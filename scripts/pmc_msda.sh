#!/bin/bash
# PMC passes (one counter group per run, separate --pmc passes) over scripts/msda_bwd_bench.py,
# summed per kernel: where the MSDA backward kernels' time goes.
#   bash scripts/pmc_msda.sh <out dir>
set -o pipefail
OUT=$1; mkdir -p $OUT
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
pass() {
  local tag=$1; shift
  cd /tmp && timeout -s KILL 90 rocprofv3 --pmc "$@" -d $R/$OUT/$tag -o run --output-format csv -- \
    python3 $R/scripts/msda_bwd_bench.py --reps 2 > $R/$OUT/$tag.log 2>&1
}
pass sq1 SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_VMEM_RD GRBM_GUI_ACTIVE || exit 1
pass sq2 SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_INSTS_SALU SQ_INSTS_SMEM SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS || exit 1
pass tcc TCC_HIT_sum TCC_MISS_sum || exit 1
pass fetch FETCH_SIZE || exit 1
pass write WRITE_SIZE || exit 1
cd $R && python3 - $OUT <<'PY'
import csv, glob, os, sys, collections, json
out = sys.argv[1]
tot = collections.defaultdict(lambda: collections.defaultdict(float))
n = collections.defaultdict(set)
for f in glob.glob(os.path.join(out, "**", "*counter_collection.csv"), recursive=True):
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"]
        for key in ("msda_sort_kernel", "msda_sorted_bwd_kernel", "msda_value_sum_kernel", "msda_fused_bwd_cl"):
            if key in k:
                tot[key][r["Counter_Name"]] += float(r["Counter_Value"])
                n[key].add((f, r["Dispatch_Id"]))
res = {}
for k, cs in tot.items():
    d = len(n[k]) / 5.0   # dispatches per pass
    res[k] = {c: v / max(d, 1) for c, v in sorted(cs.items())}
print(json.dumps(res, indent=1))
json.dump(res, open(os.path.join(out, "pmc_msda.json"), "w"), indent=1)
PY
