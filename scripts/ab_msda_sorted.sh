#!/bin/bash
# Kernel times of dp_msda_bwd_sorted's three kernels (scripts/msda_bwd_bench.py under rocprofv3
# kernel trace) for the production library and the ablation variant libraries given as
# tag=path arguments (variant libraries, e.g. built with DETRPOSE_EXTRA_FLAGS into detrpose_amd/lib/variants/).
#   bash scripts/ab_msda_sorted.sh <out dir> [tag=lib ...]
set -o pipefail
OUT=$1; shift; mkdir -p $OUT
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
run() {
  cd /tmp && timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $R/$OUT/$1 -o run -- python $R/scripts/msda_bwd_bench.py --reps 3 > $R/$OUT/$1.log 2>&1
}
run base || exit 1
DETRPOSE_MSDA_K3_CPL=8 run k3cpl8 || exit 1
for tv in "$@"; do
  tag=${tv%%=*}; lib=${tv#*=}
  DETRPOSE_HIP_LIB=$R/$lib DETRPOSE_ALLOW_STALE_LIB=1 run $tag || exit 1
done
cd $R && python - $OUT <<'PY'
import csv, glob, os, sys, collections
out = sys.argv[1]
for d in sorted(glob.glob(os.path.join(out, "*/"))):
    t = collections.defaultdict(list)
    for f in glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            n = r["Kernel_Name"]
            for k in ("msda_sort_kernel", "msda_sorted_bwd_kernel", "msda_value_sum_kernel", "msda_fused_bwd_cl"):
                if k in n:
                    t[k].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1000)
    print(os.path.basename(d.rstrip("/")), {k: [round(sum(v[:len(v)//2]) / max(1, len(v)//2), 1), round(sum(v[len(v)//2:]) / max(1, len(v) - len(v)//2), 1)] for k, v in t.items()})
PY
