"""Average rocprofv3 --pmc counters per kernel over the passes written by pmc_conv.sh.
    python scripts/pmc_summary.py gpurun_out/pmc_conv1"""
import collections
import csv
import glob
import sys

acc = collections.defaultdict(lambda: collections.defaultdict(list))
dur = collections.defaultdict(list)
for f in sorted(glob.glob(sys.argv[1] + "/p*/*counter_collection.csv")):
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"][:90]
        acc[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, cs in acc.items():
    if "rocclr" in k or "elementwise" in k or "distribution" in k:
        continue
    print(k)
    for c, v in sorted(cs.items()):
        print(f"   {c:36s} {sum(v) / len(v):16.4g}   (n={len(v)})")
