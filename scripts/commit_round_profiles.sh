#!/bin/bash
# Copy one gpu_round.sh output directory's summaries into profiles/ under a round tag:
#   bash scripts/commit_round_profiles.sh r4f
# (kernel stats, per-op times, bench line, pytest log, PMC traffic / SQ summaries, training
# per-op profile). Run on the CPU side after gpurun merged gpurun_out/<tag>.
set -e
TAG=$1
D=gpurun_out/$TAG
test -d $D || { echo "no $D"; exit 1; }
[ -f $D/pytest_gpu.log ] && cp $D/pytest_gpu.log profiles/${TAG}_pytest_gpu.txt
if [ -s $D/bench.json ]; then
  python - "$D/bench.json" "profiles/${TAG}_bench_line.json" <<'PY'
import json, sys
line = [l for l in open(sys.argv[1]) if l.startswith("{")][-1]
json.dump(json.loads(line), open(sys.argv[2], "w"), indent=1)
print("img/s", json.loads(line)["value"])
PY
fi
IPS=$(python -c "import json;print(int(json.load(open('profiles/${TAG}_bench_line.json'))['value']))" 2>/dev/null || echo x)
[ -f $D/prof/run_kernel_stats.csv ] && cp $D/prof/run_kernel_stats.csv profiles/${TAG}_${IPS}ips_kernel_stats.csv
[ -f $D/ops.json ] && cp $D/ops.json profiles/${TAG}_ops.json
[ -f $D/train_ops.json ] && cp $D/train_ops.json profiles/${TAG}_train_ops.json
if [ -f $D/pmc_fetch/run_counter_collection.csv ] && [ -f $D/pmc_write/run_counter_collection.csv ]; then
  python scripts/pmc_traffic.py $D/pmc_fetch/run_counter_collection.csv $D/pmc_write/run_counter_collection.csv \
    profiles/${TAG}_pmc_traffic.json
  cp profiles/${TAG}_pmc_traffic.json profiles/pmc_traffic.json   # what bench.py quotes (same source hash)
fi
[ -f $D/pmc_sq/run_counter_collection.csv ] && python scripts/pmc_sq.py $D/pmc_sq/run_counter_collection.csv \
  profiles/${TAG}_pmc_sq.json
ls -la profiles/ | grep $TAG
