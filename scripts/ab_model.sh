#!/bin/bash
# Model-level GPU check: the named model tests (pytest -k), then one bench run with the
# per-op profile.   bash scripts/ab_model.sh <tag> "<pytest -k expr>"
set -o pipefail
OUT=gpurun_out/${1:-model}; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_model.py -k "$2" -x -q --timeout 200 --timeout-method thread > $OUT/model.log 2>&1 || { tail -30 $OUT/model.log; exit 1; }
tail -1 $OUT/model.log
timeout -k 10 200 python -u bench.py --steps 50 --warmup 10 --no-cpu-baseline --no-latency --no-secondary --profile-ops $OUT/ops.json > $OUT/bench.json 2> $OUT/bench.err || { tail -20 $OUT/bench.err; exit 1; }
python -c "import json; d=json.load(open('$OUT/bench.json')); print(d['value'], d['roofline']['frac'], d['kernel_ms_per_step'])"
