#!/bin/bash
# Round 6 final pass at HEAD: the whole GPU suite, smoke(), and the bench line's training leg.
set -o pipefail
OUT=gpurun_out/${1:-r6zh}; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v -s --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 \
  || { tail -40 $OUT/pytest_gpu.log; exit 1; }
tail -1 $OUT/pytest_gpu.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { tail -20 $OUT/smoke.log; exit 1; }
tail -1 $OUT/smoke.log
NT="--no-cpu-baseline --no-latency --no-secondary --no-gemm-peak"
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 $NT > $OUT/bench.json 2> $OUT/bench.err || { tail -20 $OUT/bench.err; exit 1; }
python -c "import json; d=json.load(open('$OUT/bench.json')); print(d['value'], d['ms_per_step'], d['train_step']['ms_per_step'], json.dumps(d['train_step']['phase_ms_one_sub_batch']))"
