#!/bin/bash
# Round 6 closing, training side at HEAD: the full bench line, the 2-rank shared-GPU rehearsal of
# the world-aware train leg, and the steady-state training kernel statistics per step.
set -o pipefail
OUT=gpurun_out/${1:-r6zf}; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 400 python -u bench.py > $OUT/bench.json 2> $OUT/bench.err || { tail -20 $OUT/bench.err; exit 1; }
python -c "import json; d=json.load(open('$OUT/bench.json')); print(d['value'], d['ms_per_step'], d['train_step']['ms_per_step'], json.dumps(d['train_step']['phase_ms_one_sub_batch']))"
NT="--no-cpu-baseline --no-latency --no-secondary --no-gemm-peak"
timeout -k 10 400 python -u bench.py --gpus 2 --shared-gpu-rehearsal --batch 8 --steps 5 --warmup 2 $NT \
  --train-batch 4 --train-steps 3 > $OUT/rehearsal2.json 2> $OUT/rehearsal2.err || { tail -20 $OUT/rehearsal2.err; exit 1; }
timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d $OUT/trace -o run -- python3 scripts/train_trace.py > $OUT/trace.log 2>&1 || { tail -20 $OUT/trace.log; exit 1; }
python scripts/trace_steps.py $(find $OUT/trace -name '*kernel_trace.csv' | head -1) 3 $OUT/train_kernel_steps.csv | head -12
rm -rf $OUT/trace
