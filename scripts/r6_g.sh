#!/bin/bash
# Round 6: weight-gradient split heuristic + padded head gradients: GEMM / training tests, bench train leg, trace.
set -o pipefail
OUT=gpurun_out/${1:-r6g}; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_train_ops.py -k "gemm" -x -q -s --timeout 300 --timeout-method thread > $OUT/ops.log 2>&1 || { tail -30 $OUT/ops.log; exit 1; }
grep -E "passed|failed" $OUT/ops.log | tail -2
timeout -k 10 800 python -u -m pytest tests/test_gpu_train_step.py tests/test_gpu_full_train_step.py tests/test_gpu_full_train_step_l.py tests/test_gpu_train.py -x -q --timeout 500 --timeout-method thread > $OUT/train.log 2>&1 || { tail -30 $OUT/train.log; exit 1; }
tail -1 $OUT/train.log
NT="--no-cpu-baseline --no-latency --no-secondary --no-gemm-peak"
timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 $NT > $OUT/bench.json 2> $OUT/bench.err || { tail -20 $OUT/bench.err; exit 1; }
python -c "import json; d=json.load(open('$OUT/bench.json')); print(d['value'], json.dumps(d['train_step']['ms_per_step']), json.dumps(d['train_step']['phase_ms_one_sub_batch']))"
timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d $OUT/trace -o run -- python3 scripts/train_trace.py > $OUT/trace.log 2>&1 || { tail -20 $OUT/trace.log; exit 1; }
python scripts/trace_steps.py $(find $OUT/trace -name '*kernel_trace.csv' | head -1) 3 $OUT/train_kernel_steps.csv | head -16
rm -rf $OUT/trace
