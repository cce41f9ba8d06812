#!/bin/bash
# Round 6 third pass: forced-state L parity (bounds set), world-2 Trainer, steady-state training trace.
set -o pipefail
OUT=gpurun_out/${1:-r6c}; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_full_train_step_l.py -k "own_forward_state" -x -q -s --timeout 500 --timeout-method thread > $OUT/forced.log 2>&1
grep -E "forced-state|stored layer|passed|failed|^E " $OUT/forced.log | tail -12
timeout -k 10 600 python -u -m pytest tests/test_gpu_trainer_dist.py -x -q -s --timeout 500 --timeout-method thread > $OUT/dist.log 2>&1
grep -E "step|passed|failed|^E " $OUT/dist.log | tail -14
timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d $OUT/trace -o run -- python3 scripts/train_trace.py > $OUT/trace.log 2>&1 || { tail -20 $OUT/trace.log; exit 1; }
python scripts/trace_steps.py $(find $OUT/trace -name '*kernel_trace.csv' | head -1) 3 $OUT/train_kernel_steps.csv
rm -rf $OUT/trace
