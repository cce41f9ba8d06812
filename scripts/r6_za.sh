#!/bin/bash
# Round 6 (late): deterministic forward GEMMs (no init-then-split on a Linear with a bias), batched
# criterion row copies, one EMA launch for the running statistics: tests, training bench leg.
set -o pipefail
OUT=gpurun_out/${1:-r6za2}; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_train_ops.py tests/test_gpu_encoder_train_ops.py -x -q --timeout 300 --timeout-method thread > $OUT/ops.log 2>&1 || { tail -30 $OUT/ops.log; exit 1; }
tail -1 $OUT/ops.log
timeout -k 10 900 python -u -m pytest tests/test_gpu_train_graphs.py tests/test_gpu_train_step.py tests/test_gpu_full_train_step.py tests/test_gpu_full_train_step_l.py tests/test_gpu_train.py tests/test_gpu_trainer_dist.py tests/test_gpu_encoder_train_step.py -x -v -s --timeout 500 --timeout-method thread > $OUT/train.log 2>&1 || { tail -40 $OUT/train.log; exit 1; }
tail -1 $OUT/train.log
NT="--no-cpu-baseline --no-latency --no-secondary --no-gemm-peak"
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 $NT > $OUT/bench.json 2> $OUT/bench.err || { tail -20 $OUT/bench.err; exit 1; }
python -c "import json; d=json.load(open('$OUT/bench.json')); print(d['value'], d['ms_per_step'], json.dumps(d['train_step']['ms_per_step']), json.dumps(d['train_step']['phase_ms_one_sub_batch']))"
