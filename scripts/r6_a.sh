#!/bin/bash
# Round 6 first pass: halo-conv kernel tests, the bf16 L split training test, the pipelined vs
# unpipelined halo conv A/B (outputs compared), and one bench run with the per-op profile.
set -o pipefail
OUT=gpurun_out/${1:-r6a}; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_train_ops.py tests/test_gpu_train_step.py tests/test_gpu_encoder_train_ops.py -k "wgrad or conv2d or attention_fwd_bwd_bf16 or adamw or step_guard" -x -q -s --timeout 200 --timeout-method thread > $OUT/kern.log 2>&1 || { tail -30 $OUT/kern.log; exit 1; }
tail -2 $OUT/kern.log
timeout -k 10 300 python -u scripts/conv_bench.py --shapes all --rounds 3 --no-blas --check \
  --libs detrpose_amd/lib/libdetrpose_hip.so,detrpose_amd/lib/variants/nopipe/libdetrpose_hip.so > $OUT/cb.txt 2>&1 || { tail -30 $OUT/cb.txt; exit 1; }
cat $OUT/cb.txt
timeout -k 10 200 python -u bench.py --steps 50 --warmup 10 --no-cpu-baseline --no-latency --no-secondary --no-train --profile-ops $OUT/ops.json > $OUT/bench.json 2> $OUT/bench.err || { tail -20 $OUT/bench.err; exit 1; }
python -c "import json; d=json.load(open('$OUT/bench.json')); print(d['value'], d['roofline']['frac'], d['roofline']['avg_launch_us'], d['kernel_ms_per_step'])"
timeout -k 10 400 python -u -m pytest tests/test_gpu_full_train_step_l.py -k "split_backbone" -x -q -s --timeout 350 --timeout-method thread > $OUT/split.log 2>&1 || { grep -E "split|passed|failed|Error" $OUT/split.log | tail -30; exit 1; }
grep -E "bf16 split|passed|failed" $OUT/split.log
timeout -k 10 400 python -u -m pytest tests/test_gpu_model.py -x -q -s --timeout 350 --timeout-method thread > $OUT/model.log 2>&1 || { tail -30 $OUT/model.log; exit 1; }
tail -2 $OUT/model.log
