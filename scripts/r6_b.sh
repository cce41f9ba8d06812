#!/bin/bash
# Round 6 second pass: new GEMM/conv kernel tests, the forced-state L training parity (fp32 + bf16),
# the world-2 Trainer with graph segments, training graph replay, the bench (inference + training
# step) with and without the weight-gradient DMA kernel, the 192-row pipelined conv_stream A/B,
# and the model tests.
set -o pipefail
OUT=gpurun_out/${1:-r6b}; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_train_ops.py -k "gemm" -x -q -s --timeout 200 --timeout-method thread > $OUT/gemm.log 2>&1 || { tail -30 $OUT/gemm.log; exit 1; }
grep -E "wgrad|passed|failed" $OUT/gemm.log | tail -8
timeout -k 10 600 python -u -m pytest tests/test_gpu_full_train_step_l.py -k "own_forward_state" -x -q -s --timeout 500 --timeout-method thread > $OUT/forced.log 2>&1
grep -E "forced-state|stored layer|passed|failed|Error" $OUT/forced.log | tail -20
timeout -k 10 600 python -u -m pytest tests/test_gpu_trainer_dist.py tests/test_gpu_train_graphs.py -x -q -s --timeout 500 --timeout-method thread > $OUT/dist.log 2>&1 || { tail -30 $OUT/dist.log; }
grep -E "rank|step|passed|failed" $OUT/dist.log | tail -20
NT="--no-cpu-baseline --no-latency --no-secondary --no-gemm-peak"
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 $NT --profile-ops $OUT/ops.json > $OUT/bench.json 2> $OUT/bench.err || { tail -20 $OUT/bench.err; exit 1; }
python -c "import json; d=json.load(open('$OUT/bench.json')); print(d['value'], d['roofline']['frac'], d['roofline']['avg_launch_us'], d['kernel_ms_per_step']); print(json.dumps(d['train_step']))"
DETRPOSE_WGRAD_TT=0 timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 $NT > $OUT/bench_nott.json 2> $OUT/bench_nott.err || { tail -20 $OUT/bench_nott.err; exit 1; }
python -c "import json; d=json.load(open('$OUT/bench_nott.json')); print('no wgrad_tt:', d['value'], json.dumps(d['train_step']['ms_per_step']), json.dumps(d['train_step']['phase_ms_one_sub_batch']))"
timeout -k 10 300 python -u scripts/conv_bench.py --shapes gemm --rounds 3 --no-blas --check \
  --libs detrpose_amd/lib/libdetrpose_hip.so,detrpose_amd/lib/variants/nopipe/libdetrpose_hip.so > $OUT/cb.txt 2>&1 || { tail -30 $OUT/cb.txt; exit 1; }
cat $OUT/cb.txt
timeout -k 10 400 python -u -m pytest tests/test_gpu_model.py tests/test_gpu_kernels.py -x -q --timeout 350 --timeout-method thread > $OUT/model.log 2>&1 || { tail -30 $OUT/model.log; exit 1; }
tail -2 $OUT/model.log
timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d $OUT/trace -o run -- python3 scripts/train_trace.py > $OUT/trace.log 2>&1 || { tail -20 $OUT/trace.log; exit 1; }
python scripts/trace_steps.py $(find $OUT/trace -name '*kernel_trace.csv' | head -1) 3 $OUT/train_kernel_steps.csv
rm -rf $OUT/trace
