#!/bin/bash
# Round 6: fused stem with packed bias/ReLU epilogues (A/B vs the five-barrier build), stem
# bit-identity, transformer packs on their own batched tape + batched refresh copies (training
# tests, bench train leg).
set -o pipefail
OUT=gpurun_out/${1:-r6k}; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 200 python -u scripts/stem_bench.py --libs detrpose_amd/lib/libdetrpose_hip.so,detrpose_amd/lib/variants/stem0/libdetrpose_hip.so --reps 30 > $OUT/stem_ab.txt 2>&1 || { tail -20 $OUT/stem_ab.txt; exit 1; }
cat $OUT/stem_ab.txt
timeout -k 10 600 python -u -m pytest tests/test_gpu_model.py tests/test_gpu_kernels.py -k "stem" -x -q --timeout 300 --timeout-method thread > $OUT/pytest_stem.log 2>&1 || { tail -30 $OUT/pytest_stem.log; exit 1; }
tail -1 $OUT/pytest_stem.log
timeout -k 10 900 python -u -m pytest tests/test_gpu_train_step.py tests/test_gpu_full_train_step.py tests/test_gpu_full_train_step_l.py tests/test_gpu_train.py tests/test_gpu_trainer_dist.py -x -q --timeout 500 --timeout-method thread > $OUT/train.log 2>&1 || { tail -30 $OUT/train.log; exit 1; }
tail -1 $OUT/train.log
NT="--no-cpu-baseline --no-latency --no-secondary --no-gemm-peak"
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 $NT > $OUT/bench.json 2> $OUT/bench.err || { tail -20 $OUT/bench.err; exit 1; }
python -c "import json; d=json.load(open('$OUT/bench.json')); print(d['value'], d['ms_per_step'], json.dumps(d['train_step']['ms_per_step']), json.dumps(d['train_step']['phase_ms_one_sub_batch']))"
