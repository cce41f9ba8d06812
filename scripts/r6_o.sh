#!/bin/bash
# Round 6: fused stem with single-instruction bf16 pair conversions and unconditional LDS stores
# into padded planes: A/B vs the five-barrier build, stem bit-identity.
set -o pipefail
OUT=gpurun_out/${1:-r6o}; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 200 python -u scripts/stem_bench.py --libs detrpose_amd/lib/libdetrpose_hip.so,detrpose_amd/lib/variants/stem0/libdetrpose_hip.so --reps 30 > $OUT/stem_ab.txt 2>&1 || { tail -20 $OUT/stem_ab.txt; exit 1; }
cat $OUT/stem_ab.txt
timeout -k 10 600 python -u -m pytest tests/test_gpu_model.py tests/test_gpu_kernels.py -k "stem" -x -q --timeout 300 --timeout-method thread > $OUT/pytest_stem.log 2>&1 || { tail -30 $OUT/pytest_stem.log; exit 1; }
tail -1 $OUT/pytest_stem.log
timeout -k 10 300 python -u scripts/train_prof.py --batch 8 --out $OUT/train_ops_b8.json > $OUT/train_prof.log 2>&1 || { tail -20 $OUT/train_prof.log; exit 1; }
tail -30 $OUT/train_prof.log
