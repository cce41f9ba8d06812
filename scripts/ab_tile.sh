#!/bin/bash
# conv_bench on the 1x1 GEMM shapes with every big conv_stream tile forced (DETRPOSE_CONV_TILE).
set -o pipefail
OUT=gpurun_out/${1:-tile}; mkdir -p $OUT
for t in 0 1 2 3 4; do
  DETRPOSE_CONV_TILE=$t timeout -k 10 200 python -u scripts/conv_bench.py --shapes gemm --no-blas --reps 20 --rounds 3 > $OUT/cb_t$t.txt 2>&1 || { tail -20 $OUT/cb_t$t.txt; exit 1; }
  echo "== tile=$t"; cat $OUT/cb_t$t.txt
done
