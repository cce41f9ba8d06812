#!/bin/bash
# conv_bench (all shapes) of the production library vs a variant library (outputs compared).
#   bash scripts/ab_lib.sh <tag> <variant lib>
set -o pipefail
OUT=gpurun_out/${1:-ablib}; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 400 python -u scripts/conv_bench.py --shapes all --rounds 3 --no-blas --check --libs detrpose_amd/lib/libdetrpose_hip.so,$2 > $OUT/cb.txt 2>&1 || { tail -30 $OUT/cb.txt; exit 1; }
cat $OUT/cb.txt
