#!/bin/bash
# Round 6: per-op times of every launch of one L b8 training sub-batch (all ops, for the routing
# of the small-N GEMMs).
set -o pipefail
OUT=gpurun_out/${1:-r6u}; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python -u scripts/train_prof.py --batch 16 --out $OUT/train_ops_all.json > $OUT/train_prof.log 2>&1 || { tail -20 $OUT/train_prof.log; exit 1; }
tail -3 $OUT/train_prof.log | cut -c1-300
