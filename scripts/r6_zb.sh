#!/bin/bash
# Round 6 (late): per-op profile of every training launch at HEAD (scripts/train_prof.py).
set -o pipefail
OUT=gpurun_out/${1:-r6zb}; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python -u scripts/train_prof.py --batch 16 --out $OUT/train_ops_all.json > $OUT/train_prof.log 2>&1 || { tail -20 $OUT/train_prof.log; exit 1; }
tail -3 $OUT/train_prof.log
