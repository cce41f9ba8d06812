#!/bin/bash
# Round 6: the fused-stem stage ablations (DP_STEM_ABL variant mini-libraries: bit k skips
# stage k+1, 32 the image loads), then the training path after the padded-dgrad change.
set -o pipefail
OUT=gpurun_out/${1:-r6h}; mkdir -p $OUT
export TMPDIR=/tmp
L=""; for A in 0 1 2 4 8 16 32 63; do L="$L,detrpose_amd/lib/variants/stem$A/libdetrpose_hip.so"; done
timeout -k 10 200 python -u scripts/stem_bench.py --libs ${L:1} --reps 20 > $OUT/stem_abl.txt 2>&1 || { tail -20 $OUT/stem_abl.txt; exit 1; }
cat $OUT/stem_abl.txt
bash scripts/r6_g.sh $1/g || exit 1
