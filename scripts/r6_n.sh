#!/bin/bash
# Round 6: 5x5 depthwise A/B on the 40x40 maps: persistent 8x20 tiles (production) vs one 8x40
# tile of 512 threads per block (dw1) vs one 4x40 tile of 256 threads (dw2); checksums must agree.
set -o pipefail
OUT=gpurun_out/${1:-r6n}; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 200 python -u scripts/dw_fwd_bench.py --reps 30 --libs detrpose_amd/lib/variants/dw1/libdetrpose_hip.so,detrpose_amd/lib/variants/dw2/libdetrpose_hip.so > $OUT/dw_ab.txt 2>&1 || { tail -20 $OUT/dw_ab.txt; exit 1; }
cat $OUT/dw_ab.txt
