#!/bin/bash
# Round 6: SQ counters of the fused stem (three-phase build) and of the 5x5 depthwise convs.
set -o pipefail
OUT=gpurun_out/${1:-r6j}; mkdir -p $OUT
export TMPDIR=/tmp
bash scripts/pmc_kernels.sh $OUT/stem scripts/stem_bench.py --reps 3 || { tail -5 $OUT/stem/p*.txt; exit 1; }
python scripts/pmc_summary.py $OUT/stem > $OUT/stem_pmc.txt
bash scripts/pmc_kernels.sh $OUT/dw scripts/dw_fwd_bench.py --reps 3 || { tail -5 $OUT/dw/p*.txt; exit 1; }
python scripts/pmc_summary.py $OUT/dw > $OUT/dw_pmc.txt
cat $OUT/stem_pmc.txt $OUT/dw_pmc.txt
rm -rf $OUT/stem/p? $OUT/dw/p?
