#!/bin/bash
# PMC passes over stem_bench.py (one counter group per rocprofv3 run).  bash scripts/pmc_stem.sh <outdir>
set -e -o pipefail
OUT=$1
export TMPDIR=/tmp
mkdir -p $OUT
i=0
for G in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU" \
         "SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_LDS_IDX_ACTIVE SQ_INSTS_MFMA SQ_INSTS_SMEM SQ_ACTIVE_INST_LDS SQ_INSTS_BRANCH" \
         "GRBM_GUI_ACTIVE GRBM_COUNT TCC_EA0_WRREQ_sum TCC_EA0_RDREQ_sum"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $G -d $OUT/p$i -o run --output-format csv -- \
    python3 scripts/stem_bench.py --reps 3 > $OUT/p$i.txt 2>&1
done
echo ok
