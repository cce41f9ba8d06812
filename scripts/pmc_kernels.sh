#!/bin/bash
# Three SQ/GRBM counter passes (one rocprofv3 --pmc run each) over a small kernel benchmark:
#   bash scripts/pmc_kernels.sh <outdir> <python script + args>
# summarise with: python scripts/pmc_summary.py <outdir>
set -e -o pipefail
OUT=$1; shift
export TMPDIR=/tmp
mkdir -p $OUT
i=0
for G in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU" \
         "SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_LDS_IDX_ACTIVE SQ_INSTS_MFMA SQ_INSTS_SMEM SQ_ACTIVE_INST_LDS SQ_INSTS_BRANCH" \
         "GRBM_GUI_ACTIVE GRBM_COUNT SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_WAVES SQ_INSTS_WAVE32_LDS"; do
  i=$((i+1))
  timeout -s KILL 60 rocprofv3 --pmc $G -d $OUT/p$i -o run --output-format csv -- python3 "$@" > $OUT/p$i.txt 2>&1
done
echo ok
