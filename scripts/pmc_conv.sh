#!/bin/bash
# PMC passes over conv_bench.py for a few shapes (one counter group per rocprofv3 run).
#   bash scripts/pmc_conv.sh <outdir> <only> [libs]
set -e -o pipefail
OUT=$1; ONLY=$2; LIBS=${3:-detrpose_amd/lib/libdetrpose_hip.so}
export TMPDIR=/tmp
mkdir -p $OUT
i=0
for G in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VMEM SQ_ACTIVE_INST_VMEM SQ_INST_LEVEL_VMEM" \
         "TA_BUSY_avr TA_DATA_STALLED_BY_TC_CYCLES_sum TCP_TCC_READ_REQ_LATENCY_sum TCP_TCC_READ_REQ_sum TCP_PENDING_STALL_CYCLES_sum TCP_TCC_WRITE_REQ_LATENCY_sum" \
         "TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum TCC_TAG_STALL_sum" \
         "SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_LDS_DATA_FIFO_FULL SQ_LDS_CMD_FIFO_FULL SQ_VMEM_TA_ADDR_FIFO_FULL SQ_VMEM_TA_CMD_FIFO_FULL SQ_INSTS_MFMA SQ_BUSY_CU_CYCLES" \
         "GRBM_GUI_ACTIVE GRBM_COUNT TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_STALL_sum"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $G -d $OUT/p$i -o run --output-format csv -- \
    python3 scripts/conv_bench.py --no-blas --reps 5 --rounds 1 --only "$ONLY" --libs "$LIBS" > $OUT/p$i.txt 2>&1
done
echo ok
