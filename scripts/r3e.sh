set -o pipefail
OUT=gpurun_out/r3e; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 200 python -u scripts/dec_bench.py --rows 1080,8640,69120 > $OUT/dec_bench.txt 2>&1 || { tail -20 $OUT/dec_bench.txt; exit 1; }
cat $OUT/dec_bench.txt
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE -d $OUT/pmc -o run --output-format csv -- python3 scripts/dec_bench.py --rows 69120 --reps 2 > $OUT/pmc.log 2>&1 || { tail -20 $OUT/pmc.log; exit 1; }
find $OUT/pmc -name "*.csv" | head
