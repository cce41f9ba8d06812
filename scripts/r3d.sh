set -o pipefail
OUT=gpurun_out/r3d; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_decoder.py tests/test_gpu_model.py -x -q --timeout 200 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
for bm in 64 96 128; do
  DETRPOSE_DEC_BM=$bm timeout -k 10 200 python -u scripts/prof_plan.py --top 0 --json $OUT/ops_bm$bm.json > $OUT/prof_bm$bm.txt 2>&1 || { tail -20 $OUT/prof_bm$bm.txt; exit 1; }
  head -3 $OUT/prof_bm$bm.txt
done
