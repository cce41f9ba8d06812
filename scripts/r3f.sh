set -o pipefail
OUT=gpurun_out/r3f; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_decoder.py tests/test_gpu_model.py -x -q --timeout 200 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
for bm in 64 96 128; do
  DETRPOSE_DEC_BM=$bm timeout -k 10 200 python -u scripts/dec_bench.py --rows 1080,69120 > $OUT/dec_bench_bm$bm.txt 2>&1 || { tail -20 $OUT/dec_bench_bm$bm.txt; exit 1; }
  echo "BM=$bm"; grep rows $OUT/dec_bench_bm$bm.txt
done
