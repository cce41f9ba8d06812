#!/bin/bash
# dp_mha_layernorm: decoder tests, then per-launch time of each DETRPOSE_MHA_MODE, then phase stamps
OUT=${1:-gpurun_out/mha}
mkdir -p $OUT
timeout -k 10 200 python -u -m pytest tests/test_gpu_decoder.py -m gpu -q -k mha --timeout 100 --timeout-method thread -s > $OUT/pytest.log 2>&1
grep -E "mha|passed|failed" $OUT/pytest.log | tail -8
for m in 0 1; do
  echo "mode $m: $(DETRPOSE_MHA_MODE=$m timeout -k 10 120 python scripts/mha_bench.py 2>/dev/null)" || exit 1
done
if [ -f detrpose_amd/lib/variants/mhat/libdetrpose_hip.so ]; then
  DETRPOSE_HIP_LIB=$PWD/detrpose_amd/lib/variants/mhat/libdetrpose_hip.so DETRPOSE_ALLOW_STALE_LIB=1 \
    timeout -k 10 120 python scripts/mha_bench.py --stamps 2>/dev/null
fi
