#!/bin/bash
# Kernel A/B + tests for the compile-time-K halo conv and the 64-row two-stage head.
set -o pipefail
OUT=gpurun_out/r3i; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 200 python scripts/conv_bench.py --shapes conv3 --no-blas --only 's0.l' > $OUT/hk.txt 2>&1 || exit 1
DETRPOSE_HALO_RTK=1 timeout -k 10 200 python scripts/conv_bench.py --shapes conv3 --no-blas --only 's0.l' >> $OUT/hk.txt 2>&1 || exit 1
grep -v amdgpu.ids $OUT/hk.txt
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_decoder.py -k 'halo or conv2d or classmax' -x -q --timeout 120 --timeout-method thread > $OUT/t.txt 2>&1 || { tail -30 $OUT/t.txt; exit 1; }
tail -1 $OUT/t.txt
bash scripts/ab_model.sh r3i_m 'bf16 or fp32_matches or stem_fused' || exit 1
python -c "import json; o=json.load(open('$OUT'.replace('r3i','r3i_m')+'/ops.json'))['op_ms']; print({k: round(v*1e3,1) for k,v in o.items() if k.startswith('ts.') or k.startswith('s0.b0.l')})"
