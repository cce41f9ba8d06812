#!/bin/bash
# Round 6: the three-phase fused stem (pixel-major image patch, stem1 beside stem3/stem4):
# isolated A/B against the five-barrier build, bit-identity and inference parity, bench line.
set -o pipefail
OUT=gpurun_out/${1:-r6i}; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 200 python -u scripts/stem_bench.py --libs detrpose_amd/lib/libdetrpose_hip.so,detrpose_amd/lib/variants/stem0/libdetrpose_hip.so --reps 30 > $OUT/stem_ab.txt 2>&1 || { tail -20 $OUT/stem_ab.txt; exit 1; }
cat $OUT/stem_ab.txt
timeout -k 10 600 python -u -m pytest tests/test_gpu_model.py tests/test_gpu_kernels.py -k "stem or fp32_matches or bf16" -x -q --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
NT="--no-cpu-baseline --no-latency --no-secondary --no-gemm-peak --no-train"
timeout -k 10 300 python -u bench.py --steps 30 --warmup 5 $NT --profile-ops $OUT/ops.json > $OUT/bench.json 2> $OUT/bench.err || { tail -20 $OUT/bench.err; exit 1; }
python -c "import json; d=json.load(open('$OUT/bench.json')); print(d['value'], d['ms_per_step'], json.dumps(d['roofline']))"
python -c "import json; d=json.load(open('$OUT/ops.json'))['op_ms']; print('stem', d.get('stem'))"
