#!/bin/bash
# A/B of the 128-channel halo conv: conv kernel tests, conv_bench over variant libraries, model parity, bench.
set -o pipefail
OUT=gpurun_out/${1:-halo}; mkdir -p $OUT
export TMPDIR=/tmp
V=detrpose_amd/lib/variants
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -k "conv2d" -x -q --timeout 120 --timeout-method thread > $OUT/kern.log 2>&1 || { tail -30 $OUT/kern.log; exit 1; }
tail -1 $OUT/kern.log
timeout -k 10 300 python -u scripts/conv_bench.py --shapes conv3 --rounds 3 --check --libs detrpose_amd/lib/libdetrpose_hip.so${2} > $OUT/cb.txt 2>&1 || { tail -30 $OUT/cb.txt; exit 1; }
cat $OUT/cb.txt
timeout -k 10 300 python -u -m pytest tests/test_gpu_model.py -x -q --timeout 200 --timeout-method thread > $OUT/model.log 2>&1 || { tail -30 $OUT/model.log; exit 1; }
tail -1 $OUT/model.log
timeout -k 10 200 python -u bench.py --steps 50 --warmup 10 --no-cpu-baseline --no-latency --no-secondary --profile-ops $OUT/ops.json > $OUT/bench.json 2> $OUT/bench.err || { tail -20 $OUT/bench.err; exit 1; }
python -c "import json; d=json.load(open('$OUT/bench.json')); print(d['value'], d['roofline']['frac'], d['kernel_ms_per_step'])"
