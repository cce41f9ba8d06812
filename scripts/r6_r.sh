#!/bin/bash
# Round 6: enc_output + LN + class-max row tile (DP_ENC_BM) 64 (production) vs 96 / 128: per-op
# times of the L b64 inference plan with each library (bench --profile-ops).
set -o pipefail
OUT=gpurun_out/${1:-r6r}; mkdir -p $OUT
export TMPDIR=/tmp
NT="--steps 20 --warmup 5 --no-cpu-baseline --no-latency --no-secondary --no-gemm-peak --no-train"
timeout -k 10 240 python -u bench.py $NT --profile-ops $OUT/ops_64.json > $OUT/b64.json 2> $OUT/b64.err || { tail -20 $OUT/b64.err; exit 1; }
for B in 96 128; do
  DETRPOSE_ALLOW_STALE_LIB=1 DETRPOSE_HIP_LIB=detrpose_amd/lib/variants/enc$B/libdetrpose_hip.so timeout -k 10 240 python -u bench.py $NT --profile-ops $OUT/ops_$B.json > $OUT/b$B.json 2> $OUT/b$B.err || { tail -20 $OUT/b$B.err; exit 1; }
done
for B in 64 96 128; do python -c "import json; d=json.load(open('$OUT/ops_$B.json'))['op_ms']; b=json.load(open('$OUT/b$B.json')); print('$B', round(d['ts.enc_out_ln']*1000,1), 'us', b['value'], b['ms_per_step'])"; done
