#!/bin/bash
# Round 6: weight-stationary enc_output + LN + class-max: decoder tests (incl. the bit-identity of
# the two forms), model parity, bench A/B (DETRPOSE_ENC_WS=0 vs 1, same library, per-op times).
set -o pipefail
OUT=gpurun_out/${1:-r6s}; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_decoder.py tests/test_gpu_model.py -x -q --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
NT="--steps 30 --warmup 5 --no-cpu-baseline --no-latency --no-secondary --no-gemm-peak --no-train"
for WS in 0 1 0 1; do
  DETRPOSE_ENC_WS=$WS timeout -k 10 240 python -u bench.py $NT --profile-ops $OUT/ops_ws$WS.json > $OUT/b_ws$WS.json 2> $OUT/b_ws$WS.err || { tail -20 $OUT/b_ws$WS.err; exit 1; }
  python -c "import json; d=json.load(open('$OUT/ops_ws$WS.json'))['op_ms']; b=json.load(open('$OUT/b_ws$WS.json')); print('ws$WS', round(d['ts.enc_out_ln']*1000,1), 'us', b['value'], b['ms_per_step'])"
done
