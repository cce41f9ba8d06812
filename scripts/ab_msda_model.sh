#!/bin/bash
# In-model MSDA A/B: bench.py per-op profile of the production library and each variant
# library (DETRPOSE_HIP_LIB), printing the six decoder layers' dp_msda times.
#   bash scripts/ab_msda_model.sh <tag> <variant name>...   (libs under detrpose_amd/lib/variants/)
set -o pipefail
OUT=gpurun_out/${1:-abmsda}; shift; mkdir -p $OUT
export TMPDIR=/tmp
for rnd in 1 2; do
for v in prod "$@"; do
  if [ $v = prod ]; then LIBP=detrpose_amd/lib/libdetrpose_hip.so; else LIBP=detrpose_amd/lib/variants/$v/libdetrpose_hip.so; fi
  DETRPOSE_HIP_LIB=$LIBP timeout -k 10 200 python -u bench.py --steps 30 --warmup 5 --no-cpu-baseline --no-latency \
    --no-secondary --profile-ops $OUT/ops_${v}_$rnd.json > $OUT/bench_${v}_$rnd.json 2> $OUT/bench_${v}_$rnd.err \
    || { tail -20 $OUT/bench_${v}_$rnd.err; exit 1; }
  python -c "
import json; d=json.load(open('$OUT/ops_${v}_$rnd.json'))['op_ms']; b=json.load(open('$OUT/bench_${v}_$rnd.json'))
m=[d['dec%d.msda'%i] for i in range(6)]
print('$v r$rnd', 'img/s %.0f'%b['value'], 'msda sum %.3f ms'%sum(m), ' '.join('%.1f'%(1e3*x) for x in m))"
done
done
