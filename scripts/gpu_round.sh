#!/bin/bash
# One GPU-box pass: parity tests, bench line, rocprofv3 kernel stats, PMC passes
# (FETCH_SIZE, WRITE_SIZE, and an SQ pass: MFMA busy / LDS bank conflicts / wait states).
#   gpurun --timeout 1200 -- bash scripts/gpu_round.sh [tag]
# env: SKIP_TESTS=1, SKIP_PMC=1, TESTS="tests/x.py" (default: tests -m gpu)
# Every GPU step has its own time limit; steps are chained so the first failure ends the run.
set -e -o pipefail
TAG=${1:-r2}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
SKIP_TESTS=${SKIP_TESTS:-0}
TESTS=${TESTS:-tests}
if [ "$SKIP_TESTS" != 1 ]; then
  timeout -k 10 900 python -u -m pytest $TESTS -m gpu -x -v -s --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 \
    || { tail -40 $OUT/pytest_gpu.log; exit 1; }
  tail -3 $OUT/pytest_gpu.log
fi
timeout -k 10 400 python -u bench.py > $OUT/bench.json 2> $OUT/bench.err || { tail -20 $OUT/bench.err; exit 1; }
cat $OUT/bench.json
PB="--steps 10 --warmup 3 --no-cpu-baseline --no-latency --no-secondary --no-train --no-gemm-peak"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- \
  python3 bench.py $PB --profile-ops $OUT/ops.json > $OUT/prof_bench.json 2> $OUT/prof.err \
  || { tail -20 $OUT/prof.err; exit 1; }
if [ "${SKIP_PMC:-0}" != 1 ]; then
  PP="--steps 2 --warmup 1 --no-cpu-baseline --no-latency --no-secondary --no-train --no-gemm-peak"
  timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d $OUT/pmc_fetch -o run --output-format csv -- \
    python3 bench.py $PP > /dev/null 2> $OUT/pmc_fetch.err
  timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d $OUT/pmc_write -o run --output-format csv -- \
    python3 bench.py $PP > /dev/null 2> $OUT/pmc_write.err
  timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY \
    SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE \
    -d $OUT/pmc_sq -o run --output-format csv -- python3 bench.py $PP > /dev/null 2> $OUT/pmc_sq.err
fi
find $OUT -name '*.csv' | head -20
echo done
