#!/bin/bash
# Round-6 closing pass, part 1: the whole GPU suite and smoke() at HEAD.
set -o pipefail
OUT=gpurun_out/${1:-r6z}; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v -s --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 \
  || { tail -40 $OUT/pytest_gpu.log; exit 1; }
tail -3 $OUT/pytest_gpu.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { tail -20 $OUT/smoke.log; exit 1; }
tail -3 $OUT/smoke.log
