#!/bin/bash
# Isolates a non-finite training step (bench train leg inputs) between the MSDA backward variant
# and hipGraph replay, then runs the graph-vs-eager test.
mkdir -p gpurun_out/r5y
for cfg in "sorted 1" "atomic 1" "sorted 0"; do
  set -- $cfg
  DETRPOSE_MSDA_BWD=$1 DETRPOSE_TRAIN_GRAPHS=$2 timeout -k 10 200 python -u scripts/train_nan_probe.py --steps 6 > gpurun_out/r5y/probe_$1_$2.log 2>&1 || { tail -5 gpurun_out/r5y/probe_$1_$2.log; exit 1; }
  grep step gpurun_out/r5y/probe_$1_$2.log
done
timeout -k 10 400 python -u -m pytest tests/test_gpu_train_graphs.py -m gpu -v -s --timeout 300 --timeout-method thread > gpurun_out/r5y/pytest.log 2>&1
tail -3 gpurun_out/r5y/pytest.log; grep -E "max rel|graph - eager|replayed" gpurun_out/r5y/pytest.log
timeout -k 10 300 python -u -m pytest tests/test_msda_train.py -m gpu -q --timeout 200 --timeout-method thread > gpurun_out/r5y/pytest_msda.log 2>&1; tail -1 gpurun_out/r5y/pytest_msda.log
bash scripts/ab_msda_sorted.sh gpurun_out/r5y/ab
