#!/bin/bash
# MSDA sorted backward (tests, A/B, sort-kernel phase timing), hipGraph training tapes, halo NR4 conv tests
mkdir -p gpurun_out/r5y4
timeout -k 10 300 python -u -m pytest tests/test_msda_train.py -m gpu -q --timeout 200 --timeout-method thread > gpurun_out/r5y4/pytest_msda.log 2>&1; tail -1 gpurun_out/r5y4/pytest_msda.log
bash scripts/ab_msda_sorted.sh gpurun_out/r5y4/ab
DETRPOSE_HIP_LIB=$PWD/detrpose_amd/lib/variants/kst/libdetrpose_hip.so DETRPOSE_ALLOW_STALE_LIB=1 timeout -k 10 120 python scripts/msda_ks_timing.py > gpurun_out/r5y4/ks_timing.json 2>&1; tail -1 gpurun_out/r5y4/ks_timing.json
timeout -k 10 400 python -u -m pytest tests/test_gpu_train_graphs.py tests/test_gpu_kernels.py -k "graph or conv2d" -m gpu -v -s --timeout 300 --timeout-method thread > gpurun_out/r5y4/pytest.log 2>&1
tail -2 gpurun_out/r5y4/pytest.log; grep -E "graph - eager|replayed|FAIL" gpurun_out/r5y4/pytest.log | head -20
