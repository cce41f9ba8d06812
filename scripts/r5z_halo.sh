#!/bin/bash
# conv_halo NR-deep weight-ring variants vs production on the 128-channel 3x3 shapes (outputs checked)
mkdir -p gpurun_out/r5z
timeout -k 10 300 python -u scripts/conv_bench.py --shapes conv3 --only fpn --rounds 3 --no-blas --check \
  --libs detrpose_amd/lib/libdetrpose_hip.so,detrpose_amd/lib/variants/nr3/libdetrpose_hip.so,detrpose_amd/lib/variants/nr4/libdetrpose_hip.so \
  > gpurun_out/r5z/cb.txt 2>&1; tail -20 gpurun_out/r5z/cb.txt
