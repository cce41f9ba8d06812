mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 240 --timeout-method thread tests/test_gpu_kernels.py -k "conv2d or stem or dwconv" > gpurun_out/r4c_conv.txt 2>&1 && \
timeout -k 10 300 python -u scripts/conv_bench.py --libs detrpose_amd/lib/variants/head/libdetrpose_hip.so,detrpose_amd/lib/libdetrpose_hip.so --shapes conv3 --rounds 5 --check > gpurun_out/r4c_convab.txt 2>&1 && \
timeout -k 10 300 python -u bench.py --steps 100 --no-cpu-baseline --no-latency --no-secondary --no-train --profile-ops gpurun_out/r4c_ops.json > gpurun_out/r4c_bench.txt 2>&1
