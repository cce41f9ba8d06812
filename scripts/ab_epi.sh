set -o pipefail
mkdir -p gpurun_out/abl2; export TMPDIR=/tmp
V=detrpose_amd/lib/variants
timeout -k 10 300 python -u scripts/conv_bench.py --shapes conv3 --only fpn,s1.l --rounds 3 --libs detrpose_amd/lib/libdetrpose_hip.so,$V/habl4/libdetrpose_hip.so,$V/habl8/libdetrpose_hip.so,$V/habl16/libdetrpose_hip.so,$V/habl24/libdetrpose_hip.so > gpurun_out/abl2/cb3.txt 2>&1 && cat gpurun_out/abl2/cb3.txt &&
timeout -k 10 300 python -u scripts/conv_bench.py --shapes gemm --rounds 3 --no-blas --libs detrpose_amd/lib/libdetrpose_hip.so,$V/snost/libdetrpose_hip.so > gpurun_out/abl2/cbg.txt 2>&1 && cat gpurun_out/abl2/cbg.txt
