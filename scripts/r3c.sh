set -o pipefail
mkdir -p gpurun_out/r3c
timeout -k 10 300 python -u -m pytest tests/test_gpu_decoder.py tests/test_gpu_model.py -x -v -s --timeout 200 --timeout-method thread > gpurun_out/r3c/pytest.log 2>&1
rc=$?
tail -5 gpurun_out/r3c/pytest.log
[ $rc -ne 0 ] && { grep -E "FAIL|Error|error" gpurun_out/r3c/pytest.log | head -20; exit $rc; }
timeout -k 10 300 python -u bench.py --steps 50 --warmup 10 --no-cpu-baseline --no-latency --no-secondary --profile-ops gpurun_out/r3c/ops.json > gpurun_out/r3c/bench.json 2> gpurun_out/r3c/bench.err || { tail -20 gpurun_out/r3c/bench.err; exit 1; }
cat gpurun_out/r3c/bench.json
