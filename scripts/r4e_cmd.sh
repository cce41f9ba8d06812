mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -v --timeout 240 --timeout-method thread tests/test_gpu_encoder_train_ops.py tests/test_gpu_train_ops.py tests/test_msda_train.py -s > gpurun_out/r4e_ops.txt 2>&1
