# full default bench (incl. the training-step leg) + rocprofv3 kernel stats of a short run
set -e
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python3 -u bench.py > gpurun_out/r4d_bench.txt 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r4d_prof -o run -- python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-latency --no-secondary --train-steps 5 > gpurun_out/r4d_prof.log 2>&1
