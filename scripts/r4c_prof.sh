# rocprofv3 kernel stats of a short bench run with the row-band conv kernel on / off
set -e
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_band -o run -- python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-latency --no-secondary --no-train > gpurun_out/prof_band.log 2>&1
DETRPOSE_NO_BAND=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_halo -o run -- python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-latency --no-secondary --no-train > gpurun_out/prof_halo.log 2>&1
