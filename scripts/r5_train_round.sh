#!/bin/bash
# Training-leg measurements (round 5): bench train leg (config default, grad_accum 2), per-op
# tape profile at b16 accum 1 (comparable with r4m_train_ops.json), rocprofv3 kernel stats of the
# training step, and the 2-rank shared-GPU rehearsal of the world-aware train leg.
#   gpurun --timeout 1200 -- bash scripts/r5_train_round.sh TAG
set -e -o pipefail
TAG=${1:-r5t}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
NT="--no-cpu-baseline --no-latency --no-secondary"
timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 $NT > $OUT/bench_train.json 2> $OUT/bench_train.err \
  || { tail -20 $OUT/bench_train.err; exit 1; }
python -c "import json,sys; d=json.load(open('$OUT/bench_train.json')); print(json.dumps(d['train_step']))"
timeout -k 10 300 python -u scripts/train_prof.py --accum 1 --out $OUT/train_ops_b16a1.json > $OUT/train_prof.log 2>&1 \
  || { tail -20 $OUT/train_prof.log; exit 1; }
tail -3 $OUT/train_prof.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof_train -o run --output-format csv -- \
  python3 scripts/train_prof.py --accum 1 --out $OUT/train_ops_prof.json > $OUT/prof_train.log 2>&1 \
  || { tail -20 $OUT/prof_train.log; exit 1; }
timeout -k 10 400 python -u bench.py --gpus 2 --shared-gpu-rehearsal --batch 8 --steps 5 --warmup 2 $NT \
  --train-batch 4 --train-steps 3 > $OUT/rehearsal2.json 2> $OUT/rehearsal2.err || { tail -20 $OUT/rehearsal2.err; exit 1; }
python -c "import json; l=[x for x in open('$OUT/rehearsal2.json') if x.startswith('{')][-1]; print(json.dumps(json.loads(l)['train_step']))"
find $OUT -name '*stats.csv' | head
echo done
