#!/bin/bash
# Per-op times of the L b64 inference step with and without the halo conv kernel (every 3x3
# conv on conv_stream's implicit GEMM instead): the per-shape rule for dp_conv2d_halo.
OUT=${1:-gpurun_out/nohalo}
mkdir -p $OUT
PB="--steps 10 --warmup 3 --no-cpu-baseline --no-latency --no-secondary --no-train"
timeout -k 10 300 python -u bench.py $PB --profile-ops $OUT/ops_halo.json > $OUT/halo.json 2> $OUT/halo.err || { tail -5 $OUT/halo.err; exit 1; }
DETRPOSE_NO_HALO=1 timeout -k 10 300 python -u bench.py $PB --profile-ops $OUT/ops_nohalo.json > $OUT/nohalo.json 2> $OUT/nohalo.err || { tail -5 $OUT/nohalo.err; exit 1; }
python - $OUT <<'PY'
import json, sys
o = sys.argv[1]
a, b = json.load(open(o + "/ops_halo.json")), json.load(open(o + "/ops_nohalo.json"))
for k, v in a["op_ms"].items():
    if "conv_halo" in a["op_kernel"].get(k, ""):
        w = b["op_ms"].get(k, float("nan"))
        print(f"{k:22s} halo {v*1e3:7.1f}us  stream {w*1e3:7.1f}us  {b['op_kernel'].get(k,'')[:50]}")
for f in ("halo", "nohalo"):
    l = [x for x in open(f"{o}/{f}.json") if x.startswith("{")][-1]
    print(f, json.loads(l)["value"], "img/s")
PY
