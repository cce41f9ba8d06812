#!/bin/bash
# Depthwise backward: tests, then the L b16 training tapes' dw_bwd family with the 4-channel
# vector kernels (default) and the scalar ones (DETRPOSE_DW_BWD_VEC=0).
OUT=${1:-gpurun_out/dwbwd}
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_encoder_train_ops.py -m gpu -q -k depthwise --timeout 200 --timeout-method thread > $OUT/pytest.log 2>&1
tail -1 $OUT/pytest.log
for v in 1 0; do
  DETRPOSE_DW_BWD_VEC=$v timeout -k 10 300 python -u scripts/train_prof.py --accum 1 --out $OUT/ops_vec$v.json > $OUT/prof_vec$v.log 2>&1 || { tail -5 $OUT/prof_vec$v.log; exit 1; }
done
python - $OUT <<'PY'
import json, sys
o = sys.argv[1]
for v in (1, 0):
    d = json.load(open(f"{o}/ops_vec{v}.json"))
    fam = {}
    for t in d["tapes"].values():
        for ms, f in t["top_families"]:
            if "dw_bwd" in f:
                fam[f] = ms
    print("vec", v, "step_ms", d["step_ms"], fam)
PY
