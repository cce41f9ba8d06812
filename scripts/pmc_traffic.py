"""Per-forward HBM traffic by kernel family from two rocprofv3 --pmc passes
(FETCH_SIZE and WRITE_SIZE, KB per dispatch). gfx950 correction (MI355X_MICROARCH.md
§HBM): FETCH_SIZE counts half the bytes of 16-byte-per-lane streaming reads, so reads
are doubled; WRITE_SIZE is exact for 16-byte stores.

    python scripts/pmc_traffic.py <fetch counter_collection.csv> <write ...csv> [out.json]
"""
import collections
import csv
import json
import os
import re
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def family(name):
    # every implicit-GEMM conv variant (conv_stream/halo/gemm_kernel) is one family
    if re.search(r"conv_(stream|halo|gemm)_kernel", name):
        return "conv"
    # stem register-direct kernel: the plain instantiations are dp_conv2d launches (stem2b, stem4),
    # the POOL one is dp_conv2d_pool (stem2a + max-pool)
    m = re.search(r"conv_direct_kernel(?:ILi\d+ELi\d+ELi\d+ELb([01])E|<\d+, \d+, \d+, (true|false))", name)
    if m:
        return "conv2x2_pool" if (m.group(1) == "1" or m.group(2) == "true") else "conv"
    for key in ("dwconv_kernel", "dwconv_lds_kernel", "layernorm_kernel", "attn_mfma_kernel", "attn_short_kernel",
                "msda_kernel", "msda_wave_kernel", "add_rows_kernel", "stem_conv_kernel", "stem1_mfma_kernel",
                "maxpool_kernel", "class_max_kernel",
                "topk_kernel", "gate_ln_kernel", "sine_embed_kernel", "lqe_kernel", "pose_refine_kernel",
                "linear_ln_kernel", "ffn_ln_kernel", "query_pos_kernel", "pose_mlp_kernel", "ln_classmax_kernel",
                "mha_ln_kernel", "linear_ln_cls_kernel", "attn_long_kernel", "stem_fused_kernel", "dwconv_tile_kernel",
                "linear_small_kernel", "gate_ln_kernel"):
        if key in name:
            return key
    return "other"


def agg(path, counter, key=family):
    tot = collections.defaultdict(float)
    calls = collections.Counter()
    for r in csv.DictReader(open(path)):
        if r["Counter_Name"] != counter:
            continue
        f = key(r["Kernel_Name"])
        tot[f] += float(r["Counter_Value"]) * 1024.0
        calls[f] += 1
    return tot, calls


def main():
    fetch, calls = agg(sys.argv[1], "FETCH_SIZE")
    write, _ = agg(sys.argv[2], "WRITE_SIZE")
    nfwd = calls["topk_kernel"]
    from detrpose_amd.build import source_hash
    out = {"forwards_profiled": nfwd, "source_hash": source_hash(), "workload": ["l", 64, "bf16"], "families": {}}
    for f in sorted(fetch, key=lambda k: -fetch[k]):
        rd = 2.0 * fetch[f] / nfwd
        wr = write.get(f, 0.0) / nfwd
        out["families"][f] = {"read_bytes_corrected": rd, "write_bytes": wr, "total_bytes": rd + wr,
                              "launches": calls[f] / nfwd}
        print(f"{f:22s} read {rd / 1e9:7.3f} GB  write {wr / 1e9:7.3f} GB  per forward ({calls[f] / nfwd:.0f} launches)")
    # per kernel instantiation (canonical rocprofv3 name, detrpose_amd.profiling): bench.py quotes
    # the dominant kernel's measured traffic from here
    from detrpose_amd.profiling import canonical_kernel_name
    kf, kc = agg(sys.argv[1], "FETCH_SIZE", canonical_kernel_name)
    kw, _ = agg(sys.argv[2], "WRITE_SIZE", canonical_kernel_name)
    out["kernels"] = {k: {"read_bytes_corrected": 2.0 * kf[k] / nfwd, "write_bytes": kw.get(k, 0.0) / nfwd,
                          "total_bytes": (2.0 * kf[k] + kw.get(k, 0.0)) / nfwd, "launches": kc[k] / nfwd}
                      for k in sorted(kf, key=lambda k: -kf[k])}
    if len(sys.argv) > 3:
        with open(sys.argv[3], "w") as fh:
            json.dump(out, fh, indent=1)


if __name__ == "__main__":
    main()
