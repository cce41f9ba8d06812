"""dp_mha_layernorm at DETRPose-L b64 inference shapes (within: 3840 sequences of 18 rows;
across: 1152 sequences of 60 rows with the pos re-add and the fused 288-output next Linear):
HIP-event time per launch, and with a library built with -DDP_MHA_TIMING the per-block phase
times (wave 0's wall-clock stamps).

    python scripts/mha_bench.py [--stamps]
"""
import ctypes as C
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

PHASES = ["x load", "V gemm", "K gemm", "Q gemm", "barrier", "attention", "residual+barrier", "out gemm", "layernorm",
          "store", "next linear"]


def main():
    from detrpose_amd import _lib
    from detrpose_amd._lib import contiguous_rows
    from detrpose_amd.fragments import frag_pack
    lib = _lib.load()
    stamps = "--stamps" in sys.argv
    s = C.c_void_p(torch.cuda.current_stream().cuda_stream)
    g = torch.Generator().manual_seed(0)
    c, nh, T, nq, B, nn_ = 256, 8, 18, 60, 64, 288
    rows = B * nq * T

    def bf(*shape, scale=1.0):
        return (torch.randn(*shape, generator=g) * scale).bfloat16()

    x = bf(rows, c).cuda()
    wqkv, wo, wn = frag_pack(bf(3 * c, c, scale=c ** -0.5)).cuda(), frag_pack(bf(c, c, scale=c ** -0.5)).cuda(), \
        frag_pack(bf(nn_, c, scale=c ** -0.5)).cuda()
    bqkv, bo, bn = (torch.randn(n, generator=g).cuda() * 0.1 for n in (3 * c, c, nn_))
    gamma, beta = (1 + 0.1 * torch.randn(c, generator=g)).cuda(), (0.1 * torch.randn(c, generator=g)).cuda()
    pos = bf(rows // T * (T - 1), c).cuda()
    out = torch.zeros(rows, 2 * c, dtype=torch.bfloat16, device="cuda")
    nout = torch.zeros(rows, nn_, dtype=torch.bfloat16, device="cuda")
    res = {}
    for mode in ("within", "across"):
        if mode == "within":
            geo, post, nxt = (B * nq, 1, T, 0, 1, T), None, None
        else:
            geo, post, nxt = (B, T, nq * T, 1, T, nq), pos, nout

        def run():
            _lib.check(lib.dp_mha_layernorm(out.data_ptr(), contiguous_rows(2 * c), x.data_ptr(), contiguous_rows(c),
                                            *geo, wqkv.data_ptr(), bqkv.data_ptr(), wo.data_ptr(), bo.data_ptr(),
                                            gamma.data_ptr(), beta.data_ptr(), C.c_float(1e-5), c, nh,
                                            post.data_ptr() if post is not None else None, contiguous_rows(c), T, 1,
                                            nxt.data_ptr() if nxt is not None else None, nn_,
                                            wn.data_ptr() if nxt is not None else None,
                                            bn.data_ptr() if nxt is not None else None, nn_ if nxt is not None else 0,
                                            s), "dp_mha_layernorm")
        for _ in range(5):
            run()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        n = 50
        e0.record()
        for _ in range(n):
            run()
        e1.record()
        torch.cuda.synchronize()
        r = {"us_per_launch": round(e0.elapsed_time(e1) * 1e3 / n, 2)}
        if stamps:
            run()
            torch.cuda.synchronize()
            nblk = B * nq // 4 if mode == "within" else B * T
            buf = np.zeros(8192 * 12, dtype=np.int64)
            lib.dp_debug_mha_stamps.argtypes = [C.c_void_p, C.c_int32]
            assert lib.dp_debug_mha_stamps(buf.ctypes.data, buf.size) == 0
            st = buf.reshape(8192, 12)[:nblk].astype(np.float64)
            seq = np.concatenate([st[:, 11:12], st[:, :11]], 1)
            ph = np.diff(seq, axis=1) * 10e-3
            t0 = seq[:, 0].min()
            r["phases"] = {PHASES[k]: [round(float(ph[:, k].mean()), 2), round(float(ph[:, k].max()), 2)]
                           for k in range(ph.shape[1])}
            r["block_us_mean"] = round(float((seq[:, -1] - seq[:, 0]).mean() * 10e-3), 2)
            r["span_us"] = round(float((seq[:, -1].max() - t0) * 10e-3), 2)
            r["start_spread_us"] = np.percentile((seq[:, 0] - t0) * 10e-3, [0, 25, 50, 75, 100]).round(1).tolist()
        res[mode] = r
    print(json.dumps(res))


if __name__ == "__main__":
    main()
