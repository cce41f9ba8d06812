"""The row-block fused decoder kernels (csrc/decoder.hip) against plain PyTorch fp32 on
the same bf16-rounded inputs and weights (weights passed in the MFMA-fragment layout,
detrpose_amd.fragments.frag_pack): out_proj + residual + LayerNorm (+ pos re-add),
the Gate with its Linear, the FFN + LayerNorm (also in place), the query-pos MLP with the
in-place pos add, and the pose MLP (with the previous corners). Row counts are not
multiples of the 64-row block, so the tail block is exercised too.

Tolerance: the references round where the kernels store bf16 (inputs, weights, the MLP hidden
layers, Q / K / V, the attention probabilities, O), so what remains is f32 summation order and
the one rounding of the output (or, for the f32-output pose corners, a hidden element whose f32
accumulation rounded the other way): one bf16 ulp of the output scale, i.e. 2^-7 times the
power of two at or below max(1, max|ref|).
"""
import ctypes as C
import math

import pytest
import torch
import torch.nn.functional as F

from detrpose_amd import _lib
from detrpose_amd._lib import contiguous_rows, rowmap
from detrpose_amd.fragments import frag_pack

pytestmark = pytest.mark.gpu

def _check(got, ref, what):
    scale = max(1.0, ref.abs().max().item())
    ulp = 2.0 ** (math.floor(math.log2(scale)) - 7)   # one bf16 ulp at the output scale
    err = (got - ref).abs().max().item()
    print(f"{what}: max err {err:.3g} = {err / ulp:.3g} bf16 ulp of scale {scale:.3g}")
    assert err <= ulp, f"{what}: max err {err:.3g} > 1 bf16 ulp {ulp:.3g} (scale {scale:.3g})"


def _bf(*shape, scale=1.0, g=None):
    return (torch.randn(*shape, generator=g) * scale).bfloat16()


def _s():
    return C.c_void_p(torch.cuda.current_stream().cuda_stream)


def _ln(x, gamma, beta):
    return F.layer_norm(x, (x.shape[-1],), gamma, beta, 1e-5)


@pytest.mark.parametrize("c", [128, 256, 384])
@pytest.mark.parametrize("post", [False, True])
def test_linear_layernorm(c, post):
    g = torch.Generator().manual_seed(c + post)
    T, rows = 18, 18 * 61   # 1098 rows: 17 full blocks + a tail
    x, res = _bf(rows, c, g=g), _bf(rows, c, g=g)
    w = _bf(c, c, scale=c ** -0.5, g=g)
    b, gamma, beta = torch.randn(c, generator=g) * 0.1, 1 + 0.1 * torch.randn(c, generator=g), 0.1 * torch.randn(c, generator=g)
    krows = rows // T * (T - 1)
    pos = _bf(krows, c, g=g)
    ld = 2 * c   # written into the first half of a wider row, as the decoder does
    out = torch.zeros(rows, ld, dtype=torch.bfloat16, device="cuda")
    dx, dres, dw, dpos = x.cuda(), res.cuda(), frag_pack(w).cuda(), pos.cuda()
    db, dg, dbe = b.cuda(), gamma.cuda(), beta.cuda()
    lib = _lib.load()
    _lib.check(lib.dp_linear_layernorm(out.data_ptr(), contiguous_rows(ld), dx.data_ptr(), contiguous_rows(c), c,
                                       dw.data_ptr(), db.data_ptr(), dres.data_ptr(), contiguous_rows(c),
                                       dg.data_ptr(), dbe.data_ptr(), C.c_float(1e-5), rows, c,
                                       dpos.data_ptr() if post else None, contiguous_rows(c), T, 1, _s()))
    torch.cuda.synchronize()
    ref = _ln(x.float() @ w.float().t() + b + res.float(), gamma, beta)
    if post:
        ref = ref.reshape(rows // T, T, c)
        ref[:, 1:] += pos.float().reshape(rows // T, T - 1, c)
        ref = ref.reshape(rows, c)
    got = out[:, :c].float().cpu()
    _check(got, ref, f"linear_layernorm c{c} post{post}")
    assert (out[:, c:] == 0).all()


@pytest.mark.parametrize("c", [128, 256, 384])
def test_gate_linear_layernorm(c):
    g = torch.Generator().manual_seed(7 + c)
    rows = 1000
    x = _bf(rows, 2 * c, g=g)
    w = _bf(2 * c, 2 * c, scale=(2 * c) ** -0.5, g=g)
    b, gamma, beta = torch.randn(2 * c, generator=g) * 0.1, 1 + 0.1 * torch.randn(c, generator=g), 0.1 * torch.randn(c, generator=g)
    out = torch.empty(rows, c, dtype=torch.bfloat16, device="cuda")
    dx, dw, db, dg, dbe = x.cuda(), frag_pack(w).cuda(), b.cuda(), gamma.cuda(), beta.cuda()
    lib = _lib.load()
    _lib.check(lib.dp_gate_linear_layernorm(out.data_ptr(), contiguous_rows(c), dx.data_ptr(), contiguous_rows(2 * c),
                                            dw.data_ptr(), db.data_ptr(), dg.data_ptr(), dbe.data_ptr(),
                                            C.c_float(1e-5), rows, c, _s()))
    torch.cuda.synchronize()
    xf = x.float()
    gates = torch.sigmoid(xf @ w.float().t() + b)
    ref = _ln(gates[:, :c] * xf[:, :c] + gates[:, c:] * xf[:, c:], gamma, beta)
    _check(out.float().cpu(), ref, f"gate c{c}")


@pytest.mark.parametrize("c,f", [(128, 512), (256, 1024), (384, 1024), (384, 2048)])
def test_ffn_layernorm_in_place(c, f):
    g = torch.Generator().manual_seed(c + f)
    rows = 1000
    x = _bf(rows, c, g=g)
    w1, w2 = _bf(f, c, scale=c ** -0.5, g=g), _bf(c, f, scale=f ** -0.5, g=g)
    b1, b2 = 0.1 * torch.randn(f, generator=g), 0.1 * torch.randn(c, generator=g)
    gamma, beta = 1 + 0.1 * torch.randn(c, generator=g), 0.1 * torch.randn(c, generator=g)
    dx = x.cuda()
    d = [t.cuda() for t in (frag_pack(w1), b1, frag_pack(w2), b2, gamma, beta)]   # kept alive across the launch
    lib = _lib.load()
    _lib.check(lib.dp_ffn_layernorm(dx.data_ptr(), contiguous_rows(c), dx.data_ptr(), contiguous_rows(c),
                                    d[0].data_ptr(), d[1].data_ptr(), f, d[2].data_ptr(), d[3].data_ptr(),
                                    d[4].data_ptr(), d[5].data_ptr(), C.c_float(1e-5), rows, c, _s()))
    torch.cuda.synchronize()
    h = torch.relu(x.float() @ w1.float().t() + b1).bfloat16().float()   # the hidden layer is a bf16 operand
    ref = _ln(x.float() + h @ w2.float().t() + b2, gamma, beta)
    _check(dx.float().cpu(), ref, f"ffn c{c} f{f}")


def _sine(ref_kp, dim_t):
    """TransformerDecoder.sine_embedding (transformer.py:518-540), the oracle's restatement."""
    from oracle.detrpose_cpu import sine_embedding
    return sine_embedding(ref_kp, dim_t)


@pytest.mark.parametrize("c", [128, 256, 384])
def test_query_pos(c):
    g = torch.Generator().manual_seed(11 + c)
    nq_rows, K, T = 61, 17, 18
    krows = nq_rows * K
    ref = torch.rand(nq_rows, T, 2, generator=g)
    dim_t = 10000 ** (2 * (torch.arange(c // 2) // 2) / (c // 2)).float()
    w0, w1 = _bf(c, c, scale=c ** -0.5, g=g), _bf(c, c, scale=c ** -0.5, g=g)
    b0, b1 = 0.1 * torch.randn(c, generator=g), 0.1 * torch.randn(c, generator=g)
    tgt = _bf(nq_rows * T, c, g=g)
    dtgt = tgt.cuda()
    pos = torch.empty(krows, c, dtype=torch.bfloat16, device="cuda")
    d = [t.cuda() for t in (ref, dim_t, frag_pack(w0), b0, frag_pack(w1), b1)]   # kept alive across the launch
    lib = _lib.load()
    _lib.check(lib.dp_query_pos(d[0].data_ptr(), krows, K, d[1].data_ptr(), d[2].data_ptr(), d[3].data_ptr(),
                                d[4].data_ptr(), d[5].data_ptr(), pos.data_ptr(), dtgt.data_ptr(),
                                rowmap(c, K, T * c, c), c, _s()))
    torch.cuda.synchronize()
    se = _sine(ref[None, :, 1:], dim_t).reshape(krows, c).bfloat16().float()
    h = torch.relu(se @ w0.float().t() + b0).bfloat16().float()
    p_ref = h @ w1.float().t() + b1
    _check(pos.float().cpu(), p_ref, f"query_pos c{c}")
    t_ref = tgt.float().reshape(nq_rows, T, c).clone()
    t_ref[:, 1:] += pos.float().cpu().reshape(nq_rows, K, c)
    got = dtgt.float().cpu().reshape(nq_rows, T, c)
    assert (got[:, 0] == tgt.float().reshape(nq_rows, T, c)[:, 0]).all()   # instance rows untouched
    _check(got, t_ref, f"query_pos tgt += pos c{c}")


@pytest.mark.parametrize("c", [128, 256, 384])
@pytest.mark.parametrize("add", [False, True])
def test_pose_mlp(c, add):
    g = torch.Generator().manual_seed(13 + c + add)
    nq_rows, K, T, nout = 61, 17, 18, 66
    krows = nq_rows * K
    a, b = _bf(nq_rows * T, c, g=g), _bf(nq_rows * T, c, g=g)
    w0, w1 = _bf(c, c, scale=c ** -0.5, g=g), _bf(c, c, scale=c ** -0.5, g=g)
    w2 = _bf(nout, c, scale=c ** -0.5, g=g)
    b0, b1, b2 = (0.1 * torch.randn(n, generator=g) for n in (c, c, nout))
    prev = torch.randn(krows, nout, generator=g)
    out = torch.empty(krows, nout, device="cuda")
    kp = rowmap(c, K, T * c, c)
    da, db_ = a.cuda(), b.cuda()
    d = [t.cuda() for t in (frag_pack(w0), b0, frag_pack(w1), b1, frag_pack(w2), b2, prev)]   # kept alive
    lib = _lib.load()
    _lib.check(lib.dp_pose_mlp(da.data_ptr(), kp, db_.data_ptr() if add else None, kp, krows, d[0].data_ptr(),
                               d[1].data_ptr(), d[2].data_ptr(), d[3].data_ptr(), d[4].data_ptr(), d[5].data_ptr(),
                               nout, d[6].data_ptr() if add else None, out.data_ptr(), c, _s()))
    torch.cuda.synchronize()
    x = a.float().reshape(nq_rows, T, c)[:, 1:]
    if add:
        x = (x + b.float().reshape(nq_rows, T, c)[:, 1:]).bfloat16().float()
    x = x.reshape(krows, c)
    h1 = torch.relu(x @ w0.float().t() + b0).bfloat16().float()
    h2 = torch.relu(h1 @ w1.float().t() + b1).bfloat16().float()
    ref = h2 @ w2.float().t() + b2 + (prev if add else 0)
    _check(out.cpu(), ref, f"pose_mlp c{c} add{add}")


def _mha_ref(x, wqkv, bqkv, wo, bo, nhead):
    """nn.MultiheadAttention(q = k = v = x) in fp32 at the kernel's bf16 store points: q, k, v
    (the projection's MFMA fragments / V image), the unnormalised probabilities exp(s - max)
    (the PV MFMA operand; the row sum stays f32) and O (the out_proj input); x: [nseq, L, C]."""
    c = x.shape[-1]
    dh = c // nhead
    qkv = (x @ wqkv.t() + bqkv).bfloat16().float()
    q, k, v = (t.reshape(*x.shape[:2], nhead, dh).transpose(1, 2) for t in qkv.split(c, -1))
    s = q @ k.transpose(-1, -2) / dh ** 0.5
    e = torch.exp(s - s.max(-1, keepdim=True).values)
    o = (e.bfloat16().float() @ v) / e.sum(-1, keepdim=True)
    o = o.transpose(1, 2).reshape(x.shape).bfloat16().float()
    return o @ wo.t() + bo


@pytest.mark.parametrize("mode", ["within", "across", "across_post", "within_tail", "across_post_next"])
def test_mha_layernorm(mode):
    """dp_mha_layernorm (the decoder's within / across token attention + out_proj + residual +
    LN, transformer.py:403-422) against torch fp32 on the same bf16 inputs: within = groups of
    18 contiguous rows; across = the 60 queries of a token slot, rows 18 apart, with and
    without the keypoint-row pos re-add; within_tail: a sequence count that leaves a partial
    last block; across_post_next: plus the fused next Linear (the MSDA offsets / logits
    projection, 288 outputs) on the stored rows."""
    g = torch.Generator().manual_seed(11 + len(mode))
    c, nh, T, nq = 256, 8, 18, 60
    B = 2
    nseq_w = B * nq - (5 if mode == "within_tail" else 0)
    rows = B * nq * T
    x = _bf(rows, c, g=g)
    wqkv = _bf(3 * c, c, scale=c ** -0.5, g=g)
    wo = _bf(c, c, scale=c ** -0.5, g=g)
    bqkv, bo = torch.randn(3 * c, generator=g) * 0.1, torch.randn(c, generator=g) * 0.1
    gamma, beta = 1 + 0.1 * torch.randn(c, generator=g), 0.1 * torch.randn(c, generator=g)
    krows = rows // T * (T - 1)
    pos = _bf(krows, c, g=g)
    post = mode.startswith("across_post")
    nxt = mode.endswith("next")
    nn_ = 288
    wn = _bf(nn_, c, scale=c ** -0.5, g=g)
    bn = torch.randn(nn_, generator=g) * 0.1
    nout = torch.zeros(rows, nn_, dtype=torch.bfloat16, device="cuda")
    dwn, dbn = frag_pack(wn).cuda(), bn.cuda()
    ld = 2 * c
    out = torch.zeros(rows, ld, dtype=torch.bfloat16, device="cuda")
    dx, dpos = x.cuda(), pos.cuda()
    dq, dbq, dwo, dbo, dg, dbe = (t.cuda() for t in (frag_pack(wqkv), bqkv, frag_pack(wo), bo, gamma, beta))
    if mode.startswith("within"):
        geo = (nseq_w, 1, T, 0, 1, T)
    else:
        geo = (B, T, nq * T, 1, T, nq)
    lib = _lib.load()
    _lib.check(lib.dp_mha_layernorm(out.data_ptr(), contiguous_rows(ld), dx.data_ptr(), contiguous_rows(c), *geo,
                                    dq.data_ptr(), dbq.data_ptr(), dwo.data_ptr(), dbo.data_ptr(), dg.data_ptr(),
                                    dbe.data_ptr(), C.c_float(1e-5), c, nh, dpos.data_ptr() if post else None,
                                    contiguous_rows(c), T, 1, nout.data_ptr() if nxt else None, nn_,
                                    dwn.data_ptr() if nxt else None, dbn.data_ptr() if nxt else None,
                                    nn_ if nxt else 0, _s()), "dp_mha_layernorm")
    torch.cuda.synchronize()
    xf = x.float()
    if mode.startswith("within"):
        seqs = xf[:nseq_w * T].reshape(nseq_w, T, c)
        y = _mha_ref(seqs, wqkv.float(), bqkv, wo.float(), bo, nh)
        ref = _ln(seqs + y, gamma, beta).reshape(-1, c)
        got = out[:nseq_w * T, :c].float().cpu()
        assert (out[nseq_w * T:] == 0).all()
    else:
        seqs = xf.reshape(B, nq, T, c).transpose(1, 2).reshape(B * T, nq, c)
        y = _mha_ref(seqs, wqkv.float(), bqkv, wo.float(), bo, nh)
        ref = _ln(seqs + y, gamma, beta).reshape(B, T, nq, c).transpose(1, 2).reshape(rows, c)
        if post:
            ref = ref.reshape(rows // T, T, c)
            ref[:, 1:] += pos.float().reshape(rows // T, T - 1, c)
            ref = ref.reshape(rows, c)
        got = out[:, :c].float().cpu()
    _check(got, ref, f"mha {mode}")
    assert (out[:, c:] == 0).all()
    if nxt:   # the next Linear runs on the STORED rows
        nref = out[:, :c].float().cpu() @ wn.float().t() + bn
        _check(nout.float().cpu(), nref, "mha next linear")


def test_linear_layernorm_classmax():
    """dp_linear_layernorm_classmax (enc_output + enc_output_norm + masked rows + class max,
    transformer.py:1232-1240) against torch fp32 on the same bf16 inputs; rows not a multiple
    of the 128-row block; the class max is taken over the stored bf16 row."""
    g = torch.Generator().manual_seed(5)
    c, ncls, period = 256, 2, 70
    rows = 128 * 9 + 77
    x = _bf(rows, c, g=g)
    w = _bf(c, c, scale=c ** -0.5, g=g)
    b, gamma, beta = torch.randn(c, generator=g) * 0.1, 1 + 0.1 * torch.randn(c, generator=g), 0.1 * torch.randn(c, generator=g)
    mask = (torch.rand(period, generator=g) < 0.2).to(torch.uint8)
    masked_row = torch.randn(c, generator=g)
    cw, cb = torch.randn(ncls, c, generator=g) * 0.1, torch.randn(ncls, generator=g)
    out = torch.empty(rows, c, dtype=torch.bfloat16, device="cuda")
    score = torch.empty(rows, device="cuda")
    dev = [t.cuda() for t in (x, frag_pack(w), b, gamma, beta, mask, masked_row, cw, cb)]
    lib = _lib.load()
    _lib.check(lib.dp_linear_layernorm_classmax(out.data_ptr(), dev[0].data_ptr(), rows, c, dev[1].data_ptr(),
                                                dev[2].data_ptr(), dev[3].data_ptr(), dev[4].data_ptr(),
                                                C.c_float(1e-5), dev[5].data_ptr(), period, dev[6].data_ptr(),
                                                dev[7].data_ptr(), dev[8].data_ptr(), ncls, score.data_ptr(), _s()),
               "dp_linear_layernorm_classmax")
    torch.cuda.synchronize()
    ref = _ln(x.float() @ w.float().t() + b, gamma, beta)
    m = mask.bool()[torch.arange(rows) % period]
    ref[m] = masked_row
    got = out.float().cpu()
    _check(got, ref, "linear_ln_classmax")
    sref = (got @ cw.t() + cb).max(1).values        # class max over the stored rows
    assert (score.cpu() - sref).abs().max().item() <= 1e-4
