"""MSDA core at the training interface (dp_msda_core_fwd / dp_msda_core_bwd).

CPU: the oracle's differentiable restatement (oracle.msda_core, an explicit 4-corner gather)
is pinned to the reference's own op: autograd of F.grid_sample(bilinear, zeros,
align_corners=False) as ms_deform_attn_core_pytorch calls it
(/root/reference/src/models/detrpose/ms_deform_attn.py:145-193), forward AND gradients, on
the reference's MSDA vectors (tests/golden/msda_*.npz, produced by the reference).

GPU: the HIP forward vs the reference's golden outputs, and the HIP backward (grad_value by
f32 atomics, grad_loc, grad_attn) vs autograd of the pinned oracle. Tolerances: f32 1e-4 of
each gradient's scale (atomic summation order differs); bf16 value / grad_out storage rounds
to 8 mantissa bits, checked against the oracle on the same rounded inputs at 2e-2.
"""
import os

import numpy as np
import pytest
import torch
import torch.nn.functional as F

from oracle.detrpose_cpu import msda_core

SIZES = ["n", "l", "x"]


def _vectors(golden_dir, size):
    g = np.load(os.path.join(golden_dir, f"msda_{size}.npz"))
    return {k: torch.from_numpy(g[k]) for k in g.files}


def _grid_sample_core(value, shapes, loc, attn):
    """ms_deform_attn_core_pytorch's default branch over value (N, S, nH*Dh): per level
    F.grid_sample at 2*loc-1, then the attention-weighted sum over (level, point)."""
    N, S, Cc = value.shape
    _, Lq, nH, L, P, _ = loc.shape
    Dh = Cc // nH
    grids = 2 * loc - 1
    out, start = 0, 0
    for l, (h, w) in enumerate(shapes):
        v = value[:, start:start + h * w].reshape(N, h, w, nH, Dh).permute(0, 3, 4, 1, 2).reshape(N * nH, Dh, h, w)
        start += h * w
        g = grids[:, :, :, l].permute(0, 2, 1, 3, 4).reshape(N * nH, Lq, P, 2)
        s = F.grid_sample(v, g, mode="bilinear", padding_mode="zeros", align_corners=False)
        a = attn[:, :, :, l].permute(0, 2, 1, 3).reshape(N * nH, 1, Lq, P)
        out = out + (s * a).sum(-1)
    return out.reshape(N, nH * Dh, Lq).transpose(1, 2)


def _grads(fn, value, shapes, loc, attn, gout):
    v, lc, a = (t.clone().requires_grad_(True) for t in (value, loc, attn))
    out = fn(v, shapes, lc, a)
    out.backward(gout)
    return out.detach(), v.grad, lc.grad, a.grad


def _edge_locs(loc, seed):
    """Spread some points outside [0, 1] (zeros padding, partly-outside corners)."""
    g = torch.Generator().manual_seed(seed)
    loc = loc.clone()
    m = torch.rand(loc.shape[:-1], generator=g) < 0.1
    loc[m] = loc[m] * 1.6 - 0.3
    return loc


@pytest.mark.parametrize("size", SIZES)
def test_oracle_msda_backward_matches_grid_sample(golden_dir, size):
    d = _vectors(golden_dir, size)
    shapes = [tuple(int(v) for v in hw) for hw in d["shapes"]]
    loc = _edge_locs(d["loc"], 1)
    gout = torch.randn(d["out"].shape, generator=torch.Generator().manual_seed(2))
    ref = _grads(_grid_sample_core, d["value"], shapes, loc, d["attn"], gout)
    got = _grads(msda_core, d["value"], shapes, loc, d["attn"], gout)
    assert torch.allclose(_grid_sample_core(d["value"], shapes, d["loc"], d["attn"]), d["out"], atol=1e-5)
    for name, r, o in zip(("out", "grad_value", "grad_loc", "grad_attn"), ref, got):
        err = (r - o).abs().max().item()
        assert err <= 1e-4 * max(1.0, r.abs().max().item()), (name, err)


def test_value_from_levels_layout():
    from detrpose_amd.msda import value_from_levels
    N, nH, Dh, shapes = 2, 4, 8, [(3, 5), (2, 2)]
    value = torch.randn(N, sum(h * w for h, w in shapes), nH * Dh)
    lv, start = [], 0
    for h, w in shapes:   # the reference's per-level (N*nH, Dh, H*W) split of value
        lv.append(value[:, start:start + h * w].reshape(N, h * w, nH, Dh).permute(0, 2, 3, 1).reshape(N * nH, Dh, h * w))
        start += h * w
    assert torch.equal(value_from_levels(lv, nH), value)


@pytest.mark.gpu
@pytest.mark.parametrize("size", SIZES)
@pytest.mark.parametrize("dt", ["fp32", "bf16"])
def test_msda_core_fwd_bwd_gpu(golden_dir, size, dt):
    from detrpose_amd.msda import ms_deform_attn_core
    d = _vectors(golden_dir, size)
    shapes = [tuple(int(v) for v in hw) for hw in d["shapes"]]
    loc = _edge_locs(d["loc"], 3)
    gout = torch.randn(d["out"].shape, generator=torch.Generator().manual_seed(4))
    value = d["value"]
    tdt = torch.float32 if dt == "fp32" else torch.bfloat16
    if dt == "bf16":   # the oracle sees the same rounded storage
        value, gout = value.bfloat16().float(), gout.bfloat16().float()
    ref = _grads(msda_core, value, shapes, loc, d["attn"], gout)
    v = value.to("cuda", tdt).requires_grad_(True)
    lc = loc.cuda().requires_grad_(True)
    a = d["attn"].cuda().requires_grad_(True)
    out = ms_deform_attn_core(v, shapes, lc, a)
    out.backward(gout.to("cuda", tdt))
    torch.cuda.synchronize()
    tol = 1e-4 if dt == "fp32" else 2e-2
    if dt == "fp32":   # the reference's own vectors, unmodified locations
        out0 = ms_deform_attn_core(d["value"].cuda(), shapes, d["loc"].cuda(), d["attn"].cuda())
        assert (out0.cpu() - d["out"]).abs().max().item() <= 1e-5 * max(1.0, d["out"].abs().max().item())
    for name, r, o in zip(("out", "grad_value", "grad_loc", "grad_attn"), ref, (out, v.grad, lc.grad, a.grad)):
        o = o.detach().float().cpu()
        err = (r - o).abs().max().item()
        assert torch.isfinite(o).all() and err <= tol * max(1.0, r.abs().max().item()), (name, dt, err)


@pytest.mark.gpu
def test_msda_core_bwd_atomic_hotspot():
    """Every (token, point) samples the same 2x2 corner neighbourhood: grad_value of those rows
    is the sum of thousands of atomics; checked against the oracle's autograd."""
    from detrpose_amd.msda import ms_deform_attn_core
    torch.manual_seed(0)
    N, nH, Dh, L, P, Lq = 2, 8, 32, 2, 4, 300
    shapes = [(8, 8), (4, 4)]
    S = 80
    value = torch.randn(N, S, nH * Dh)
    loc = torch.full((N, Lq, nH, L, P, 2), 0.5) + 0.01 * torch.randn(N, Lq, nH, L, P, 2)
    attn = torch.softmax(torch.randn(N, Lq, nH, L * P), -1).reshape(N, Lq, nH, L, P)
    gout = torch.randn(N, Lq, nH * Dh)
    ref = _grads(msda_core, value, shapes, loc, attn, gout)
    v = value.cuda().requires_grad_(True)
    lc = loc.cuda().requires_grad_(True)
    a = attn.cuda().requires_grad_(True)
    ms_deform_attn_core(v, shapes, lc, a).backward(gout.cuda())
    torch.cuda.synchronize()
    for name, r, o in zip(("grad_value", "grad_loc", "grad_attn"), ref[1:], (v.grad, lc.grad, a.grad)):
        err = (r - o.cpu()).abs().max().item()
        assert err <= 1e-4 * max(1.0, r.abs().max().item()), (name, err)


@pytest.mark.gpu
def test_msda_core_rejects_mixed_devices():
    """A CPU loc / attn next to a GPU value must raise before any pointer reaches the kernel."""
    from detrpose_amd.msda import ms_deform_attn_core
    N, nH, Dh, L, P, Lq = 1, 2, 8, 1, 2, 4
    shapes = [(4, 4)]
    value = torch.randn(N, 16, nH * Dh, device="cuda")
    loc = torch.rand(N, Lq, nH, L, P, 2)
    attn = torch.rand(N, Lq, nH, L, P)
    with pytest.raises(RuntimeError, match="same GPU"):
        ms_deform_attn_core(value, shapes, loc, attn.cuda())
    with pytest.raises(RuntimeError, match="same GPU"):
        ms_deform_attn_core(value, shapes, loc.cuda(), attn)
