"""The training tapes build on the CPU for every model size (no launches: the plans only record
C-ABI calls), and every trained parameter of the network receives a gradient: some recorded
backward launch writes into its slot of the flat gradient buffer (GEMM / conv descriptors'
outputs, the BatchNorm / LAB / LayerNorm / embedding gradient pointers). This is the
structural half of the GPU parity tests (tests/test_gpu_full_train_step.py pins the values)."""
import ctypes as C

import pytest
import torch

from detrpose_amd import build_model


def _pointers(tape):
    """Every integer argument of the tape's launches and every pointer field of its descriptors."""
    ptrs = set()
    for _, _, args in tape.ops:
        for a in args:
            if isinstance(a, int):
                ptrs.add(a)
            elif isinstance(a, C.c_void_p) and a.value:
                ptrs.add(a.value)
    for d in tape.keep:
        for name, _ in getattr(d, "_fields_", []):
            v = getattr(d, name)
            if isinstance(v, int) and v > 4096:
                ptrs.add(v)
    return ptrs


@pytest.mark.parametrize("size,B", [("n", 2), ("l", 1)])
def test_every_parameter_gets_a_gradient(size, B):
    from detrpose_amd.train_engine import TrainEngine
    model, _ = build_model(size, dtype="bf16")
    eng = TrainEngine(model, "bf16", "cpu", train_backbone=True)
    bb = eng.backbone_plan(B, 640, 640)
    shapes = [(v.H, v.W) for v in bb.outs]
    ep = eng.encoder_plan(B, shapes, feats=bb.outs, feats_plan=bb)
    plan = eng.plan(B, 36, shapes, memory=ep.memory, d_memory=ep.d_memory)
    ptrs = set()
    for t in (plan.bw, ep.bw, bb.bw):
        ptrs |= _pointers(t)
    names = [n for n, p in model.named_parameters() if p.requires_grad]
    assert sorted(names) == sorted(eng.pnames)
    missing = []
    for n in names:
        g = eng.grads[n]
        lo, hi = g.data_ptr(), g.data_ptr() + g.numel() * 4
        if not any(lo <= p < hi for p in ptrs):
            missing.append(n)
    assert not missing, missing[:10]
    # the d memory hand-off and the backbone outputs' gradients are wired
    assert ep.d_memory.data_ptr() in _pointers(plan.bw)
    assert all(v.buf.g is not None for v in bb.outs)
    assert len(bb.fw.ops) > 30 and len(ep.bw.ops) > 100
    # the weight packs on their own tapes (run once per optimizer step), none left in the forwards
    assert len(bb.pk.ops) > 30 and len(ep.pk.ops) > 30
    assert not any(n.startswith("pack.") for n, _, _ in bb.fw.ops + ep.fw.ops)


def test_bf16_tapes_route_to_the_fast_kernels():
    """bf16 L tapes: the k x k weight gradients run as implicit GEMMs (dp_conv_wgrad; only stem1,
    over the f32 image, keeps im2col columns), the transformer's linears and their input
    gradients on the 1x1 conv kernel (dp_gemm keeps the weight gradients)."""
    from detrpose_amd.train_engine import TrainEngine
    model, _ = build_model("l", dtype="bf16")
    eng = TrainEngine(model, "bf16", "cpu", train_backbone=True)
    bb = eng.backbone_plan(1, 640, 640)
    shapes = [(v.H, v.W) for v in bb.outs]
    ep = eng.encoder_plan(1, shapes, feats=bb.outs, feats_plan=bb)
    plan = eng.plan(1, 36, shapes, memory=ep.memory, d_memory=ep.d_memory)
    lib = eng.lib
    names = lambda t, fn: [n for n, f, _ in t.ops if f is fn]   # noqa: E731
    im2col = names(bb.bw, lib.dp_im2col) + names(ep.bw, lib.dp_im2col)
    assert im2col == ["stem1.im2col"], im2col
    assert len(names(bb.bw, lib.dp_conv_wgrad)) >= 15 and len(names(ep.bw, lib.dp_conv_wgrad)) > 10
    fw_conv = names(plan.fw, lib.dp_conv2d)
    assert any(n.endswith(".ffn1") for n in fw_conv) and any(n.endswith(".ffn2") for n in fw_conv), fw_conv[:8]
    assert any(n.endswith(".ffn2.dx") for n in names(plan.bw, lib.dp_conv2d))
