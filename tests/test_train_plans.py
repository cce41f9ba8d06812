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
    # the weight packs on their own tapes (run once per optimizer step; the transformer's W^T
    # input-gradient packs too), each tape's packs merged
    # into ONE dp_conv_pack_batch launch over a table of > 30 descriptors with distinct outputs;
    # none left in the forwards
    from detrpose_amd._lib import PackDesc
    for pk, least in ((bb.pk, 30), (ep.pk, 30), (plan.pk, 20)):
        (name, fn, (tab, n, _)), = pk.ops
        assert name == "pack.batch" and n > least
        raw = next(t for t in pk.keep if t.data_ptr() == tab)
        descs = (PackDesc * n).from_buffer_copy(raw.cpu().numpy().tobytes())
        assert len({d.out for d in descs}) == n and all(d.w for d in descs)
    assert not any(n.startswith("pack.") for n, _, _ in bb.fw.ops + ep.fw.ops + plan.fw.ops)


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
    # dp_conv_wgrad_zs: the same kernel on a scratch kept zeroed (no zero-fill launch per call)
    assert len(names(bb.bw, lib.dp_conv_wgrad_zs)) >= 15 and len(names(ep.bw, lib.dp_conv_wgrad_zs)) > 10
    assert not names(bb.bw, lib.dp_conv_wgrad) + names(ep.bw, lib.dp_conv_wgrad)
    fw_conv = names(plan.fw, lib.dp_conv2d)
    assert any(n.endswith(".ffn1") for n in fw_conv) and any(n.endswith(".ffn2") for n in fw_conv), fw_conv[:8]
    assert any(n.endswith(".ffn2.dx") for n in names(plan.bw, lib.dp_conv2d))


def _world2_segments(rank, port, q):
    import os
    os.environ.update(RANK=str(rank), WORLD_SIZE="2", MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.set_num_threads(1)
    torch.distributed.init_process_group("gloo", rank=rank, world_size=2)
    try:
        from detrpose_amd.train_engine import Tape, TrainEngine
        model, _ = build_model("n", dtype="fp32")
        eng = TrainEngine(model, "fp32", "cpu", train_backbone=True)
        bb = eng.backbone_plan(1, 640, 640)
        shapes = [(v.H, v.W) for v in bb.outs]
        ep = eng.encoder_plan(1, shapes, feats=bb.outs, feats_plan=bb)
        out = {}
        for nm, t in (("fw", ep.fw), ("bw", ep.bw)):
            segs = Tape.segments(t.ops)
            out[nm] = ([k for k, _ in segs], t.n_host, sum(len(x) for k, x in segs if k == "device"), len(t.ops))
        out["buckets"] = eng.grad_buckets()
        out["nbuf"] = eng.grad_flat.numel()
        q.put((rank, out))
    except Exception as e:   # reported, so the parent does not wait out its queue timeout
        q.put((rank, repr(e)))
        raise
    finally:
        torch.distributed.destroy_process_group()


def test_world2_encoder_tapes_cut_into_graph_segments():
    """At world size 2 (gloo, CPU: the plans only record launches) the encoder's training tapes
    hold the SyncBN collectives as host ops (one per BatchNorm forward and backward), and
    Tape.segments cuts them there: device runs and host ops alternate, every launch lands in
    exactly one device run (each becomes one hipGraph at replay). The DDP buckets
    (TrainEngine.grad_buckets: transformer, encoder, backbone, the order the backward finishes
    them) tile the flat gradient buffer."""
    import socket
    import torch.multiprocessing as mp
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_world2_segments, args=(r, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=300) for _ in range(2))
    for p in procs:
        p.join(timeout=60)
    assert all(isinstance(v, dict) for v in res.values()), res
    assert all(p.exitcode == 0 for p in procs)
    for r in range(2):
        for nm in ("fw", "bw"):
            kinds, n_host, n_dev, n_ops = res[r][nm]
            assert n_host >= 10 and kinds.count("host") == n_host, (nm, n_host)
            assert n_dev + n_host == n_ops
            assert all(not (a == b == "device") for a, b in zip(kinds, kinds[1:])), kinds
        b = res[r]["buckets"]
        assert [p for p, _, _ in b] == ["transformer", "encoder", "backbone"]
        spans = sorted((lo, hi) for _, lo, hi in b)
        assert spans[0][0] == 0 and all(spans[i][1] == spans[i + 1][0] for i in range(2))
        assert spans[-1][1] <= res[r]["nbuf"]


def test_stored_layer_outputs_match_oracle_taps():
    """The training plans' stored layer outputs (plan.taps, by reference prefix) are exactly the
    layer outputs the oracle's TAP hook sees, with the same shapes: the forced-state parity test
    (tests/test_gpu_full_train_step_l.py) substitutes one for the other by name."""
    import numpy as np
    import oracle.detrpose_cpu as OD
    from detrpose_amd.train_engine import TrainEngine
    model, _ = build_model("l", dtype="bf16")
    eng = TrainEngine(model, "bf16", "cpu", train_backbone=True)
    bb = eng.backbone_plan(1, 640, 640)
    shapes = [(v.H, v.W) for v in bb.outs]
    ep = eng.encoder_plan(1, shapes, feats=bb.outs, feats_plan=bb)
    want = {k: (1, v.c, v.H, v.W) for k, v in list(bb.taps.items()) + list(ep.taps.items())}
    from oracle.detrpose_cpu import backbone
    from oracle.train_cpu import train_encoder
    from detrpose_amd.configs import get_config
    cfg = get_config("l")
    P = {k: v.detach() for k, v in model.state_dict().items()}
    seen = {}

    def rec(name, y):
        assert name not in seen, name
        seen[name] = tuple(y.shape)
        return y
    OD.TAP = rec
    try:
        with torch.no_grad():
            feats = backbone(torch.zeros(1, 3, 640, 640), P, cfg["backbone"]["name"], cfg["backbone"]["return_idx"],
                             cfg["backbone"]["use_lab"])
            train_encoder(feats, P, cfg["encoder"], None)
    finally:
        OD.TAP = None
    assert set(seen) == set(want), (sorted(set(want) - set(seen))[:6], sorted(set(seen) - set(want))[:6])
    bad = [(k, seen[k], want[k]) for k in want if seen[k] != want[k]]
    assert not bad, bad[:5]
    assert len(want) > 120 and np.mean([k.startswith("encoder.") for k in want]) > 0.2
