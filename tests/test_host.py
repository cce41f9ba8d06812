"""Host-side checks that need no GPU: the C-ABI library loads and exports every symbol
include/detrpose_hip.h declares, the module tree has the reference's exact state_dict
layout, BN folding / packing match the reference math, and the whole kernel plan can
be recorded (shape-checked) for N / L / X without executing it."""
import json
import os
import re

import pytest
import torch
import torch.nn.functional as F

from detrpose_amd import build_model
from detrpose_amd import _lib
from detrpose_amd.engine import Engine, Packer
from detrpose_amd.synthetic import load_synthetic

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _header_symbols():
    txt = open(os.path.join(REPO, "include", "detrpose_hip.h")).read()
    return sorted(set(re.findall(r"\b(dp_[a-z0-9_]+)\s*\(", txt)))


def test_library_exports_header_symbols():
    lib = _lib.load()
    syms = _header_symbols()
    assert len(syms) >= 20
    for s in syms:
        assert hasattr(lib, s), f"{s} declared in include/detrpose_hip.h but not exported"
    assert set(syms) == set(_lib.EXPORTED), "ctypes prototypes out of sync with the header"
    assert lib.dp_version() >= 1


def test_library_source_hash_guard():
    """The .so carries the hash of the sources it was built from; the loader refuses a
    library whose hash differs from the sources shipped beside it (a stale prebuilt .so)."""
    from detrpose_amd.build import lib_source_hash
    lib = _lib.load()
    assert lib.dp_source_hash().decode() == lib_source_hash()
    _lib.verify_source(lib)   # matching hash: accepted
    with pytest.raises(_lib.HipError, match="rebuild"):
        _lib.verify_source(lib, expected="0000000000000000")


def test_plan_costs_and_kernel_names():
    """Every launch of a plan records its algorithmic bytes and FLOPs (bench.py's per-launch
    bounds) and every dp_conv2d launch the kernel instantiation the dispatcher picks."""
    from detrpose_amd.profiling import canonical_kernel_name
    model, _ = build_model("l")
    load_synthetic(model, 0)
    plan = Engine(model, "bf16", device="cpu").plan(4)
    plan.add_postprocess()
    for name, fn, _ in plan.ops + plan.post_ops:
        assert name in plan.op_bytes and name in plan.op_flops, name
        assert plan.op_bytes[name] > 0, name
        if fn.__name__ == "dp_conv2d":
            k = plan.kernel_of(name)
            assert k.startswith(("conv_halo_kernel<", "conv_stream_kernel<", "conv_direct_kernel<")), (name, k)
    assert "conv_halo_kernel<8, 4, 3, 3, 1, 128, false, false, 2, false, 0, 2>" in plan.op_kernel.values()
    # rocprofv3's mangled and demangled spellings reduce to the describe form
    assert canonical_kernel_name("_ZN12_GLOBAL__N_118conv_stream_kernelILi256ELi256ELi2ELi8ELi2ELb1ELi2EDF16bLi0EEEv"
                                 "12dp_conv_desciiii") == "conv_stream_kernel<256, 256, 2, 8, 2, true, 2, bf16, 0>"
    assert canonical_kernel_name('"void (anonymous namespace)::conv_halo_kernel<8, 4, 3, 3, 1, 128, false, false, 2, '
                                 'false, 0>(dp_conv_desc, int, int, int, int, (anonymous namespace)::HaloPool)"') == \
        "conv_halo_kernel<8, 4, 3, 3, 1, 128, false, false, 2, false, 0>"


def test_conv_desc_layout_matches_header():
    # the ctypes mirror must have the header's field order (checked by name list)
    txt = open(os.path.join(REPO, "include", "detrpose_hip.h")).read()
    body = txt[txt.index("typedef struct dp_conv_desc"):txt.index("} dp_conv_desc;")]
    body = re.sub(r"/\*.*?\*/", "", body, flags=re.S)
    names = re.findall(r"\*?\s*(\w+)\s*[,;]", body.split("{", 1)[1])
    mirror = [f[0].rstrip("_") for f in _lib.ConvDesc._fields_]
    assert names == mirror


@pytest.mark.parametrize("size", ["n", "l", "x"])
def test_state_dict_layout_matches_reference(golden_dir, size):
    with open(os.path.join(golden_dir, "manifest.json")) as f:
        man = json.load(f)[size]
    model, _ = build_model(size)
    sd = model.state_dict()
    assert {k: list(v.shape) for k, v in sd.items()} == man


def test_buffers_match_reference_values(golden_dir):
    # anchors / valid_mask / dim_t are architecture constants the checkpoint also carries
    from oracle.detrpose_cpu import anchors_and_mask
    model, _ = build_model("l")
    a, m = anchors_and_mask([8, 16, 32])
    assert torch.equal(model.transformer.anchors, a)
    assert torch.equal(model.transformer.valid_mask, m)


def test_bn_fold_and_pack_match_conv():
    torch.manual_seed(0)
    sd = {"x.conv.weight": torch.randn(24, 16, 3, 3), "x.bn.weight": torch.rand(24) + 0.5,
          "x.bn.bias": torch.randn(24), "x.bn.running_mean": torch.randn(24), "x.bn.running_var": torch.rand(24) + 0.5}
    pk = Packer(sd, "fp32", torch.device("cpu"))
    w, b, _ = pk.conv_bn_act("x")
    pc = pk.conv(w, b)
    x = torch.randn(1, 16, 7, 9)
    ref = F.conv2d(x, sd["x.conv.weight"], None, 1, 1)
    scale = sd["x.bn.weight"] * (sd["x.bn.running_var"] + 1e-5).rsqrt()
    ref = ref * scale[None, :, None, None] + (sd["x.bn.bias"] - sd["x.bn.running_mean"] * scale)[None, :, None, None]
    # emulate the implicit GEMM with the packed K-major weight (k = (ky*kw+kx)*cin + c)
    cols = F.unfold(x, 3, padding=1)  # (1, cin*9, L) ordered (c, ky, kx)
    cols = cols.reshape(1, 16, 9, -1).permute(0, 2, 1, 3).reshape(1, 144, -1)
    y = (pc.w[:, :144] @ cols[0]) + pc.b[:, None]
    assert torch.allclose(y.reshape(1, 24, 7, 9), ref, atol=1e-4)
    assert pc.kpad % 32 == 0 and pc.kpad >= 144


@pytest.mark.parametrize("size,dtype", [("n", "bf16"), ("l", "bf16"), ("x", "bf16"), ("l", "fp32")])
def test_plan_records_full_forward(size, dtype):
    model, _ = build_model(size, dtype=dtype)
    load_synthetic(model, 0)
    eng = Engine(model, dtype, device="cpu")   # pack + plan only; nothing is launched
    plan = eng.plan(2)
    names = [n for n, _, _ in plan.ops]
    nl = model.transformer.num_decoder_layers
    # the bf16 32-channel stems (L / X) run StemBlock as one dp_stem_fused launch
    first = "stem" if dtype == "bf16" and size in ("l", "x") else "stem1"
    assert names[0] == first and f"dec{nl - 1}.lqe1" == names[-1]
    assert ("stem1" in names) == (first == "stem1")
    assert sum(n.endswith(".msda") for n in names) == nl
    assert plan.outputs["pred_keypoints"].shape == (2, 60, 17, 2)
    assert plan.outputs["pred_logits"].shape == (2, 60, 2)


def test_forward_refuses_cpu_tensors():
    model, _ = build_model("n")
    with pytest.raises(RuntimeError):
        model.deploy()(torch.rand(1, 3, 640, 640))


def test_frag_pack_layout():
    """The MFMA-fragment weight layout (include/detrpose_hip.h): lane l = 16 g + q of
    fragment j of block (nb, s) holds W[32 nb + (q//4)*8 + 4j + q%4][32 s + 8 g : +8]."""
    from detrpose_amd.fragments import frag_pack, frag_unpack
    w = torch.randn(66, 128).bfloat16().float()
    f = frag_pack(w)
    assert f.shape == (3, 4, 2, 64, 8) and f.dtype == torch.bfloat16
    assert torch.equal(frag_unpack(f, 66), w)
    for nb, s, j, g, q in ((0, 0, 0, 0, 0), (1, 3, 1, 2, 13), (2, 1, 0, 3, 7)):
        c = 32 * nb + (q // 4) * 8 + 4 * j + q % 4
        if c < 66:
            assert torch.equal(f[nb, s, j, 16 * g + q].float(), w[c, 32 * s + 8 * g: 32 * s + 8 * g + 8])
    assert (frag_unpack(f, 96)[66:] == 0).all()
