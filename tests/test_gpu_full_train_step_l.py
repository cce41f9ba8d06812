"""BASELINE config 5 at its own model size: the DETRPose-L training step on the HIP kernels
against the reference's own step (tests/golden/train_full_l_b2a2.npz, made by
tests/golden/make_train_golden.py; oracle pinned in tests/test_train_oracle.py::
test_oracle_full_step_l_accum_matches_reference). L differs from the N fixture in every tape: the
B4 backbone without LAB, three feature levels incl. the stride-8 map, 4 sampling points x 3
levels, 6 decoder layers, the bf16-only dp_conv_wgrad / conv_stream routes. The step is
train_one_epoch's (src/solver/engine.py:41-89) with the L config's grad_accum_steps=2
(configs/detrpose/include/detrpose_hgnetv2.py:15): two sub-batches of one image, each with its
own DN draws (the reference's, fed in), BatchNorm batch statistics, matching and num_boxes,
gradients summed (TrainEngine.accumulate_grads).

Why the comparison is split at the encoder output ("Training parity at DETRPose-L"):
at L the transformer's gradient moves by ~1 % when its memory input moves by 1e-6 relative
(measured by perturbing the memory of the fp64 oracle: bilinear sampling locations crossing
pixel boundaries), and any fp32 implementation's encoder output differs from the reference's by
~5e-6, so d memory and the transformer gradients are held to relative-L2 bounds; the backbone +
encoder backward is then driven by the reference's own d memory, which pins it as tightly as
at N."""
import os
import sys

import numpy as np
import pytest
import torch

from detrpose_amd import build_model
from detrpose_amd.criterion import pack_targets
from detrpose_amd.synthetic import load_synthetic, synthetic_images

pytestmark = pytest.mark.gpu
HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
from test_gpu_encoder_train_step import _targets  # noqa: E402
from test_train_oracle import _sampled, full_step_scales, sub_batches  # noqa: E402

LOCATION = ("cross_attn.sampling_offsets", "lqe_embed.")


def _nchw(v, buf):
    return buf[:, v.off:v.off + v.c].reshape(v.B, v.H, v.W, v.c).permute(0, 3, 1, 2)


def run_full_accum(g, size, dtype="fp32", split=True, cut=False, snap=False):
    """The training step of the fixture on the HIP tapes, one sub-batch after the other.

    split: after each sub-batch's transformer backward, the encoder + backbone backward runs
    on the reference's own d memory (g["s{j}.dmem"]) instead of the tapes' (recorded first).
    cut: the TrainPlan variant without the gradient through the sampling locations
    (cut_location_grads). snap: also keep every stored backbone / encoder layer output of each
    sub-batch (out["taps"][j]: reference prefix -> NCHW f32 host copy, the plans' `taps`).
    Returns a dict of host copies: losses, matchings, top-k, d memory, sampled backbone / encoder
    outputs, and the engine."""
    from detrpose_amd.train_engine import TrainEngine
    dev = torch.device("cuda")
    model, _ = build_model(size, dtype=dtype)
    load_synthetic(model, seed=int(g["meta"][1]))
    eng = TrainEngine(model, dtype, dev, train_backbone=True)
    B = int(g["meta"][0])
    images = synthetic_images(B, seed=int(g["meta"][2])).to(dev)
    sizes, ts = _targets(g, dev)
    subs = sub_batches(g)
    out = {"losses": [], "match": [], "topk": [], "dmem": [], "outs": {}, "taps": []}
    for j, (rs, tsl, p) in enumerate(subs):
        sb = rs.stop - rs.start
        bb = eng.backbone_plan(sb, images.shape[2], images.shape[3])
        bb.set_image(images[rs])
        shapes = [(v.H, v.W) for v in bb.outs]
        ep = eng.encoder_plan(sb, shapes, feats=bb.outs, feats_plan=bb)
        plan = eng.plan(sb, int(g[p + "dn_pad_size"]), shapes, memory=ep.memory, d_memory=ep.d_memory,
                        cut_location_grads=cut)
        plan.set_dn(torch.as_tensor(g[p + "dn_label"], dtype=torch.int32, device=dev),
                    torch.sigmoid(torch.as_tensor(g[p + "dn_pose_unsig"], dtype=torch.float32, device=dev)),
                    torch.as_tensor(g[p + "dn_attn_mask"], device=dev).to(torch.uint8))
        bb.forward()
        ep.forward()
        plan.forward()
        for tag, views in (("bb", bb.outs), ("enc", ep.levels)):
            for i, v in enumerate(views):
                out["outs"][f"{p}{tag}{i}"] = _nchw(v, v.buf.x).double().cpu().reshape(-1).numpy()
        if snap:
            out["taps"].append({k: _nchw(v, v.buf.x).float().cpu() for k, v in list(bb.taps.items()) +
                                list(ep.taps.items())})
        keys, vals = plan.criterion(pack_targets(ts[rs], eng.K, dev), sizes[rs], int(g[p + "dn_num_group"]))
        plan.backward()
        torch.cuda.synchronize()
        out["losses"].append(dict(zip(keys, vals.cpu().tolist())))
        out["match"].append(plan.match.cpu().numpy().astype(np.int64))
        out["topk"].append(plan.topi.cpu().numpy())
        out["dmem"].append(ep.d_memory.double().cpu().numpy().reshape(sb, -1, eng.C))
        if split:
            ep.d_memory.copy_(torch.as_tensor(g[p + "dmem"], device=dev).reshape(ep.d_memory.shape))
        ep.backward()
        bb.backward()
        eng.accumulate_grads(first=j == 0, last=j == len(subs) - 1)
    torch.cuda.synchronize()
    out["eng"] = eng
    return out


@pytest.fixture(scope="module")
def golden_l(golden_dir):
    return np.load(os.path.join(golden_dir, "train_full_l_b2a2.npz"))


@pytest.fixture(scope="module")
def full_l(golden_l):
    return run_full_accum(golden_l, "l")


def test_l_step_forward_losses_matching(golden_l, full_l):
    """Backbone / encoder outputs of both sub-batches within 2e-4 of scale (measured 0.9-1.1e-4
    over runs: the encoder's f32-atomic BatchNorm sums change order run to run); every loss of
    both sub-batches within 5e-4 relative; the kernels' own per-head Hungarian assignments equal
    to the reference matcher's."""
    g, r = golden_l, full_l
    worst = 0.0
    for name, got in r["outs"].items():
        idx, val, s, a = _sampled(g, name)
        scale = max(float(np.abs(val).max()), a / got.size)
        err = float(np.abs(got[idx] - val).max()) / scale
        worst = max(worst, err)
        assert err <= 2e-4, (name, err)
    lw = []
    for j, (_, _, p) in enumerate(sub_batches(g)):
        ref = dict(zip([str(k) for k in g[p + "loss_keys"]], g[p + "loss_vals"]))
        got = r["losses"][j]
        assert sorted(got) == sorted(ref)
        lw += [(abs(got[k] - ref[k]) / max(abs(ref[k]), 1.0), p + k) for k in ref]
        np.testing.assert_array_equal(r["match"][j], g[p + "match"], err_msg=p)
    lw.sort(reverse=True)
    print(f"outputs worst rel err {worst:.3g}; losses worst {lw[:4]}")
    assert lw[0][0] <= 5e-4, lw[:4]


def test_l_step_d_memory_and_transformer_gradients(golden_l, full_l):
    """d loss / d memory (each sub-batch) and every transformer parameter's accumulated gradient
    against the reference's, end to end: relative L2 <= 0.25 (measured on MI355X over runs: d memory
    2.3-2.7 % / 7.4-9.7 %, worst parameter 0.11-0.16, transformer median 1.1-2.8 %; at L these move
    by ~1 % per 1e-6 relative change of the memory (module docstring), and the encoder's
    BatchNorm statistics are float-atomic sums, so every run's memory differs by ~1e-6 and the
    matching / bilinear footprints move with it — test_l_step_fp32_per_parameter_location_cut
    pins the same kernels tightly)."""
    g, r = golden_l, full_l
    bad = []
    for j, (_, _, p) in enumerate(sub_batches(g)):
        rd = g[p + "dmem"].astype(np.float64)
        l2 = float(np.linalg.norm(r["dmem"][j] - rd) / np.linalg.norm(rd))
        print(f"{p}d memory rel L2 {l2:.3g}")
        if l2 > 0.25:
            bad.append((p + "dmem", l2))
    eng = r["eng"]
    names = sorted(k[:-len("__idx")] for k in g.files if k.startswith("grad.") and k.endswith("__idx")
                   and not k.startswith(("grad.backbone.", "grad.encoder.")))
    scales = full_step_scales(g, names)
    rows = []
    for n in names:
        flat = eng.grads["transformer." + n[len("grad."):]].double().cpu().reshape(-1).numpy()
        idx, val, s, a = _sampled(g, n)
        if scales[n] < 1e-5:
            continue
        d = flat[idx] - val
        rows.append((float(np.linalg.norm(d) / max(np.linalg.norm(val), 1e-30)), float(np.abs(d).max()) / scales[n], n))
    rows.sort(reverse=True)
    for row in rows[:10]:
        print("transformer %s: rel L2 %.3g, max %.3g of scale" % (row[2], row[0], row[1]))
    print("transformer median rel L2 %.3g" % np.median([r_[0] for r_ in rows]))
    assert len(rows) > 250
    assert not bad, bad
    assert rows[0][0] <= 0.25, rows[:5]


def test_l_step_backbone_encoder_gradients(golden_l, full_l):
    """Every backbone and encoder parameter's accumulated gradient, the backward driven by the
    reference's own d memory: relative L2 within 1e-2 (measured 4.6e-3), sampled entries within
    5e-2 of scale (measured 1.8e-2, a 5x5 depthwise weight of stage 2: ReLU masks of
    pre-activations within ~1e-5 of zero differ between any two fp32 forwards), sums within
    3e-3 of sum |g| (7e-4); the encoder's BatchNorm running statistics after both sub-batches
    within 1e-4."""
    g, r = golden_l, full_l
    eng = r["eng"]
    names = sorted(k[:-len("__idx")] for k in g.files if k.startswith(("grad.backbone.", "grad.encoder."))
                   and k.endswith("__idx"))
    scales = full_step_scales(g, names)
    rows = []
    for n in names:
        flat = eng.grads[n[len("grad."):]].double().cpu().reshape(-1).numpy()
        idx, val, s, a = _sampled(g, n)
        if scales[n] < 1e-5:
            assert float(np.abs(flat).max()) < 1e-4, (n, float(np.abs(flat).max()))
            continue
        d = flat[idx] - val
        rows.append((float(np.abs(d).max()) / scales[n], float(np.linalg.norm(d) / max(np.linalg.norm(val), 1e-30)),
                     abs(flat.sum() - s) / max(a, 1e-30), n))
    rows.sort(reverse=True)
    for row in rows[:8]:
        print("%s: rel err %.3g, l2 %.3g, sum %.3g" % (row[3], row[0], row[1], row[2]))
    assert sum(n.startswith("grad.backbone.") for n in names) >= 80
    assert rows[0][0] <= 5e-2, rows[:5]
    assert max(r_[1] for r_ in rows) <= 1e-2, sorted(rows, key=lambda r_: -r_[1])[:5]
    assert max(r_[2] for r_ in rows) <= 3e-3, sorted(rows, key=lambda r_: -r_[2])[:5]
    for k in [k for k in g.files if k.startswith("bn.")]:
        np.testing.assert_allclose(eng.running[k[3:]].cpu().numpy(), g[k], rtol=1e-4, atol=1e-5, err_msg=k)


def forced_per_parameter(g, size, run, cut=True):
    """The fp32 oracle's whole training step (oracle/train_cpu.py, pinned to the reference) on
    the HIP run's own two-stage selection and per-head matchings, sub-batch by sub-batch, with
    the location gradients cut like the run's (cut_loc): returns (per-sub-batch oracle losses,
    {parameter: relative L2 of the run's gradient against the oracle's}) over every trained
    parameter whose oracle gradient does not vanish."""
    from test_train_oracle import oracle_train_step_full
    force = [{"topk": t, "match": m} for t, m in zip(run["topk"], run["match"])]
    lds, grads, _, _, _ = oracle_train_step_full(size, g, force=force, split=False, cut_loc=cut)
    eng = run["eng"]
    rel = {}
    for k, v in grads.items():
        key = k[len("grad."):]
        key = key if key.startswith(("encoder.", "backbone.")) else "transformer." + key
        ref = v.detach().double().reshape(-1).numpy()
        got = eng.grads[key].double().cpu().reshape(-1).numpy()
        nr = np.linalg.norm(ref)
        if nr < 1e-6 * max(1.0, ref.size ** 0.5):   # analytically zero (a bias ahead of a BatchNorm)
            continue
        rel[key] = float(np.linalg.norm(got - ref) / nr)
    return lds, rel


def family(k):
    return ("backbone.lab" if k.startswith("backbone.") and ".lab." in k else
            "backbone" if k.startswith("backbone.") else "encoder" if k.startswith("encoder.") else "transformer")


def per_parameter_table(rel, tag):
    """Per-family medians / maxima of the per-parameter relative L2 errors (printed)."""
    fam = {}
    for k, v in rel.items():
        fam.setdefault(family(k), []).append((v, k))
    for f, rows in sorted(fam.items()):
        rows.sort(reverse=True)
        print(f"{tag} per-parameter rel L2 [{f}] n={len(rows)} median {np.median([r[0] for r in rows]):.3g} "
              f"worst {[(round(v, 4), k) for v, k in rows[:3]]}")
    return fam


def loss_errors(g, run, lds):
    worst = []
    for j, (_, _, p) in enumerate(sub_batches(g)):
        ref = {k: float(v) for k, v in lds[j].items()}
        worst += [(abs(run["losses"][j][k] - ref[k]) / max(abs(ref[k]), 1.0), p + k) for k in ref]
    worst.sort(reverse=True)
    return worst


def test_l_step_fp32_per_parameter_location_cut(golden_l):
    """Every trained parameter of the L step, per parameter, with the function made continuous:
    the location gradients cut on both sides (TrainPlan cut_location_grads / the oracle's
    cut_loc) and the oracle forced onto the run's own selection and matchings. fp32: losses within
    5e-4 relative, each parameter's gradient within 1e-2 relative L2 (the LAB-free L backbone
    included)."""
    g = golden_l
    r = run_full_accum(g, "l", dtype="fp32", split=False, cut=True)
    lds, rel = forced_per_parameter(g, "l", r)
    worst = loss_errors(g, r, lds)
    print("fp32 (cut) vs oracle, worst losses:", worst[:4])
    fam = per_parameter_table(rel, "fp32 cut")
    assert worst[0][0] <= 5e-4, worst[:4]
    assert len(rel) > 500
    for f, rows in fam.items():
        assert rows[0][0] <= FP32_CUT_BOUNDS[f], (f, rows[:3])


# fp32, location gradients cut (relative L2 per parameter). Measured on MI355X: transformer
# median 1.9e-4, worst 6.6e-3 (enc_pose_embed); encoder median 1.8e-2, worst 2.7e-2; backbone
# median 2.0e-2, worst 3.0e-2. The backbone / encoder figures are the conditioning of this
# fixture, not kernel error: the fp32 oracle itself moves by median 0.4-0.5 %, worst 0.8 %
# between float32 and float64 on the same forced selection (B = 1 sub-batches: training-mode
# BatchNorm over one image's map, DESIGN.md, "Training parity at DETRPose-L").
FP32_CUT_BOUNDS = {"transformer": 1e-2, "encoder": 5e-2, "backbone": 5e-2}

# bf16, location gradients cut: (median, worst) relative L2 per family, ~1.3-1.5x the MI355X
# measurement printed by per_parameter_table (a regression guard). LAB scalars: median only
# (single numbers summed over a whole map, some analytically ~0). Measured:
#   N  transformer median 0.017 worst 0.49 (enc_pose_embed), encoder 0.18 / 0.37,
#      backbone 0.21 / 0.51;
#   L  transformer median 0.042 worst 0.51 (layer 5's attention_weights), encoder 0.69 / 1.12,
#      backbone 0.84 / 1.24.
# At L the bf16 gradient below the decoder is not a perturbation of the fp32 one on this
# fixture: besides the sampling locations (cut here), the VFL loss's OKS targets
# (criterion.py:58-93, keypoint_loss.py:5-34) move by ~10 % for a 1e-3 keypoint error on the
# fixture's small synthetic persons (area down to 1e-3 of the image), which bf16's ~1e-2
# keypoint error reaches: single losses move by up to 18 % with the selection and matching
# forced ("Training parity at DETRPose-L").
# At L the backbone / encoder worst parameters sit above 1.0 relative L2 end to end, so only the
# medians are bounded there, below 1.0 (a zero gradient has relative L2 = 1 for every parameter
# and fails them); test_l_step_bf16_split_backbone_encoder is the check that pins the bf16
# backbone + encoder backward per parameter. The L transformer's worst parameter is the LQE
# head's first reg_conf layer (its input is the top-k statistics of the predicted corner
# distributions): over round-6 runs it measured 0.49, 0.50, 0.72, 0.77 (float-atomic weight
# gradients are not run-to-run deterministic), so its bound is 0.9, still below a zeroed
# gradient's 1.0.
BF16_BOUNDS = {
    "n": {"transformer": (0.03, 0.75), "encoder": (0.27, 0.6), "backbone": (0.32, 0.8), "backbone.lab": (0.32, None)},
    "l": {"transformer": (0.06, 0.9), "encoder": (0.9, None), "backbone": (0.97, None)},
}
BF16_LOSS_BOUND = {"n": 8e-2, "l": 0.25}   # measured N 1.4-5.2 % (over runs), L 18-20 %


def check_bf16_families(fam, size):
    for f, rows in fam.items():
        med_b, worst_b = BF16_BOUNDS[size][f]
        med = float(np.median([r[0] for r in rows]))
        assert med <= med_b, (f, med)
        assert worst_b is None or rows[0][0] <= worst_b, (f, rows[:3])


def test_l_step_bf16_per_parameter_location_cut(golden_l):
    """bf16 L step (bf16 activations / activation gradients, f32 accumulation and parameter
    gradients) against the fp32 oracle on the bf16 run's own top-k and matchings, location
    gradients cut on both sides (see the fp32 variant): every loss within BF16_LOSS_BOUND
    (relative to max(|loss|, 1); measured 0.18), and EACH parameter's gradient within its
    family's relative-L2 bound (BF16_BOUNDS: the median and the worst parameter of each family;
    why the L figures are large is written there)."""
    g = golden_l
    r = run_full_accum(g, "l", dtype="bf16", split=False, cut=True)
    lds, rel = forced_per_parameter(g, "l", r)
    worst = loss_errors(g, r, lds)
    print("bf16 (cut) vs forced fp32 oracle, worst losses:", worst[:5])
    fam = per_parameter_table(rel, "L bf16 cut")
    assert worst[0][0] <= BF16_LOSS_BOUND["l"], worst[:5]
    check_bf16_families(fam, "l")


# The backbone + encoder backward on the GPU run's OWN forward state ("teacher forcing"). At L this
# fixture's backbone / encoder gradients are ill-conditioned in the forward state: on the fp32
# oracle with the reference's d memory, 0.4 % noise on the input image moves them by 15 % (median
# relative L2), rounding the backbone + encoder weights to bf16 by 45 % / 38 %, rounding only the
# AIFI layer's weights by 5 % ("Training parity at DETRPose-L"). A bf16 forward's state
# differs from fp32 by bf16 storage at every layer, so against the fp32 gradients no bf16
# implementation can come within a few 1e-2. Instead the fp32 oracle runs its backbone + encoder
# forward with every stored layer output replaced by the GPU run's stored value
# (oracle.detrpose_cpu.TAP: y + (gpu - y).detach(), the oracle's own gradient path), so its
# backward (driven by the reference's d memory, as the GPU's) is the fp32 backward AT the GPU's
# forward state: what is left is the rounding of the GPU's backward itself. Bounds: (median,
# worst) relative L2 per family over whole parameter tensors, from the MI355X measurement the
# test prints.
# Measured on MI355X (profiles/r6b_pytest_forced.txt): fp32 backbone median 2.4e-4 / worst 8.5e-4,
# encoder 3.8e-6 / 1.6e-4; bf16 backbone 0.098 / 0.20 (the backbone's ~40 layers of bf16 activation
# gradients compound), encoder 0.015 / 0.56 (the two downsample cv1 BatchNorm weights, 0.56 / 0.38:
# a dgamma = sum(dy x_hat) that cancels; they sit at the same ~40x the family median in fp32). A
# missing or zeroed gradient has relative L2 1.0: above every worst bound.
FORCED_BOUNDS = {"fp32": {"encoder": (1e-4, 2e-3), "backbone": (1e-3, 5e-3)},
                 "bf16": {"encoder": (0.025, 0.8), "backbone": (0.15, 0.3)}}


def forced_oracle_grads(g, size, run):
    """The fp32 oracle's accumulated backbone + encoder gradients of the fixture's step with every
    stored layer output forced to the GPU run's (run["taps"][j] per sub-batch) and the backward
    from the reference's d memory. Returns ({name: gradient}, {tap names the oracle read})."""
    import oracle.detrpose_cpu as OD
    from test_train_oracle import oracle_train_step_full
    state = {"j": -1, "used": set()}

    def force(name, y):
        if name == "backbone.stem.stem1":
            state["j"] += 1
        gv = run["taps"][state["j"]][name]
        assert tuple(gv.shape) == tuple(y.shape), (name, tuple(gv.shape), tuple(y.shape))
        state["used"].add(name)
        return y + (gv.to(y.dtype) - y).detach()

    OD.TAP = force
    try:
        _, grads, _, _, _ = oracle_train_step_full(size, g, split=True)
    finally:
        OD.TAP = None
    assert state["j"] == len(run["taps"]) - 1
    return {k[len("grad."):]: v.detach() for k, v in grads.items() if k.startswith(("grad.backbone.", "grad.encoder."))}, \
        state["used"]


def forced_rows(ref, grads, zero=(), all_zero=False):
    """Per backbone / encoder parameter: (relative L2 of the GPU gradient against the forced
    oracle's, name); `zero` names (or every parameter, all_zero) read as zero gradients (the
    negative controls). Parameters whose oracle gradient vanishes analytically are skipped: a bias
    whose every consumer normalises it away (input_proj's BatchNorm bias and the AIFI's last
    LayerNorm bias, each followed only by convs into a training-mode BatchNorm), recognised by a
    gradient RMS below 1e-4 of its family's median (rounding noise)."""
    rms = {k: float(v.double().norm()) / max(1, v.numel()) ** 0.5 for k, v in ref.items()}
    fam_rms = {}
    for k, r in rms.items():
        fam_rms.setdefault(k.split(".")[0], []).append(r)
    fam_rms = {f: float(np.median(v)) for f, v in fam_rms.items()}
    rows = []
    for k, v in ref.items():
        r = v.double().reshape(-1).numpy()
        nr = np.linalg.norm(r)
        if rms[k] < 1e-4 * fam_rms[k.split(".")[0]]:
            continue
        got = grads[k].double().cpu().reshape(-1).numpy()
        if all_zero or k in zero:
            got = np.zeros_like(got)
        rows.append((float(np.linalg.norm(got - r) / nr), k))
    return rows


def forced_check(rows, bounds, verbose=False):
    """None when every family meets its (median, worst) bounds, else the first failure."""
    fam = {}
    for r_ in rows:
        fam.setdefault(r_[1].split(".")[0], []).append(r_)
    fails = []
    for f, rs in sorted(fam.items()):
        rs.sort(reverse=True)
        med = float(np.median([r_[0] for r_ in rs]))
        if verbose:
            print(f"forced-state per-parameter rel L2 [{f}] n={len(rs)} median {med:.3g} worst "
                  f"{[(round(r_[0], 5), r_[1]) for r_ in rs[:4]]}")
        if med > bounds[f][0]:
            fails.append((f, "median", med))
        if rs[0][0] > bounds[f][1]:
            fails.append((f, "worst", rs[:3]))
    return fails[0] if fails else None


@pytest.mark.parametrize("dtype", ["fp32", "bf16"])
def test_l_step_backbone_encoder_backward_at_own_forward_state(golden_l, dtype):
    """DETRPose-L backbone + encoder backward, per parameter, on the run's own forward state: the
    tapes run the step's forward (both sub-batches), then their encoder + backbone backward from
    the REFERENCE's d memory of each sub-batch; the fp32 oracle (pinned to the reference) runs
    the same step with every stored layer output forced to the GPU's (FORCED_BOUNDS comment) and
    the same d memory. Every backbone / encoder parameter's accumulated gradient (whole tensors)
    within its family's (median, worst) relative-L2 bound. Negative controls, which must FAIL the
    same check: an all-zero gradient arena, and the real gradients with one parameter zeroed (the
    deepest, stem1's weight; an encoder FPN conv)."""
    g = golden_l
    r = run_full_accum(g, "l", dtype=dtype, split=True, snap=True)
    eng = r["eng"]
    ref, used = forced_oracle_grads(g, "l", r)
    taps = set(r["taps"][0])
    assert used == taps, (sorted(taps - used)[:5], sorted(used - taps)[:5])
    rows = forced_rows(ref, eng.grads)
    assert sum(k.startswith("backbone.") for _, k in rows) >= 80
    assert sum(k.startswith("encoder.") for _, k in rows) >= 100
    b = FORCED_BOUNDS[dtype]
    print(f"{dtype}: {len(used)} stored layer outputs forced per sub-batch")
    fail = forced_check(rows, b, verbose=True)
    assert fail is None, fail
    assert forced_check(forced_rows(ref, eng.grads, all_zero=True), b) is not None, "zero-gradient control passed"
    for probe in ("backbone.stem.stem1.conv.weight", "encoder.fpn_blocks.0.cv4.conv.weight"):
        assert any(k == probe for _, k in rows), probe
        assert forced_check(forced_rows(ref, eng.grads, zero=(probe,)), b) is not None, f"zeroed {probe} passed"
