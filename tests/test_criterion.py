"""Training criterion: HungarianMatcher + Criterion (losses ['vfl', 'keypoints']).

CPU: the LSAP restatement (oracle/lsap_cpu.py) reproduces scipy.optimize.linear_sum_assignment
(the reference's solver, matcher.py:97) index for index, ties included; the criterion
restatement (oracle/criterion_cpu.py) reproduces the reference's own matchings, cost matrix,
union matching, loss values and gradients on tests/golden/criterion_*.npz (made by
tests/golden/make_train_golden.py from the reference).

GPU (through the C ABI): dp_hungarian_match / dp_match_union / dp_pose_loss behind
detrpose_amd.criterion vs the same fixtures: matchings and union index for index, cost matrix
and losses within 1e-5 relative (f32, different reduction order), gradients within 1e-5 of
their scale; and vs the oracle on a b64 batch (the L training batch per GPU) and on
tie-heavy costs (dyadic keypoints, so the f32 costs are exact and the LSAP tie-breaks decide).
"""
import os

import numpy as np
import pytest
import torch

from oracle import criterion_cpu as oc
from oracle.lsap_cpu import lsap

CASES = ["a", "b", "c"]


def _load(golden_dir, name):
    g = np.load(os.path.join(golden_dir, f"criterion_{name}.npz"))
    return {k: g[k] for k in g.files}


def _inputs(g, device="cpu", requires_grad=False):
    H = int(g["n_aux"]) + 3
    heads = []
    for i in range(H):
        lg = torch.from_numpy(g[f"logits{i}"]).to(device).requires_grad_(requires_grad)
        kp = torch.from_numpy(g[f"kps{i}"]).to(device).requires_grad_(requires_grad)
        heads.append((lg, kp))
    return heads


def _targets(g, device):
    K = int(g["K"])
    off = np.concatenate([[0], np.cumsum(g["sizes"])])
    out = []
    for b in range(len(g["sizes"])):
        s = slice(off[b], off[b + 1])
        out.append({"labels": torch.from_numpy(g["tgt_labels"][s]).to(device),
                    "keypoints": torch.from_numpy(g["tgt_kps"][s].reshape(-1, 3 * K)).to(device),
                    "area": torch.from_numpy(g["tgt_area"][s]).to(device),
                    "boxes": torch.zeros(off[b + 1] - off[b], 4, device=device)})
    return out


def _outputs(heads, n_aux):
    def d(i):
        return {"pred_logits": heads[i][0], "pred_keypoints": heads[i][1]}
    return {**d(0), "aux_outputs": [d(1 + i) for i in range(n_aux)], "aux_pre_outputs": d(1 + n_aux),
            "aux_interm_outputs": [d(2 + n_aux)]}


# ---------------------------------------------------------------- CPU: oracle pinning

def test_lsap_matches_scipy():
    from scipy.optimize import linear_sum_assignment
    rng = np.random.default_rng(1)
    for trial in range(600):
        nr, nc = int(rng.integers(1, 64)), int(rng.integers(1, 24))
        if trial % 2:
            nr, nc = nc, nr
        c = rng.integers(0, 3, (nr, nc)).astype(np.float32) if trial % 3 else rng.random((nr, nc)).astype(np.float32)
        a, b = linear_sum_assignment(c), lsap(c)
        assert np.array_equal(a[0], b[0]) and np.array_equal(a[1], b[1]), (trial, nr, nc)


@pytest.mark.parametrize("name", CASES)
def test_oracle_criterion_golden(golden_dir, name):
    g = _load(golden_dir, name)
    K, ncls, n_aux = int(g["K"]), int(g["ncls"]), int(g["n_aux"])
    heads = _inputs(g, requires_grad=True)
    tl, tk, ta = (torch.from_numpy(g[k]) for k in ("tgt_labels", "tgt_kps", "tgt_area"))
    losses, matches, go = oc.criterion(heads, g["sizes"], tl, tk, ta, K, ncls, n_aux)
    assert np.array_equal(matches, g["match"])
    assert np.array_equal(go, g["go"])
    # the final head's cost matrix, image by image (the reference's columns are all targets)
    off = np.concatenate([[0], np.cumsum(g["sizes"])])
    for b in range(len(g["sizes"])):
        if off[b + 1] == off[b]:
            continue
        C = oc.match_cost(heads[0][0][b].detach(), heads[0][1][b].detach(), tl[off[b]:off[b + 1]],
                          tk[off[b]:off[b + 1]], ta[off[b]:off[b + 1]], K)
        ref = g["cost_final"][b][:, off[b]:off[b + 1]]
        np.testing.assert_allclose(C.numpy(), ref, rtol=1e-6, atol=1e-5)
    assert list(losses) == list(g["loss_keys"])
    np.testing.assert_allclose([float(v) for v in losses.values()], g["loss_vals"], rtol=1e-5, atol=1e-6)
    total = sum(losses.values())
    grads = torch.autograd.grad(total, [h[0] for h in heads] + [h[1] for h in heads])
    H = len(heads)
    for i in range(H):
        np.testing.assert_allclose(grads[i].numpy(), g[f"grad_logits{i}"], rtol=1e-5, atol=1e-6)
        np.testing.assert_allclose(grads[H + i].numpy(), g[f"grad_kps{i}"], rtol=1e-5, atol=1e-6)


def test_criterion_scope_errors():
    from detrpose_amd.criterion import Criterion, HungarianMatcher
    m = HungarianMatcher(2.0, 0.25, 10.0, 4.0)
    with pytest.raises(NotImplementedError):
        Criterion(2, m, {"loss_vfl": 2.0}, ["vfl", "local"], 17)
    c = Criterion(2, m, {"loss_vfl": 2.0}, ["vfl"], 17)
    with pytest.raises(AssertionError):   # criterion.py:313-314: the aux heads are required
        c({"pred_logits": None, "dn_meta": {}}, [])
    with pytest.raises(NotImplementedError):
        HungarianMatcher(num_body_points=5)


# ---------------------------------------------------------------- GPU: HIP kernels

def _hip_run(g, device="cuda"):
    from detrpose_amd.criterion import Criterion, HungarianMatcher
    K, ncls, n_aux = int(g["K"]), int(g["ncls"]), int(g["n_aux"])
    heads = _inputs(g, device, requires_grad=True)
    targets = _targets(g, device)
    m = HungarianMatcher(cost_class=2.0, focal_alpha=0.25, cost_keypoints=10.0, cost_oks=4.0, num_body_points=K)
    crit = Criterion(ncls, m, {"loss_vfl": 2.0, "loss_keypoints": 10.0, "loss_oks": 4.0}, ["vfl", "keypoints"], K)
    losses = crit(_outputs(heads, n_aux), targets)
    return crit, m, heads, targets, losses


@pytest.mark.gpu
@pytest.mark.parametrize("name", CASES)
def test_hip_criterion_golden(golden_dir, name):
    g = _load(golden_dir, name)
    crit, m, heads, targets, losses = _hip_run(g)
    match, go, _ = crit.last_match
    assert np.array_equal(match.cpu().numpy(), g["match"]), "per-head matchings differ from the reference"
    assert np.array_equal(go.cpu().numpy(), g["go"]), "union matching differs from the reference"
    assert list(losses) == list(g["loss_keys"])
    got = torch.stack(list(losses.values())).detach().cpu().numpy()
    np.testing.assert_allclose(got, g["loss_vals"], rtol=1e-5, atol=1e-6)
    total = sum(losses.values())
    H = len(heads)
    grads = torch.autograd.grad(total, [h[0] for h in heads] + [h[1] for h in heads])
    for i in range(H):
        for got_g, key in ((grads[i], f"grad_logits{i}"), (grads[H + i], f"grad_kps{i}")):
            ref = g[key]
            scale = max(np.abs(ref).max(), 1e-12)
            err = np.abs(got_g.cpu().numpy() - ref).max()
            assert err <= 1e-5 * scale + 1e-7, (key, err, scale)
    # the reference's matcher API: list of (query_idx, target_idx) per image, queries ascending
    with torch.no_grad():
        idx = m({"pred_logits": heads[0][0], "pred_keypoints": heads[0][1]}, targets)
    for b, (I, J) in enumerate(idx):
        want = np.nonzero(g["match"][0, b] >= 0)[0]
        assert np.array_equal(I.numpy(), want) and np.array_equal(J.numpy(), g["match"][0, b][want])
    # the cost matrix of the final head vs the reference's (per image block)
    from detrpose_amd.criterion import pack_targets
    packed = pack_targets(targets, int(g["K"]), "cuda")
    _, cost = m.match([heads[0][0].detach()], [heads[0][1].detach()], packed, cost_out=True)
    off = np.concatenate([[0], np.cumsum(g["sizes"])])
    for b in range(len(g["sizes"])):
        n = off[b + 1] - off[b]
        if n:
            np.testing.assert_allclose(cost[0, b, :, :n].cpu().numpy(), g["cost_final"][b][:, off[b]:off[b + 1]],
                                       rtol=1e-5, atol=1e-5)


def _random_case(B, Q, K, sizes, seed, dyadic=False):
    g = torch.Generator().manual_seed(seed)
    H = 8
    heads = []
    for _ in range(H):
        lg = torch.randn(B, Q, 2, generator=g) * 2
        kp = torch.sigmoid(torch.randn(B, Q, 2 * K, generator=g) * 2)
        if dyadic:
            kp = (kp * 4).round() / 4
        heads.append((lg, kp))
    tl, tk, ta = [], [], []
    for n in sizes:
        xy = torch.rand(n, 2 * K, generator=g)
        vis = (torch.rand(n, K, generator=g) > 0.3).float()
        if dyadic:
            xy = (xy * 4).round() / 4
            vis = torch.zeros(n, K)
            vis[:, 0] = 1.0
        tl.append(torch.randint(0, 2, (n,), generator=g))
        tk.append(torch.cat([xy, vis], 1))
        ta.append(torch.rand(n, generator=g) * 0.3 + 0.002)
    return heads, torch.cat(tl), torch.cat(tk), torch.cat(ta)


@pytest.mark.gpu
def test_hip_criterion_b64_vs_oracle():
    """L training batch per GPU: 64 images x 60 queries, 0..20 people per image."""
    from detrpose_amd.criterion import Criterion, HungarianMatcher
    B, Q, K = 64, 60, 17
    sizes = [int(x) for x in np.random.default_rng(5).integers(0, 21, B)]
    heads, tl, tk, ta = _random_case(B, Q, K, sizes, 21)
    ref_losses, ref_match, ref_go = oc.criterion([(a.clone().requires_grad_(True), b.clone().requires_grad_(True))
                                                  for a, b in heads], np.array(sizes), tl, tk, ta, K, 2, 5)
    dh = [(a.cuda().requires_grad_(True), b.cuda().requires_grad_(True)) for a, b in heads]
    off = np.concatenate([[0], np.cumsum(sizes)])
    targets = [{"labels": tl[off[b]:off[b + 1]].cuda(), "keypoints": tk[off[b]:off[b + 1]].cuda(),
                "area": ta[off[b]:off[b + 1]].cuda()} for b in range(B)]
    crit = Criterion(2, HungarianMatcher(2.0, 0.25, 10.0, 4.0), {"loss_vfl": 2.0, "loss_keypoints": 10.0,
                                                                 "loss_oks": 4.0}, ["vfl", "keypoints"], K)
    losses = crit(_outputs(dh, 5), targets)
    match, go, _ = crit.last_match
    assert np.array_equal(match.cpu().numpy(), ref_match)
    assert np.array_equal(go.cpu().numpy(), ref_go)
    np.testing.assert_allclose([float(v) for v in losses.values()], [float(v) for v in ref_losses.values()],
                               rtol=2e-5, atol=1e-6)


@pytest.mark.gpu
def test_hip_match_ties_vs_scipy_rule():
    """Costs from dyadic keypoints with one visible joint and only the L1 term: exact f32
    values with many ties, so the matching is decided by the LSAP tie-breaks."""
    from detrpose_amd.criterion import pack_targets, match_heads
    B, Q, K = 16, 60, 17
    sizes = [int(x) for x in np.random.default_rng(9).integers(1, 30, B)]
    heads, tl, tk, ta = _random_case(B, Q, K, sizes, 33, dyadic=True)
    off = np.concatenate([[0], np.cumsum(sizes)])
    targets = [{"labels": tl[off[b]:off[b + 1]].cuda(), "keypoints": tk[off[b]:off[b + 1]].cuda(),
                "area": ta[off[b]:off[b + 1]].cuda()} for b in range(B)]
    packed = pack_targets(targets, K, "cuda")
    got = match_heads([h[0].cuda() for h in heads], [h[1].cuda() for h in heads], packed, K, 0.0, 1.0, 0.0,
                      0.25).cpu().numpy()
    for h, (lg, kp) in enumerate(heads):
        want = oc.match(lg, kp, np.array(sizes), tl, tk, ta, K, cost_class=0.0, cost_kp=1.0, cost_oks=0.0)
        assert np.array_equal(got[h], want), h
