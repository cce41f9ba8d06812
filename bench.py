"""Throughput (and bs=1 latency) benchmark of the DETRPose inference forward on MI355X.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--size l] [--batch 64]
    python -m torch.distributed.run --nnodes=1 --nproc-per-node N --master-addr 127.0.0.1 \
        --master-port P bench.py --gpus N --steps K --warmup W

Metric (BASELINE.json): images/sec + p50 ms/img, DETRPose-L bf16 640x640, batch 64 per
GPU. One step = one forward of the HIP plan over one resident batch of synthetic
640x640 images + PostProcess (the reference benchmark's Model = model + postprocessor,
tools/benchmark/torch_benchmark.py:82-91), replayed as one hipGraph; with N>1 ranks
each rank forwards its own batch (data parallel, weak scaling) and the outputs are
all-gathered over RCCL (one all_gather_into_tensor of 8,640 B/img). Rank 0 prints one
JSON line. Weights: seeded fan-in random init (no checkpoint offline); data synthetic.

`--gpus N` with no torch.distributed environment starts `torch.distributed.run` with N
ranks as a child process (before anything touches the GPU) and exits with its code; a
run whose world size differs from --gpus fails.

Also reported (rank 0):
  roofline      the dominant kernel: the kernel instantiation with the most device time per
                step (dp_conv2d launches are named by the dispatcher, dp_conv2d_describe),
                bound by its own launches' algorithmic bytes vs FLOPs; achieved = their
                FLOPs (or bytes) / their HIP-event time. `traffic` = measured HBM bytes of
                those launches from the committed rocprofv3 PMC passes, quoted only when
                they were taken on this exact source (detrpose_amd.build.source_hash).
                Beside it the dp_conv2d family and the per-launch bound over every launch;
  latency_bs1   the reference's latency protocol (torch_benchmark.py:29-51): batch 1,
                400 warm-up and 1000 timed Model(images, sizes) calls (hipGraph replay,
                synchronised each), mean of the fastest 100 and the median;
  secondary     DETRPose-N bf16 batch 32 (BASELINE configs[1]) and DETRPose-X bf16 batch 32
                (the per-GPU shard of configs[3]) throughput;
  cpu_baseline  the CPU oracle restatement (oracle/detrpose_cpu.py, kind "port") at
                batch 1 and 8 (2 warm-up + 5 timed) on the host cores (N=1 only).
"""
from __future__ import annotations

import argparse
import json
import os
import socket
import statistics
import subprocess
import sys
import time

import torch

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, REPO)

PEAK_BF16_TFLOPS = 2500.0   # MI355X dense bf16 MFMA (MI355X_MICROARCH.md; no sparsity)
PEAK_F32_TFLOPS = 157.3
PEAK_HBM_GBS = 8000.0
METRIC = "images/sec + p50 ms/img, DETRPose-L bf16 640x640 at 1/2/4/8 MI355X"
PMC_FILE = "profiles/pmc_traffic.json"


def parse(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--size", default="l", choices=["n", "l", "x"])
    ap.add_argument("--batch", type=int, default=64, help="images per GPU")
    ap.add_argument("--dtype", default="bf16", choices=["bf16", "fp32"])
    ap.add_argument("--no-graph", action="store_true")
    ap.add_argument("--cpu-baseline-seconds", type=float, default=25.0, help="cap on the CPU baseline leg")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-latency", action="store_true")
    ap.add_argument("--no-gemm-peak", action="store_true", help="skip the measured bf16 GEMM peak (BASELINE.md's "
                    "denominator of the end-to-end MFMA fraction)")
    ap.add_argument("--no-secondary", action="store_true")
    ap.add_argument("--no-train", action="store_true", help="skip the training-step leg (BASELINE configs[4])")
    ap.add_argument("--train-batch", type=int, default=16, help="images per GPU of the training-step leg")
    ap.add_argument("--train-steps", type=int, default=10)
    ap.add_argument("--latency-runs", type=int, default=1000)
    ap.add_argument("--latency-warmup", type=int, default=400)
    ap.add_argument("--profile-ops", type=str, default="", help="write per-op times (JSON) to this path")
    ap.add_argument("--shared-gpu-rehearsal", action="store_true",
                    help="N>1 on a one-GPU box: every rank on cuda:0, gloo collectives with host staging "
                         "(checks the N-rank path on real kernels; not a scaling number)")
    ap.add_argument("--cpu-dry-run", action="store_true",
                    help="test hook: gloo on CPU with a stub step (checks launch, world size and gather order)")
    return ap.parse_args(argv)


# ----------------------------------------------------------------------------- launch


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def maybe_spawn(a) -> int | None:
    """--gpus N>1 outside torch.distributed.run: run N ranks as a child torchrun (no GPU
    call has happened in this process yet) and return its exit code."""
    if a.gpus <= 1 or "WORLD_SIZE" in os.environ:
        return None
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={a.gpus}",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), os.path.abspath(__file__),
           *sys.argv[1:]]
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    return subprocess.run(cmd, env=env).returncode


# ----------------------------------------------------------------------------- legs


def pmc_traffic(a, kernel, launches):
    """Measured HBM bytes per step of one kernel instantiation from the committed rocprofv3 PMC
    passes (scripts/pmc_traffic.py), only if they were taken on this exact source and
    workload; otherwise (None, reason)."""
    from detrpose_amd.build import source_hash
    path = os.path.join(REPO, PMC_FILE)
    if not os.path.exists(path):
        return None, "no PMC profile committed"
    d = json.load(open(path))
    if d.get("source_hash") != source_hash():
        return None, f"PMC profile is for source {d.get('source_hash')}, this is {source_hash()}: not quoted"
    if tuple(d.get("workload", ())) != (a.size, a.batch, a.dtype):
        return None, "PMC profile is for another workload"
    k = d.get("kernels", {}).get(kernel)
    if not k or round(k["launches"]) != launches:
        return None, "PMC profile has no entry with this launch count for the kernel"
    return round(k["total_bytes"]), f"rocprofv3 PMC FETCH_SIZE x2 + WRITE_SIZE ({PMC_FILE}, source {d['source_hash']})"


def cpu_baseline(size, cap_seconds):
    """Oracle (CPU fp32 restatement of the reference forward) on host cores at batch 1 and
    8, 2 warm-up + 5 timed forwards each, bounded by cap_seconds."""
    from detrpose_amd import build_model
    from detrpose_amd.configs import get_config
    from detrpose_amd.synthetic import load_synthetic, synthetic_images
    from oracle.detrpose_cpu import OracleDETRPose
    cores = len(os.sched_getaffinity(0))
    cores = min(cores, int(os.environ.get("OMP_NUM_THREADS", cores)))
    torch.set_num_threads(cores)
    m, _ = build_model(size)
    load_synthetic(m, 0)
    orc = OracleDETRPose(get_config(size), m.state_dict())
    res, t_start = {}, time.perf_counter()
    for bs in (1, 8):
        img = synthetic_images(bs, 1)
        for _ in range(2):
            orc(img)
        ts = []
        for _ in range(5):
            t0 = time.perf_counter()
            orc(img)
            ts.append(time.perf_counter() - t0)
            if time.perf_counter() - t_start > cap_seconds and len(ts) >= 2:
                break
        res[bs] = (bs * len(ts) / sum(ts), len(ts))
    best = max(res, key=lambda b: res[b][0])
    return {"value": round(res[best][0], 3), "unit": "images/sec", "cores": cores, "kind": "port",
            "by_batch": {str(b): round(v[0], 3) for b, v in res.items()},
            "sample": f"DETRPose-{size.upper()} fp32 CPU oracle (oracle/detrpose_cpu.py, torch CPU ops, {cores} "
                      f"threads), batch 1 and 8, 2 warm-up + " + " / ".join(f"{v[1]} timed at b{b}"
                                                                                for b, v in res.items())
                      + f"; value = best batch (b{best})"}


def _bound(nbytes, flops, peak):
    """(bound kind, lower-bound ms) of algorithmic bytes / FLOPs on MI355X."""
    t_hbm = nbytes / (PEAK_HBM_GBS * 1e9)
    t_mfma = flops / (peak * 1e12)
    return ("hbm" if t_hbm >= t_mfma else "mfma"), max(t_hbm, t_mfma) * 1e3


def roofline_report(a, plan, op_ms, op_fn, peak):
    """Roofline of the dominant kernel: the kernel instantiation (Plan.kernel_of: rocprofv3's
    canonical name) with the most device time per step, bound by its own launches'
    algorithmic bytes vs FLOPs. Beside it: the dp_conv2d family (rounds 1-3's line), and the
    per-launch bound max(bytes / HBM peak, FLOPs / MFMA peak) summed over EVERY launch of the
    step (each op records its algorithmic bytes and FLOPs, Plan.cost)."""
    kern = {n: plan.kernel_of(n) for n in op_ms}
    groups = {}
    for n, ms in op_ms.items():
        g = groups.setdefault(kern[n], {"ms": 0.0, "bytes": 0.0, "flops": 0.0, "launches": 0, "ops": []})
        g["ms"] += ms
        g["bytes"] += plan.op_bytes[n]
        g["flops"] += plan.op_flops[n]
        g["launches"] += 1
        g["ops"].append(n)
    dom = max(groups, key=lambda k: groups[k]["ms"])
    g = groups[dom]
    kind, lb = _bound(g["bytes"], g["flops"], peak)
    gbs = g["bytes"] / (g["ms"] * 1e-3) / 1e9
    tfs = g["flops"] / (g["ms"] * 1e-3) / 1e12
    traffic, traffic_note = pmc_traffic(a, dom, g["launches"])
    total_ms = sum(op_ms.values())
    per_op = {n: _bound(plan.op_bytes[n], plan.op_flops[n], peak)[1] for n in op_ms}
    conv = [n for n in op_ms if op_fn[n] == "dp_conv2d"]
    c_ms = sum(op_ms[n] for n in conv)
    c_b = sum(plan.op_bytes[n] for n in conv)
    c_f = sum(plan.op_flops[n] for n in conv)
    c_kind, _ = _bound(c_b, c_f, peak)
    c_lb = sum(per_op[n] for n in conv)
    top = sorted(groups.items(), key=lambda kv: -kv[1]["ms"])[:8]
    return {
        "bound": kind,
        "kernel": dom,
        "achieved": round(tfs if kind == "mfma" else gbs, 2),
        "peak": peak if kind == "mfma" else PEAK_HBM_GBS,
        "unit": "TFLOP/s" if kind == "mfma" else "GB/s",
        "frac": round(tfs / peak if kind == "mfma" else gbs / PEAK_HBM_GBS, 4),
        "traffic": traffic,
        "traffic_note": traffic_note,
        "launches_per_step": g["launches"],
        "ms_per_step": round(g["ms"], 4),
        "avg_launch_us": round(1e3 * g["ms"] / g["launches"], 2),
        "flops_per_step": g["flops"],
        "algorithmic_bytes_per_step": round(g["bytes"]),
        "achieved_tflops": round(tfs, 2),
        "achieved_gbs": round(gbs, 1),
        "bound_ms": round(lb, 4),
        "how": "achieved = the kernel's algorithmic FLOPs (or bytes) over its launches in one step / their summed "
               "HIP-event time (Plan.profile, median of 3 passes on the launch stream); the same FLOPs x profiled "
               "steps / rocprofv3 TotalDurationNs reproduces it",
        "family": {"kernel": "dp_conv2d family (conv_stream/conv_halo/stem-direct: every dense conv/linear launch)",
                   "bound": c_kind, "ms_per_step": round(c_ms, 3), "launches_per_step": len(conv),
                   "algorithmic_bytes": round(c_b), "achieved_gbs": round(c_b / (c_ms * 1e-3) / 1e9, 1),
                   "achieved_tflops": round(c_f / (c_ms * 1e-3) / 1e12, 2),
                   "hbm_frac": round(c_b / (c_ms * 1e-3) / 1e9 / PEAK_HBM_GBS, 4),
                   "mfma_frac": round(c_f / (c_ms * 1e-3) / 1e12 / peak, 4),
                   "per_launch_bound_ms": round(c_lb, 3), "bound_over_actual": round(c_lb / c_ms, 4)},
        "all_launches": {"ms_per_step": round(total_ms, 3), "launches": len(op_ms),
                         "covered_by_per_op_bounds": round(sum(op_ms[n] for n in op_ms if n in plan.op_bytes)
                                                           / total_ms, 4),
                         "per_launch_bound_ms": round(sum(per_op.values()), 3),
                         "bound_over_actual": round(sum(per_op.values()) / total_ms, 4)},
        "top_kernels": [{"kernel": k, "ms_per_step": round(v["ms"], 3), "launches": v["launches"],
                         "bound": _bound(v["bytes"], v["flops"], peak)[0],
                         "bound_over_actual": round(_bound(v["bytes"], v["flops"], peak)[1] / v["ms"], 4)}
                        for k, v in top],
    }



def synthetic_targets(batch, K=17, seed=3, dev="cuda"):
    """COCO-shaped synthetic targets: 1-6 persons per image, xyxy boxes, keypoints inside the box
    with ~75 % visible, normalised area."""
    g = torch.Generator().manual_seed(seed)
    ts = []
    for b in range(batch):
        n = int(torch.randint(1, 7, (1,), generator=g))
        c = torch.rand(n, 2, generator=g) * 0.6 + 0.2
        wh = torch.rand(n, 2, generator=g) * 0.3 + 0.05
        xy = (c[:, None] + (torch.rand(n, K, 2, generator=g) - 0.5) * wh[:, None]).clamp(0, 1)
        vis = (torch.rand(n, K, generator=g) > 0.25).float()
        ts.append({"labels": torch.zeros(n, dtype=torch.int64, device=dev),
                   "boxes": torch.cat([c - wh / 2, c + wh / 2], 1).to(dev),
                   "keypoints": torch.cat([xy.flatten(1), vis], 1).to(dev), "area": (wh.prod(1) * 0.53).to(dev)})
    return ts


def train_leg(size, dtype, dev, batch, steps, warmup=3, rank=0, world=1):
    """BASELINE configs[4]: the training step of detrpose_amd.train.Trainer (scope 'full') on this
    rank's shard of `batch` images: backbone forward (FrozenBatchNorm2d), encoder training forward
    (BatchNorm batch statistics, SyncBN across ranks), transformer training forward with
    OKS-denoising queries, criterion (matching, losses and their gradients; num_boxes all-reduced),
    transformer / encoder / backbone backward — per sub-batch of the config's grad_accum_steps —,
    DDP's gradient mean (one all-reduce of the flat f32 gradient), clip_grad_norm_ + AdamW +
    ModelEMA. Timed like the inference line: barrier + synchronize around `steps` steps, the
    slowest rank's time. Then one instrumented step times every collective (synchronised: a
    separate number, not part of ms_per_step) and HIP events split one sub-batch into phases."""
    from detrpose_amd import build_model, encoder_train
    from detrpose_amd.synthetic import load_synthetic, synthetic_images
    from detrpose_amd.train import Trainer
    from detrpose_amd import dist as dp
    model, _ = build_model(size, dtype=dtype)
    load_synthetic(model, 0)
    tr = Trainer(model, dtype=dtype, device=dev)
    images = synthetic_images(batch, seed=11 + rank).to(dev)
    ts = synthetic_targets(batch, seed=3 + rank, dev=dev)
    for _ in range(warmup):
        tr.step(images, ts)
    torch.cuda.synchronize()
    if world > 1:
        dp.dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        keys, vals = tr.step(images, ts)
    torch.cuda.synchronize()
    if world > 1:
        dp.dist.barrier()
    torch.cuda.synchronize()
    own = time.perf_counter() - t0
    el = dp.max_over_ranks(own, world, dev)
    ms = el * 1e3 / steps
    graphs = None
    if tr.graphs:   # the same steps with every tape launched op by op from Python (no hipGraph replay)
        tr.graphs = False
        tr.step(images, ts)
        torch.cuda.synchronize()
        t1 = time.perf_counter()
        for _ in range(steps):
            tr.step(images, ts)
        torch.cuda.synchronize()
        eager = (time.perf_counter() - t1) * 1e3 / steps
        tr.graphs = True
        tr.step(images, ts)   # tapes back on their graphs for the phase split below
        torch.cuda.synchronize()
        graphs = {"tapes_replayed_from_hipgraphs": True, "eager_ms_per_step": round(eager, 3),
                  "graph_ms_per_step": round(ms, 3), "eager_over_graph": round(eager / ms, 3)}
    comm = None
    if world > 1:   # one instrumented step: every collective synchronised and timed
        encoder_train.COMM_LOG = []
        torch.cuda.synchronize()
        t1 = time.perf_counter()
        tr.step(images, ts)
        torch.cuda.synchronize()
        inst = time.perf_counter() - t1
        log, encoder_train.COMM_LOG = encoder_train.COMM_LOG, None
        big = max(log, key=lambda x: x[0])
        comm = {"collectives_per_step": len(log), "ms_in_collectives": round(sum(x[1] for x in log) * 1e3, 3),
                "instrumented_step_ms": round(inst * 1e3, 3),
                "grad_allreduce_bytes": big[0], "grad_allreduce_ms": round(big[1] * 1e3, 3),
                "backend": dp.dist.get_backend()}
    # phase split of one more sub-batch (HIP events around each phase; on every rank, whose
    # SyncBN collectives pair up)
    plan = tr.plan
    bb, ep = tr.bb, tr.ep
    sub = batch // tr.grad_accum_steps
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(10)]
    ev[0].record()
    bb.forward()
    ev[1].record()
    ep.forward()
    ev[2].record()
    plan.forward()
    ev[3].record()
    from detrpose_amd.criterion import pack_targets
    from detrpose_amd.train import dn_meta
    packed = pack_targets(ts[batch - sub:], 17, dev)
    plan.criterion(packed, packed.sizes, dn_meta(packed.sizes)[1])
    ev[4].record()
    plan.backward()
    ev[5].record()
    ep.backward()
    ev[6].record()
    bb.backward()
    ev[7].record()
    tr.eng.optimizer_step(**tr.opt)
    tr.eng.ema_update(**tr.ema)
    ev[8].record()
    torch.cuda.synchronize()
    names = ["backbone_fwd", "encoder_fwd", "transformer_fwd", "criterion", "transformer_bwd", "encoder_bwd",
             "backbone_bwd", "clip+adamw+ema"]
    phases = {n: round(ev[i].elapsed_time(ev[i + 1]), 3) for i, n in enumerate(names)}
    fl = {"backbone": sum(bb.op_flops.values()), "encoder": sum(ep.op_flops.values()),
          "transformer": sum(plan.op_flops.values())}
    t = {"backbone": phases["backbone_fwd"] + phases["backbone_bwd"],
         "encoder": phases["encoder_fwd"] + phases["encoder_bwd"],
         "transformer": phases["transformer_fwd"] + phases["transformer_bwd"]}
    cfg = tr.opt
    out = {"workload": f"DETRPose-{size.upper()} training step (BASELINE configs[4]) on {world} GPU(s), {batch} "
                       f"images per GPU in grad_accum_steps={tr.grad_accum_steps} sub-batches of {sub}: backbone "
                       f"(FrozenBN) + encoder (BatchNorm batch statistics{', SyncBN' if world > 1 else ''}) + "
                       f"transformer with OKS-denoising queries, criterion (incl. dn_* losses), full backward, "
                       f"{'DDP gradient mean, ' if world > 1 else ''}clip_grad_norm_({cfg['max_norm']}) + AdamW "
                       f"(backbone lr {cfg['backbone_lr']:g}) + ModelEMA; {dtype}, synthetic targets (1-6 persons "
                       f"per image)",
           "n_gpus": world, "ms_per_step": round(ms, 3), "images_per_sec": round(batch * world / ms * 1e3, 2),
           "images_per_sec_per_gpu": round(batch / ms * 1e3, 2), "steps": steps, "grad_accum_steps": tr.grad_accum_steps,
           "dn_pad_last_sub_batch": plan.P, "hipgraphs": graphs, "phase_ms_one_sub_batch": phases,
           "tflops_by_part": {k: round(fl[k] / (t[k] * 1e-3) / 1e12, 2) if t[k] > 0 else None for k in fl},
           "sub_batch_tflop": round(sum(fl.values()) / 1e12, 3),
           "losses_finite": bool(torch.isfinite(vals).all()), "update_skipped": tr.eng.step_skipped()}
    if comm is not None:
        out["collectives"] = comm
    return out


def gemm_peak(dev, n=8192, reps=20):
    """BASELINE.md's denominator for the end-to-end MFMA fraction: the bf16 GEMM rate this GPU
    reaches on a large square product (torch.matmul = hipBLASLt, n^3, median of reps launches
    timed with HIP events, after warm-up). Timed outside the benchmark's region."""
    torch.manual_seed(0)
    x = torch.randn(n, n, device=dev, dtype=torch.bfloat16)
    y = torch.randn(n, n, device=dev, dtype=torch.bfloat16)
    for _ in range(5):
        torch.matmul(x, y)
    torch.cuda.synchronize()
    ts = []
    for _ in range(reps):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        torch.matmul(x, y)
        e1.record()
        torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1))
    ms = statistics.median(ts)
    del x, y
    return {"tflops": round(2.0 * n ** 3 / (ms * 1e-3) / 1e12, 1), "shape": f"{n}x{n}x{n} bf16",
            "how": "torch.matmul (hipBLASLt), median of %d launches, HIP events" % reps}


def latency_bs1(model, pp, dev, runs, warmup):
    """tools/benchmark/torch_benchmark.py:29-51 on the HIP path: Model(images, sizes) at
    batch 1 (one hipGraph replay incl. the input copy), synchronised around every call."""
    from detrpose_amd.export import DeployModel
    from detrpose_amd.synthetic import synthetic_images
    dm = DeployModel(model, pp)
    img = synthetic_images(1, seed=7).to(dev)
    size = torch.tensor([[640, 640]], device=dev)
    for _ in range(warmup):
        dm.replay(img, size)
    ts = []
    for _ in range(runs):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        dm.replay(img, size)
        torch.cuda.synchronize()
        ts.append(time.perf_counter() - t0)
    srt = sorted(ts)
    fast = srt[:100]
    return {"mean_fastest100_ms": round(1e3 * sum(fast) / len(fast), 4),
            "p50_ms": round(1e3 * statistics.median(ts), 4), "runs": runs, "warmup": warmup,
            "protocol": "torch_benchmark.py:29-51 (bs=1, Model = model + PostProcess, hipGraph replay)"}


def throughput(model, dev, batch, steps, warmup, seed=1):
    """Images/s of graph replays over one resident batch (single-rank secondary configs)."""
    from detrpose_amd.synthetic import synthetic_images
    plan = model.engine(dev).plan(batch)
    plan.input.copy_(synthetic_images(batch, seed=seed).to(dev))
    g = plan.graph()
    for _ in range(warmup):
        g.replay()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        g.replay()
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    out = plan.out_flat
    return batch * steps / el, bool(torch.isfinite(out).all())


# ----------------------------------------------------------------------------- main


def cpu_dry_run(a):
    """Test hook for the N-rank launch: gloo on CPU, a stub 'forward' that writes each
    image's rank/index into the out_flat layout, the same all-gather + unflatten as the GPU
    path; prints the JSON line (n_gpus = world) with the gather check."""
    from detrpose_amd import dist as dp
    rank, world, dev = dp.init("gloo")
    if world != a.gpus:
        raise SystemExit(f"bench: world size {world} != --gpus {a.gpus}")
    per = a.batch
    flat = torch.empty(per * 60 * (2 + 34))
    t0 = time.perf_counter()
    for _ in range(a.warmup + a.steps):
        flat.fill_(float(rank))
        g = dp.gather_outputs(flat, world)
    el = dp.max_over_ranks(time.perf_counter() - t0, world, dev)
    outs = dp.unflatten(g, world, per)
    ok = all(bool((outs["pred_logits"][r * per:(r + 1) * per] == r).all()) for r in range(world))
    if rank == 0:
        print(json.dumps({"metric": METRIC, "value": round(per * a.steps * world / el, 2), "unit": "images/sec",
                          "n_gpus": world, "steps": a.steps, "warmup": a.warmup, "dry_run": "cpu-gloo",
                          "gather_check": "ok" if ok else "FAILED"}), flush=True)
    if world > 1:
        dp.dist.barrier()
        dp.dist.destroy_process_group()
    if not ok:
        raise SystemExit(1)


def main():
    a = parse()
    rc = maybe_spawn(a)
    if rc is not None:
        sys.exit(rc)
    if a.cpu_dry_run:
        return cpu_dry_run(a)
    from detrpose_amd import dist as dp
    rank, world, dev = dp.init("nccl", shared_gpu=a.shared_gpu_rehearsal)
    if world != a.gpus:
        raise SystemExit(f"bench: torch.distributed world size {world} != --gpus {a.gpus}")
    dist = dp.dist if world > 1 else None

    from detrpose_amd import GFLOP_PER_IMAGE, build_model
    from detrpose_amd.synthetic import load_synthetic, synthetic_images

    model, pp = build_model(a.size, dtype=a.dtype)
    load_synthetic(model, 0)
    model.deploy()
    eng = model.engine(dev)
    plan = eng.plan(a.batch)
    plan.add_postprocess()
    plan.input.copy_(synthetic_images(a.batch, seed=1 + rank).to(dev))   # resident in HBM before timing
    gathered = None
    if dist is not None:
        gathered = torch.empty(world * plan.out_flat.numel(), dtype=torch.float32, device=dev)

    def step():
        if a.no_graph:
            plan.run(post=True)
        else:
            g.replay()
        if dist is not None:
            dp.gather_outputs(plan.out_flat, world, gathered)

    g = None if a.no_graph else plan.graph()
    for _ in range(a.warmup):
        step()
    torch.cuda.synchronize()
    if dist is not None:
        dist.barrier()
    torch.cuda.synchronize()
    evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(a.steps)]
    t0 = time.perf_counter()
    for e0, e1 in evs:
        e0.record()
        step()
        e1.record()
    torch.cuda.synchronize()
    if dist is not None:
        dist.barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    step_ms = [e0.elapsed_time(e1) for e0, e1 in evs]
    elapsed = dp.max_over_ranks(elapsed, world, dev)
    total_imgs = a.batch * a.steps * world
    value = total_imgs / elapsed
    ms_per_step = elapsed * 1000.0 / a.steps
    p50_ms_img = statistics.median(step_ms) / a.batch
    finite = bool(torch.isfinite(plan.out_flat).all())
    if dist is not None:
        finite = bool(torch.isfinite(gathered).all())

    if rank == 0:
        # per-op HIP-event pass over the same plan (outside the timed region)
        op_ms = plan.profile(reps=3)
        op_fn = {nm: f.__name__ for nm, f, _ in plan.ops + plan.post_ops}
        peak = PEAK_BF16_TFLOPS if a.dtype == "bf16" else PEAK_F32_TFLOPS
        roofline = roofline_report(a, plan, op_ms, op_fn, peak)
        fam = {}
        for n, ms in op_ms.items():
            fam[op_fn[n]] = fam.get(op_fn[n], 0.0) + ms
        msda = [n for n in op_ms if n.endswith(".msda")]
        msda_gbs = sum(plan.op_bytes[n] for n in msda) / (sum(op_ms[n] for n in msda) * 1e-3) / 1e9 if msda else None
        if a.profile_ops:
            with open(a.profile_ops, "w") as f:
                json.dump({"op_ms": op_ms, "op_flops": plan.op_flops, "op_bytes": plan.op_bytes,
                           "op_kernel": {n: plan.kernel_of(n) for n in op_ms}}, f, indent=1)
        gflop = GFLOP_PER_IMAGE[a.size]
        out = {
            "metric": METRIC,
            "value": round(value, 2),
            "unit": "images/sec",
            "n_gpus": world,
            "steps": a.steps,
            "warmup": a.warmup,
            "ms_per_step": round(ms_per_step, 3),
            "p50_ms_per_img": round(p50_ms_img, 4),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": a.dtype,
            "data": "synthetic (uniform [0,1) 640x640 images; seeded fan-in random weights, no checkpoint offline)",
            "config": {"workload": f"DETRPose-{a.size.upper()} inference forward + PostProcess, 640x640, "
                                   f"batch {a.batch} per GPU, hipGraph replay", "batch_per_gpu": a.batch,
                       "global_batch": a.batch * world, "image": "640x640", "parallelism": f"dp{world}",
                       "graph": not a.no_graph},
            "outputs_finite": finite,
            "roofline": roofline,
            "e2e_mfma_frac": round(value / world * gflop * 1e9 / (peak * 1e12), 4),
            "gflop_per_image": gflop,
            "kernel_ms_per_step": {k: round(v, 3) for k, v in sorted(fam.items(), key=lambda kv: -kv[1])},
            "msda_algorithmic_gbs": round(msda_gbs, 1) if msda_gbs else None,
        }
        if dist is not None:
            # rank 0's slice of the all-gathered buffer is its own output (rank order kept)
            n0 = plan.out_flat.numel()
            out["gather_rank0_matches"] = bool(torch.equal(gathered[:n0], plan.out_flat))
        if a.shared_gpu_rehearsal:
            out["rehearsal"] = (f"{world} ranks sharing one GPU, gloo collectives with host staging: checks the "
                                "N-rank launch/barrier/gather path on real kernels; not a scaling number")
        if not a.no_gemm_peak:
            # "achieved fraction of the MFMA roofline, computed as img/s x GFLOP/img /
            # measured peak bf16 GEMM FLOP/s" (per GPU)
            gp = gemm_peak(dev)
            out["gemm_peak_measured"] = gp
            out["e2e_frac_of_measured_gemm_peak"] = round(value / world * gflop * 1e9 / (gp["tflops"] * 1e12), 4)
        if world == 1 and not a.no_latency:
            out["latency_bs1"] = latency_bs1(model, pp, dev, a.latency_runs, a.latency_warmup)
        if world == 1 and not a.no_secondary:
            out["secondary"] = []
            for sz, bs, what in (("n", 32, "BASELINE configs[1]"),
                                 ("x", 32, "the per-GPU shard of BASELINE configs[3], X b256 over 8 GPUs")):
                ms, _ = build_model(sz, dtype=a.dtype)
                load_synthetic(ms, 0)
                ms.deploy()
                v, fin = throughput(ms, dev, bs, max(20, a.steps // 2), 5)
                out["secondary"].append({"workload": f"DETRPose-{sz.upper()} {a.dtype} batch {bs} 640x640 ({what})",
                                         "value": round(v, 2), "unit": "images/sec", "outputs_finite": fin})
                del ms
                torch.cuda.empty_cache()
        if world == 1 and not a.no_cpu_baseline:
            out["cpu_baseline"] = cpu_baseline(a.size, a.cpu_baseline_seconds)
    if not a.no_train:
        # every rank runs the training leg (its collectives pair up across ranks); rank 0 reports
        del g
        torch.cuda.empty_cache()
        ts = train_leg(a.size, a.dtype, dev, a.train_batch, a.train_steps, rank=rank, world=world)
        torch.cuda.empty_cache()
    if rank == 0:
        if not a.no_train:
            out["train_step"] = ts
        if not finite:
            out["error"] = "non-finite outputs"
        print(json.dumps(out), flush=True)
    if dist is not None:
        dist.barrier()
        dist.destroy_process_group()
    if not finite:
        sys.exit(1)


if __name__ == "__main__":
    main()
