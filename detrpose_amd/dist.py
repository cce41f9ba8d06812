"""Data-parallel inference across the GPUs of one node.

Images are independent, so the forward shards by image: every rank (one process per GPU,
launched by torch.distributed.run) holds a full replica of the weights and forwards its own
slice of the global batch; the only exchange is one RCCL all_gather_into_tensor of the
fixed-size outputs over xGMI (8,640 B/img: pred_logits (60,2) + pred_keypoints (60,17,2)
fp32). There is no collective inside the forward.

The per-rank output buffer is the plan's `out_flat` = [logits (B*60*2) | keypoints
(B*60*17*2)]; `unflatten` turns the gathered [rank0 out_flat | rank1 out_flat | ...] back
into global-batch tensors in rank order (rank r holds images shard(global, r, world)).
"""
from __future__ import annotations

import os

import torch
import torch.distributed as dist


def env_ranks() -> tuple[int, int, int]:
    """(rank, world_size, local_rank) from the torch.distributed.run environment."""
    return (int(os.environ.get("RANK", "0")), int(os.environ.get("WORLD_SIZE", "1")),
            int(os.environ.get("LOCAL_RANK", "0")))


def init(backend: str = "nccl", shared_gpu: bool = False) -> tuple[int, int, torch.device]:
    """Initialise the process group when launched with WORLD_SIZE > 1 (backend 'nccl' is
    RCCL on ROCm; 'gloo' for CPU tests). Returns (rank, world, device).
    shared_gpu: rehearsal of the N-rank path on a one-GPU box -- every rank computes on
    cuda:0 and the collectives run on gloo with host staging (RCCL refuses two ranks on one
    GPU); it checks the launcher, plan/graph per rank, barriers and the gather order on real
    kernels, and is never a scaling measurement."""
    rank, world, local = env_ranks()
    if shared_gpu:
        backend = "gloo"
        torch.cuda.set_device(0)
        dev = torch.device("cuda", 0)
    elif backend == "nccl":
        torch.cuda.set_device(local)
        dev = torch.device("cuda", local)
    else:
        dev = torch.device("cpu")
    if world > 1 and not dist.is_initialized():
        kw = {"device_id": dev} if backend == "nccl" else {}
        dist.init_process_group(backend, **kw)
    return rank, world, dev


def _host_staged() -> bool:
    return dist.is_initialized() and dist.get_backend() == "gloo"


def shard(global_batch: int, rank: int, world: int) -> tuple[int, int]:
    """(start, count) of this rank's images. The global batch must split evenly: every rank
    runs the same captured plan shape, and all_gather_into_tensor needs equal parts."""
    if world < 1 or not 0 <= rank < world:
        raise ValueError(f"bad rank {rank} / world {world}")
    if global_batch % world:
        raise ValueError(f"global batch {global_batch} does not split evenly over {world} ranks")
    per = global_batch // world
    return rank * per, per


def gather_outputs(out_flat: torch.Tensor, world: int, out: torch.Tensor | None = None) -> torch.Tensor:
    """All-gather every rank's flat output buffer (rank order)."""
    if world == 1:
        return out_flat
    if out is None:
        out = torch.empty(world * out_flat.numel(), dtype=out_flat.dtype, device=out_flat.device)
    if out_flat.is_cuda and _host_staged():
        # gloo has no device buffers: gather host copies, then one upload (shared-GPU rehearsal)
        host = out_flat.cpu()
        parts = [torch.empty_like(host) for _ in range(world)]
        dist.all_gather(parts, host)
        out.copy_(torch.cat(parts))
        return out
    dist.all_gather_into_tensor(out, out_flat)
    return out


def flatten_outputs(outputs: dict) -> torch.Tensor:
    """{'pred_logits','pred_keypoints'} -> the plan's out_flat layout (host-side mirror)."""
    return torch.cat([outputs["pred_logits"].reshape(-1).float(), outputs["pred_keypoints"].reshape(-1).float()])


def unflatten(gathered: torch.Tensor, world: int, batch_per_rank: int, num_queries: int = 60,
              num_classes: int = 2, num_kp: int = 17) -> dict:
    """Gathered [rank][logits | keypoints] buffers -> global {'pred_logits','pred_keypoints'}."""
    per = batch_per_rank * num_queries * (num_classes + 2 * num_kp)
    if gathered.numel() != world * per:
        raise ValueError(f"gathered buffer has {gathered.numel()} values, expected {world * per}")
    g = gathered.view(world, per)
    nl = batch_per_rank * num_queries * num_classes
    logits = g[:, :nl].reshape(world * batch_per_rank, num_queries, num_classes)
    kps = g[:, nl:].reshape(world * batch_per_rank, num_queries, num_kp, 2)
    return {"pred_logits": logits, "pred_keypoints": kps}


def max_over_ranks(value: float, world: int, device: torch.device) -> float:
    """Slowest rank's value (the bench's whole-job time)."""
    if world == 1:
        return float(value)
    t = torch.tensor([value], dtype=torch.float64, device="cpu" if _host_staged() else device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())
