"""Multi-GPU data parallelism for KRRN inference.

Crops are independent at inference (eval BN, no batch statistics), so one process per GPU
runs full batches of its own crops and the only collective is one all-gather of fixed-size
per-crop pose records (64 B/crop: R 9, t 3, pred_t 3, inliers 1, as f32) over RCCL
(torch.distributed backend "nccl" is RCCL on ROCm; over xGMI). At B = 32-64 crops/GPU that is
a 2-4 KB message per rank: latency-bound, one step, no bucketing needed. Crops of different
square sizes S (LineMOD test crops snap to a 40-px grid, batchdataset.py:890-923) are bucketed
by S and each bucket split contiguously across ranks so every rank runs full batches of one S.
"""
from __future__ import annotations

import os
from collections import defaultdict
from typing import Dict, List, Optional, Sequence, Tuple

import torch
import torch.distributed as dist

RECORD = 16  # f32 per crop


def init_from_env(backend: Optional[str] = None):
    """One process per GPU (torchrun). Returns (rank, world, local_rank)."""
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1 and not dist.is_initialized():
        if backend is None:
            backend = "nccl" if torch.cuda.is_available() else "gloo"
        if backend == "nccl":
            torch.cuda.set_device(local)
            dist.init_process_group(backend, device_id=torch.device("cuda", local))
        else:
            dist.init_process_group(backend)
    return rank, world, local


def shard_range(n: int, world: int, rank: int) -> Tuple[int, int]:
    """Contiguous split of n items; the first n % world ranks get one extra."""
    q, r = divmod(n, world)
    lo = rank * q + min(rank, r)
    return lo, lo + q + (1 if rank < r else 0)


def bucket_shard(sizes: Sequence[int], world: int, rank: int) -> Dict[int, List[int]]:
    """Bucket crop indices by crop size, then split every bucket contiguously across ranks.
    Returns {S: [global crop indices owned by `rank`]} (buckets in ascending S)."""
    buckets: Dict[int, List[int]] = defaultdict(list)
    for i, s in enumerate(sizes):
        buckets[int(s)].append(i)
    out = {}
    for s in sorted(buckets):
        lo, hi = shard_range(len(buckets[s]), world, rank)
        if hi > lo:
            out[s] = buckets[s][lo:hi]
    return out


def pack_records(R: torch.Tensor, t: torch.Tensor, pred_t: Optional[torch.Tensor], inliers: torch.Tensor,
                 out: Optional[torch.Tensor] = None) -> torch.Tensor:
    B = R.shape[0]
    if out is None:
        out = torch.zeros((B, RECORD), dtype=torch.float32, device=R.device)
    out[:, 0:9].copy_(R.reshape(B, 9))
    out[:, 9:12].copy_(t.reshape(B, 3))
    if pred_t is not None:
        out[:, 12:15].copy_(pred_t.reshape(B, 3))
    out[:, 15].copy_(inliers.reshape(B))
    return out


def gather_records(rec: torch.Tensor, group=None) -> torch.Tensor:
    """All-gather [B, 16] records from every rank -> [world * B, 16] (rank-major)."""
    if not dist.is_initialized() or dist.get_world_size(group) == 1:
        return rec
    world = dist.get_world_size(group)
    out = torch.empty((world * rec.shape[0], rec.shape[1]), dtype=rec.dtype, device=rec.device)
    if dist.get_backend(group) == "nccl":
        dist.all_gather_into_tensor(out, rec.contiguous(), group=group)
    else:
        parts = list(out.chunk(world))
        dist.all_gather(parts, rec.contiguous(), group=group)
        out = torch.cat(parts)
    return out


def allreduce_max(x: float, device) -> float:
    if not dist.is_initialized():
        return x
    t = torch.tensor([x], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())
