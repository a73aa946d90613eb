"""Multi-GPU data parallelism for the batched dynamics.

The path shards trivially: every configuration is independent, so each rank (one process
per GPU) evaluates its own batch and no collective touches the data path.  The only
collective is the one-time model broadcast: rank 0 parses the URDF and broadcasts the
packed fp64 model blob (multibody_export_blob, ~1.2 KB for FR3) -- over RCCL/xGMI with
the "nccl" backend on GPUs, over gloo in the CPU tests -- and every other rank rebuilds
a bit-identical Multibody from it (multibody_new_from_blob).  Timing uses max-over-ranks.
"""
from __future__ import annotations

import numpy as np
import torch
import torch.distributed as dist


def broadcast_model(make_model, rank: int, world: int, device):
    """Rank 0 calls make_model(); the blob is broadcast; all ranks return a Multibody."""
    from . import ffi

    if rank == 0:
        mb = make_model()
        blob = torch.as_tensor(mb.blob(), dtype=torch.float64, device=device)
        size = torch.tensor([blob.numel()], dtype=torch.int64, device=device)
    else:
        mb = None
        size = torch.zeros(1, dtype=torch.int64, device=device)
    if world > 1:
        dist.broadcast(size, 0)
        if rank != 0:
            blob = torch.empty(int(size.item()), dtype=torch.float64, device=device)
        dist.broadcast(blob, 0)
        if rank != 0:
            mb = ffi.Multibody.from_blob(blob.cpu().numpy())
    return mb


def shard(total: int, rank: int, world: int):
    """Contiguous SoA slice [start, stop) of `total` configurations for `rank`
    (strong-scaling split; sizes differ by at most one)."""
    base, rem = divmod(total, world)
    start = rank * base + min(rank, rem)
    return start, start + base + (1 if rank < rem else 0)


def rank_seed(seed: int, rank: int) -> int:
    """Independent synthetic input streams per rank (weak scaling)."""
    return seed + 7919 * rank


def max_over_ranks(values, world: int, device):
    """Element-wise max of a list of floats across ranks (timing: slowest rank wins)."""
    t = torch.tensor(list(values), dtype=torch.float64, device=device)
    if world > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return t.tolist()


def gather_over_ranks(values, world: int, device):
    """Every rank's list of floats, in rank order (per-rank device / wall times)."""
    t = torch.tensor(list(values), dtype=torch.float64, device=device)
    if world == 1:
        return [t.tolist()]
    out = [torch.zeros_like(t) for _ in range(world)]
    dist.all_gather(out, t)
    return [o.tolist() for o in out]


def sum_over_ranks(values, world: int, device):
    t = torch.tensor(list(values), dtype=torch.float64, device=device)
    if world > 1:
        dist.all_reduce(t, op=dist.ReduceOp.SUM)
    return t.tolist()


def gather_checksums(x: np.ndarray, world: int, device):
    """All ranks' float64 checksums of their outputs (used to verify shards differ and
    are finite without moving the data)."""
    c = torch.tensor([float(np.sum(x)), float(np.sum(np.abs(x)))], dtype=torch.float64, device=device)
    if world == 1:
        return [c.tolist()]
    out = [torch.zeros_like(c) for _ in range(world)]
    dist.all_gather(out, c)
    return [o.tolist() for o in out]
