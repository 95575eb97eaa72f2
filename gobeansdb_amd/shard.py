"""Sharding of independent blocks/records across ranks (one process per GPU).

The codec path has no cross-block state (quicklz.h:27, QLZ_STREAMING_BUFFER=0),
so ranks never exchange data: each owns a contiguous shard and the only
collectives are the end-of-run reductions below (RCCL over xGMI on the GPU box,
gloo in the CPU tests).  DESIGN.md §7.
"""
from __future__ import annotations

import os

import numpy as np
import torch
import torch.distributed as dist


def env_rank() -> tuple[int, int, int]:
    """(rank, world_size, local_rank) from the torch.distributed.run environment."""
    return (int(os.environ.get("RANK", "0")), int(os.environ.get("WORLD_SIZE", "1")),
            int(os.environ.get("LOCAL_RANK", "0")))


def weak_shard(rank: int, blocks_per_rank: int) -> tuple[int, int]:
    """Weak scaling: rank r owns synthetic block ids [r*n, (r+1)*n)."""
    return rank * blocks_per_rank, blocks_per_rank


def partition_by_bytes(sizes, world: int) -> list[tuple[int, int]]:
    """Split records 0..len(sizes) into `world` contiguous [lo, hi) ranges with
    near-equal byte totals (balance by csize + dsize on record
    boundaries).  Empty ranges are allowed when there are fewer records than ranks."""
    sizes = np.asarray(sizes, dtype=np.int64)
    n = len(sizes)
    if world <= 1:
        return [(0, n)]
    cum = np.concatenate([[0], np.cumsum(sizes)])
    total = int(cum[-1])
    cuts = [0]
    for r in range(1, world):
        target = total * r / world
        cuts.append(int(np.searchsorted(cum, target, side="left")))
    cuts.append(n)
    cuts = np.maximum.accumulate(np.minimum(np.asarray(cuts), n))
    return [(int(cuts[r]), int(cuts[r + 1])) for r in range(world)]


def max_over_ranks(values: list[float], device=None) -> list[float]:
    """Element-wise max of per-rank timings (bench contract: the slowest rank counts)."""
    if not (dist.is_available() and dist.is_initialized()) or dist.get_world_size() == 1:
        return list(values)
    t = torch.tensor(values, dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return [float(x) for x in t.cpu()]


def sum_over_ranks(counters: dict[str, int], device=None) -> dict[str, int]:
    """Sum of per-rank counters (bytes, blocks, status counts, CRC failures)."""
    keys = sorted(counters)
    if not (dist.is_available() and dist.is_initialized()) or dist.get_world_size() == 1:
        return dict(counters)
    t = torch.tensor([counters[k] for k in keys], dtype=torch.int64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.SUM)
    return {k: int(v) for k, v in zip(keys, t.cpu())}


def xor_digest_over_ranks(digest: int, device=None) -> int:
    """XOR of per-rank 32-bit digests (e.g. XOR of per-block output CRCs) for parity spot checks."""
    if not (dist.is_available() and dist.is_initialized()) or dist.get_world_size() == 1:
        return digest & 0xFFFFFFFF
    t = torch.tensor([digest & 0xFFFFFFFF], dtype=torch.int64, device=device)
    out = [torch.zeros_like(t) for _ in range(dist.get_world_size())]
    dist.all_gather(out, t)
    x = 0
    for o in out:
        x ^= int(o.item())
    return x
