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


def partition_data_files(files, world: int) -> list[list[tuple[int, int, int]]]:
    """Split ONE corpus of .data chunk files over `world` ranks on record boundaries (SURVEY
    §8(e): contiguous record ranges balanced by bytes, cut at 256-B record starts).

    files: per file (rec_off, size): the file length and the offsets where a cut may fall, i.e.
    starts of records that follow the previous record with no gap (sizeBroken 0 in the reader,
    store/datafile.go:202-226; a hint file or a host/device pre-scan supplies them).  A file is
    cut only there, so every piece is itself a valid .data stream that DataStreamReader reads
    from its first byte to its last and finds exactly the records, sizeBroken included, that the
    whole-file read finds in that range (a broken region stays with the record after it).
    Returns per rank a list of (file index, lo, hi) byte ranges in corpus order; the ranks'
    pieces tile every file exactly."""
    unit_file, unit_lo, unit_len = [], [], []
    for f, (rec_off, size) in enumerate(files):
        starts = np.asarray(rec_off, dtype=np.int64)
        if len(starts) == 0 or starts[0] != 0:
            starts = np.concatenate([[0], starts])  # bytes before the first record ride with it
        ends = np.concatenate([starts[1:], [int(size)]])
        unit_file.append(np.full(len(starts), f, np.int64))
        unit_lo.append(starts)
        unit_len.append(ends - starts)
    if not unit_file:
        return [[] for _ in range(world)]
    uf, ulo, ul = np.concatenate(unit_file), np.concatenate(unit_lo), np.concatenate(unit_len)
    keep = ul > 0  # an empty file has nothing to replay
    uf, ulo, ul = uf[keep], ulo[keep], ul[keep]
    out = []
    for lo, hi in partition_by_bytes(ul, world):
        # runs of one file inside [lo, hi): a piece each
        cut = lo + 1 + np.nonzero(np.diff(uf[lo:hi]))[0] if hi > lo else np.zeros(0, np.int64)
        starts = np.concatenate([[lo], cut]) if hi > lo else np.zeros(0, np.int64)
        ends = np.concatenate([cut, [hi]]) if hi > lo else np.zeros(0, np.int64)
        out.append([(int(uf[a]), int(ulo[a]), int(ulo[b - 1] + ul[b - 1])) for a, b in zip(starts, ends)])
    return out


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


def xor_of(crcs) -> int:
    """XOR of 32-bit values (a device tensor or an array): one rank's parity digest."""
    a = crcs.cpu().numpy() if isinstance(crcs, torch.Tensor) else np.asarray(crcs)
    return int(np.bitwise_xor.reduce(a.astype(np.int64) & 0xFFFFFFFF)) if a.size else 0


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
