"""Multi-rank sharding logic on CPU with the gloo backend (world_size 2), no GPU."""
import os
import socket

import numpy as np
import pytest
import torch.distributed as dist
import torch.multiprocessing as mp

from gobeansdb_amd import shard


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from oracle import oracle as O
        first, n = shard.weak_shard(rank, 8)
        # each rank decodes its own shard with the CPU oracle (the checker) and
        # contributes bytes, a status count and an output digest
        nbytes, digest, bad = 0, 0, 0
        for bid in range(first, first + n):
            blk = O.gen_text(7, bid, 1000 + 37 * bid)
            st, out = O.decompress(O.compress(blk))
            bad += int(st != 0 or out != blk)
            nbytes += len(out)
            digest ^= O.crc32_write(0xFFFFFFFF, out) ^ 0xFFFFFFFF
        tot = shard.sum_over_ranks({"bytes": nbytes, "bad": bad, "blocks": n})
        slow = shard.max_over_ranks([0.5 + rank, 10.0 - rank])
        dg = shard.xor_digest_over_ranks(digest)
        q.put((rank, tot, slow, dg))
    finally:
        dist.destroy_process_group()


def test_two_rank_shard_reductions():
    world, port = 2, _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    from oracle import oracle as O
    exp_bytes = sum(1000 + 37 * b for b in range(16))
    exp_dg = 0
    for b in range(16):
        exp_dg ^= O.crc32_write(0xFFFFFFFF, O.gen_text(7, b, 1000 + 37 * b)) ^ 0xFFFFFFFF
    for rank, tot, slow, dg in res:
        assert tot == {"bytes": exp_bytes, "bad": 0, "blocks": 16}
        assert slow == [1.5, 10.0]
        assert dg == exp_dg


@pytest.mark.parametrize("world", [1, 2, 3, 8])
def test_partition_by_bytes_balanced_and_contiguous(world):
    rng = np.random.default_rng(5)
    sizes = np.exp(rng.uniform(np.log(4096), np.log(65536), 1000)).astype(np.int64)
    parts = shard.partition_by_bytes(sizes, world)
    assert parts[0][0] == 0 and parts[-1][1] == len(sizes)
    assert all(parts[i][1] == parts[i + 1][0] for i in range(world - 1))
    tot = sizes.sum()
    for lo, hi in parts:
        assert abs(sizes[lo:hi].sum() - tot / world) <= sizes.max()


def test_partition_fewer_records_than_ranks():
    parts = shard.partition_by_bytes([100, 100], 4)
    assert parts[0][0] == 0 and parts[-1][1] == 2
    assert sum(hi - lo for lo, hi in parts) == 2
