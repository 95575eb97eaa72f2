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


def _data_files():
    """The reference's golden records.data, and a generated file with corrupt regions (nextValid
    resyncs), a failed compressed body and a truncated tail."""
    import random
    import struct
    from oracle import oracle as O
    from oracle import replay as R
    here = os.path.dirname(os.path.abspath(__file__))
    golden = open(os.path.join(here, "golden", "records.data"), "rb").read()
    rng = random.Random(77)
    out = b""
    for i in range(80):
        n = int(np.exp(rng.uniform(np.log(5), np.log(20000))))
        val = O.gen_text(rng.getrandbits(32), i, n) if rng.random() < 0.7 else O.gen_image(rng.getrandbits(32), i, n)
        flag = 0
        if n > 256 and rng.random() < 0.6:
            c = O.compress(val)
            if len(c) < 0.9 * n:
                val, flag = c, R.FLAG_COMPRESS
        out += R.make_record(b"key_%016x" % rng.getrandbits(64), val, flag=flag, ver=i % 5, ts=i)
    out += R.make_record(b"kbad", b"\x4f" + bytes(40), flag=R.FLAG_COMPRESS)
    d = bytearray(out)
    for _ in range(6):
        d[rng.randrange(len(d))] ^= 0x5A
    d = bytes(d[: len(d) - 300])  # truncated inside the last record
    assert struct.unpack_from("<I", d, 0) is not None
    return [golden, d]


def _cut_points(data):
    """Starts of records read with no gap before them (sizeBroken 0): where a file may be cut."""
    from oracle import replay as R
    rows, _ = R.replay(data)
    return [r[0] for r in rows if r[1] == 0]


def _data_worker(rank, world, port, q, files):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from oracle import oracle as O
        from oracle import replay as R
        plan = shard.partition_data_files([(_cut_points(f), len(f)) for f in files], world)
        rows, ends, digest = [], [], 0
        for f, lo, hi in plan[rank]:
            # this rank replays only its byte range of the file, as a stream of its own
            got, err = R.replay(files[f][lo:hi])
            rows += [(f, off + lo) + tuple(rest) for off, *rest in got]
            ends.append((f, hi, err is not None))
            for r in got:
                digest ^= O.crc32_write(0xFFFFFFFF, r[5]) ^ 0xFFFFFFFF
        gathered = [None] * world
        dist.all_gather_object(gathered, (rows, ends))
        q.put((rank, plan, gathered, shard.xor_digest_over_ranks(digest)))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_data_files_split_over_ranks_equal_whole_replay(world):
    """A corpus of two .data files split over gloo ranks on record boundaries
    (shard.partition_data_files): the union of the ranks' replays, in rank order, equals
    oracle/replay.py over each whole file (offsets, sizeBroken, keys, versions, flags, values,
    vhash), the unexpected-EOF error appears only where a file ends, and the all-gathered XOR
    of the value CRCs equals the whole-corpus digest."""
    from oracle import oracle as O
    from oracle import replay as R
    files = _data_files()
    port = _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_data_worker, args=(r, world, port, q, files)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=180) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    exp_rows, exp_digest, exp_err = [], 0, {}
    for f, data in enumerate(files):
        rows, err = R.replay(data)
        exp_rows += [(f,) + tuple(r) for r in rows]
        exp_err[f] = err is not None
        for r in rows:
            exp_digest ^= O.crc32_write(0xFFFFFFFF, r[5]) ^ 0xFFFFFFFF
    assert any(r[2] for r in exp_rows), "the corpus has resyncs"
    for rank, plan, gathered, dg in res:
        assert dg == exp_digest
        assert all(len(p) > 0 for p in plan), "every rank got a share"
        union = [row for rows, _ in gathered for row in rows]
        assert union == exp_rows
        for rows, ends in gathered:
            for f, hi, err in ends:
                assert err == (exp_err[f] and hi == len(files[f]))


def test_partition_data_files_tiles_each_file():
    rng = np.random.default_rng(3)
    files = []
    for k in range(6):
        sizes = rng.integers(1, 40, 0 if k == 2 else rng.integers(1, 60)) * 256
        off = np.concatenate([[0], np.cumsum(sizes)[:-1]]) if len(sizes) else np.zeros(0, np.int64)
        files.append((off, int(sizes.sum())))
    for world in (1, 2, 4, 7, 16):
        plan = shard.partition_data_files(files, world)
        assert len(plan) == world
        cover = {}
        for pieces in plan:
            for f, lo, hi in pieces:
                assert lo < hi and lo % 256 == 0 and (hi % 256 == 0)
                assert lo in set(files[f][0].tolist()) | {0}
                cover.setdefault(f, []).append((lo, hi))
        for f, (off, size) in enumerate(files):
            segs = sorted(cover.get(f, []))
            if size == 0:
                assert segs == []
                continue
            assert segs[0][0] == 0 and segs[-1][1] == size
            assert all(a[1] == b[0] for a, b in zip(segs, segs[1:]))
