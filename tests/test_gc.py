"""GC rewrite of a .data chunk: gobeansdb_amd/gc.py against the record-by-record
restatement of store/gc.go:268-353 in oracle/gc.py.

CPU tests pin the destination planner (offsets + DataFileMax rotation) and the oracle itself
on the golden records; GPU tests compare every destination chunk byte for byte, the record
positions and the recomputed CRCs."""
import random

import numpy as np
import pytest

from oracle import gc as G
from oracle import oracle as O
from oracle import replay as R


def _chunk(seed: int, n: int, max_body: int = 3000):
    rnd = random.Random(seed)
    out = bytearray()
    for i in range(n):
        key = b"key_%016x" % (seed * 1000 + i)
        body = O.gen_text(seed, i, rnd.randint(0, max_body)) if rnd.random() < 0.7 else \
            bytes(rnd.getrandbits(8) for _ in range(rnd.randint(0, 600)))
        flag = 0
        if len(body) > 300 and rnd.random() < 0.6:
            body, flag = O.compress(body), R.FLAG_COMPRESS
        out += R.make_record(key, body, flag=flag, ver=rnd.randint(-2, 5), ts=1700000000 + i)
    return bytes(out)


def test_oracle_keep_all_is_identity():
    data = _chunk(1, 40)
    chunks, pos = G.gc_rewrite(data, [True] * 40, data_file_max=1 << 30)
    assert chunks == [data]
    assert [p[0] for p in pos] == [0] * 40


def test_oracle_golden_records(golden):
    data = golden.records_data
    recs, _ = R.stream_all(data)
    keep = [i % 3 != 1 for i in range(len(recs))]
    chunks, pos = G.gc_rewrite(data, keep, data_file_max=1 << 30)
    want = b"".join(data[r.offset:r.offset + r.rsize] for r, k in zip(recs, keep) if k)
    assert chunks == [want]


@pytest.mark.parametrize("seed", [2, 3, 4])
def test_plan_matches_oracle_rotation(seed):
    from gobeansdb_amd import gc
    data = _chunk(seed, 120)
    recs, _ = R.stream_all(data)
    rnd = random.Random(seed)
    keep = [rnd.random() < 0.6 for _ in recs]
    for dfm, head, nxt in ((1 << 30, 0, ()), (4096, 0, ()), (2560, 1024, ()), (700, 0, ()),
                           (4096, 1024, (512, 3840, 256)), (2560, 0, (2048,))):
        _, pos = G.gc_rewrite(data, keep, data_file_max=dfm, dst_head=head, next_heads=nxt)
        rs = np.asarray([r.rsize for r, k in zip(recs, keep) if k], np.int64)
        chunk, off = gc.plan(rs, head, dfm, nxt)
        assert [(int(c), int(o)) for c, o in zip(chunk, off)] == pos, (dfm, head, nxt)


@pytest.mark.gpu
@pytest.mark.parametrize("seed,dfm,head,nxt", [(5, 1 << 30, 0, ()), (6, 8192, 0, ()), (7, 4096, 2048, ()),
                                              (8, 600, 0, ()), (10, 4096, 1024, (512, 3584))])
def test_gpu_rewrite_matches_oracle(seed, dfm, head, nxt):
    import torch
    from gobeansdb_amd import gc, replay
    data = _chunk(seed, 150)
    recs, _ = R.stream_all(data)
    rnd = random.Random(seed)
    keep = [rnd.random() < 0.55 for _ in recs]
    want_chunks, want_pos = G.gc_rewrite(data, keep, data_file_max=dfm, dst_head=head, next_heads=nxt)
    d = torch.from_numpy(np.frombuffer(data, np.uint8).copy()).cuda()
    off, broken, end_err, _, _ = replay.index(d)
    assert off.numel() == len(recs)
    res = gc.rewrite(d, off, torch.tensor(keep, device="cuda"), dst_head=head, data_file_max=dfm, next_heads=nxt)
    torch.cuda.synchronize()
    assert [c.cpu().numpy().tobytes() for c in res.chunks] == want_chunks
    assert [(int(c), int(o)) for c, o in zip(res.chunk, res.offset)] == want_pos
    assert res.crc_mismatch == 0
    assert list(res.crc) == [r.crc for r, k in zip(recs, keep) if k]


@pytest.mark.gpu
def test_gpu_rewrite_nothing_kept():
    import torch
    from gobeansdb_amd import gc, replay
    data = _chunk(9, 10)
    d = torch.from_numpy(np.frombuffer(data, np.uint8).copy()).cuda()
    off = replay.index(d)[0]
    res = gc.rewrite(d, off, torch.zeros(off.numel(), dtype=torch.bool, device="cuda"))
    assert len(res.chunk) == 0 and res.chunks[0].numel() == 0
