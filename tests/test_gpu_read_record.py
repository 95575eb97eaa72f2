"""GPU: one GET's record read in one request (qlzx_read_record1 via replay.read_record) against the
oracle's readRecordAt + CDecompressSafe restatement (oracle/replay.py, store/datafile.go:114-170,
store/item.go:163-176), on the reference-pinned golden records.data and on generated records of
every size class the service and the general path take, with corrupted CRCs and bodies."""
import random
import struct

import numpy as np
import pytest

from oracle import oracle as O
from oracle import replay as R

pytestmark = pytest.mark.gpu


def _expect(rec: bytes):
    r = R.read_record_at(rec, 0)
    if r is None:
        return None
    flag, body = r.flag, bytes(r.body)
    if flag & R.FLAG_COMPRESS:
        st, dec = O.decompress(body)
        if st == O.OK:
            flag, body = flag - R.FLAG_COMPRESS, dec
    return flag, body


def _records(data: bytes):
    rows, _ = R.replay(data)
    out = []
    for off, *_ in rows:
        ksz, vsz = struct.unpack_from("<II", data, off + 16)
        out.append(data[off:off + 24 + ksz + vsz])
    return out


def test_read_record_golden(cuda, golden):
    from gobeansdb_amd import replay
    recs = _records(golden.records_data)
    assert recs
    for rec in recs:
        assert replay.read_record(rec) == _expect(rec)


def test_read_record_sizes_and_corruption(cuda):
    from gobeansdb_amd import replay
    rng = random.Random(66)
    for n in (0, 1, 100, 300, 4096, 16384, 40000, 65536, 70000, 200000):
        for kind in ("text", "rand"):
            v = O.gen_text(66, n, n) if kind == "text" else bytes(rng.getrandbits(8) for _ in range(n))
            c = O.compress(v) if n else b""
            for body, flag in ((v, 0), (c, R.FLAG_COMPRESS)):
                if flag and not body:
                    continue
                rec = R.make_record(b"key_%d" % n, body, flag=flag, ver=3)
                assert replay.read_record(rec) == _expect(rec), (n, kind, flag)
                bad = bytearray(rec)
                bad[0] ^= 1                     # stored CRC off by a bit
                assert replay.read_record(bytes(bad)) is None
                if len(body) > 20:
                    bad = bytearray(rec)
                    bad[24 + len(b"key_%d" % n) + len(body) // 2] ^= 0x40   # body bit flip
                    assert replay.read_record(bytes(bad)) is None
