"""The replay restatement (oracle/replay.py) against the reference's own tests (CPU)."""
import struct

from oracle import oracle as O
from oracle import replay as R


def _data_broken_file():
    # store/data_test.go:129-148: seven records under key "key"; record 4 is
    # 768 B of 'x' with FLAG_CLIENT_COMPRESS (so it spans 4 slots)
    data = b""
    for i in range(7):
        if i == 4:
            data += R.make_record(b"key", b"x" * (256 * 3), flag=0x10, ver=i)
        else:
            data += R.make_record(b"key", b"value_%d" % i, ver=i)
    d = bytearray(data)
    for start, off in [(0, 16), (1, 20), (2, 24), (3, 24 + 3), (4, 256)]:   # breakdata, :149-153
        d[start * 256 + off] = ord("0")
    return bytes(d)


def test_data_broken_resync_matches_reference_test():
    """store/data_test.go:155-172: first Next() -> value_5 at 8*256 with sizeBroken 8*256,
    then value_6 at 9*256 with sizeBroken 0."""
    rd = R.StreamReader(_data_broken_file())
    rec, off, broken, err = rd.next()
    assert err is None and rec is not None
    assert (off, broken, rec.body) == (8 * 256, 8 * 256, b"value_5")
    rec, off, broken, err = rd.next()
    assert (off, broken, rec.body, err) == (9 * 256, 0, b"value_6", None)
    assert rd.next()[0] is None


def test_golden_records_replay(golden):
    rows, err = R.replay(golden.records_data)
    assert err is None
    assert len(rows) == len(golden.records)
    for row, g in zip(rows, golden.records):
        off, broken, key, ver, flag, body, vh = row
        assert off == g["offset"] and broken == 0 and key == g["key"].encode() and ver == g["ver"]
        raw = golden.records_data[off + 24 + len(key): off + 24 + len(key) + g["vsz"]]
        crc = struct.unpack_from("<I", golden.records_data, off)[0]
        assert crc == g["crc"]
        if g["flag"] & R.FLAG_COMPRESS:
            st, plain = O.decompress(raw)
            assert st == 0 and body == plain and flag == g["flag"] - R.FLAG_COMPRESS
        else:
            assert body == raw and flag == g["flag"]
        assert vh == R.getvhash(body)


def test_fnv1a_sign_extension():
    # bytes >= 0x80 are sign-extended before the xor (utils/hash.go:12)
    assert R.fnv1a(b"") == 0x811C9DC5
    h = (0x811C9DC5 ^ 0x61) * 0x01000193 & 0xFFFFFFFF
    assert R.fnv1a(b"a") == h
    h2 = (0x811C9DC5 ^ 0xFFFFFF80) * 0x01000193 & 0xFFFFFFFF
    assert R.fnv1a(b"\x80") == h2


def test_truncated_and_partial_tail():
    a = R.make_record(b"k1", b"v" * 100)
    b = R.make_record(b"k2", b"w" * 300)
    # file ends inside record b's body: Next() reports an unexpected EOF after a
    recs, err = R.stream_all(a + b[:100])
    assert [r.key for r in recs] == [b"k1"] and err == "unexpected EOF"
    # partial header
    recs, err = R.stream_all(a + b[:10])
    assert len(recs) == 1 and err == "unexpected EOF"
    # garbage slot (invalid ksz) then a record: nextValid skips it
    recs, err = R.stream_all(a + bytes(256) + b)
    assert [(r.offset, r.size_broken) for r in recs] == [(0, 0), (512, 256)] and err is None


def test_fnv1a_reference_kat():
    """store/htree_test.go:18-23 (TestHash): utils.Fnv1a([]byte("test")) == 2949673445."""
    assert R.fnv1a(b"test") == 2949673445
    # bytes >= 0x80 are sign-extended (utils/hash.go:12, h ^= uint32(int8(b))): differs from FNV-1a
    plain = 0x811C9DC5
    for b in b"\xff":
        plain = ((plain ^ b) * 0x01000193) & 0xFFFFFFFF
    assert R.fnv1a(b"\xff") != plain
