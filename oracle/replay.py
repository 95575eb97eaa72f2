"""CPU restatement of the .data replay path -- TEST INFRASTRUCTURE ONLY.

Follows the sequential reader of the reference line by line (pure Python, for
the small fixtures of tests/):

  DataStreamReader.Next       store/datafile.go:228-277
  DataStreamReader.nextValid  store/datafile.go:202-226
  readRecordAt                store/datafile.go:114-170
  WriteRecord.getCRC          store/datafile.go:66-76 (crc32 of header[4:24] ‖ key ‖ value)
  Record.Sizes                store/item.go:219-222 (24 + ksz + vsz, padded to 256)
  IsValidKeySize/ValueSize    config/mc_config.go:33-39 (1 <= ksz <= 250, vsz <= BodyMax=50M)
  buildHintFromData           store/bucket.go:89-117 (Decompress, then Getvhash of the body)
  Payload.Decompress          store/item.go:163-176 (errors swallowed: body stays compressed)
  Getvhash                    store/item.go:89-100
  Fnv1a (sign-extending)      utils/hash.go:8-16

Only tests/ import this module; the product path is gobeansdb_amd/replay.py.
"""
from __future__ import annotations

import struct
from dataclasses import dataclass

from . import oracle as O

HDR = 24
PADDING = 256
FLAG_COMPRESS = 0x00010000
MAX_KEY_LEN = 250
BODY_MAX = 50 << 20


@dataclass
class Rec:
    offset: int
    crc: int
    ts: int
    flag: int
    ver: int
    key: bytes
    body: bytes
    size_broken: int

    @property
    def rsize(self) -> int:
        return (HDR + len(self.key) + len(self.body) + 255) >> 8 << 8


def _hdr(data: bytes, off: int):
    crc, ts, flag, ver, ksz, vsz = struct.unpack_from("<IIIiII", data, off)
    return crc, ts, flag, ver, ksz, vsz


def _valid_sizes(ksz: int, vsz: int, max_key: int, body_max: int) -> bool:
    return 0 < ksz <= max_key and vsz <= body_max


def read_record_at(data: bytes, off: int, max_key=MAX_KEY_LEN, body_max=BODY_MAX):
    """readRecordAt (store/datafile.go:114-170): the record at `off`, or None."""
    if off + HDR > len(data):
        return None
    crc, ts, flag, ver, ksz, vsz = _hdr(data, off)
    if not _valid_sizes(ksz, vsz, max_key, body_max):
        return None
    if off + HDR + ksz + vsz > len(data):  # ReadAt short read
        return None
    key = data[off + HDR: off + HDR + ksz]
    body = data[off + HDR + ksz: off + HDR + ksz + vsz]
    if O.record_crc(data[off + 4: off + HDR], key, body) != crc:
        return None
    return Rec(off, crc, ts, flag, ver, key, body, 0)


class StreamReader:
    """DataStreamReader over an in-memory chunk file."""

    def __init__(self, data: bytes, start: int = 0, max_key=MAX_KEY_LEN, body_max=BODY_MAX):
        self.data, self.offset, self.max_key, self.body_max = data, start, max_key, body_max

    def _next_valid(self):
        # store/datafile.go:202-226; the sizeBroken accumulated in Next() is
        # not carried over (nextValid's named result starts at 0)
        off2 = self.offset & ~0xFF
        broken = 0
        while off2 < len(self.data):
            r = read_record_at(self.data, off2, self.max_key, self.body_max)
            if r is not None:
                self.offset = off2 + r.rsize
                r.size_broken = broken
                return r, off2, broken, None
            broken += 256
            off2 += 256
            self.offset = off2
        return None, off2, broken, None

    def next(self):
        """(rec | None, offset, sizeBroken, err) as DataStreamReader.Next returns them."""
        d, p = self.data, self.offset
        if p >= len(d):
            return None, 0, 0, None                      # io.EOF -> err = nil
        if p + HDR > len(d):
            return None, 0, 0, "unexpected EOF"           # partial header
        crc, ts, flag, ver, ksz, vsz = _hdr(d, p)
        if not _valid_sizes(ksz, vsz, self.max_key, self.body_max):
            return self._next_valid()
        if p + HDR + ksz + vsz > len(d):
            return None, 0, 0, "unexpected EOF"           # io.ReadFull of key/body
        key = d[p + HDR: p + HDR + ksz]
        body = d[p + HDR + ksz: p + HDR + ksz + vsz]
        if O.record_crc(d[p + 4: p + HDR], key, body) != crc:
            return self._next_valid()
        r = Rec(p, crc, ts, flag, ver, key, body, 0)
        self.offset = p + r.rsize
        return r, p, 0, None


def stream_all(data: bytes, start: int = 0, max_key=MAX_KEY_LEN, body_max=BODY_MAX):
    """Every Next() result until the reader returns no record; (records, end_err)."""
    rd = StreamReader(data, start, max_key, body_max)
    out = []
    while True:
        r, off, broken, err = rd.next()
        if err is not None:
            return out, err
        if r is None:
            return out, None
        out.append(r)


def fnv1a(buf: bytes) -> int:
    """utils/hash.go:8-16: FNV-1a with the historical sign-extension of each byte."""
    h = 0x811C9DC5
    for b in buf:
        h ^= (b - 256 if b >= 128 else b) & 0xFFFFFFFF
        h = (h * 0x01000193) & 0xFFFFFFFF
    return h


def getvhash(value: bytes) -> int:
    """store/item.go:89-100."""
    n = len(value)
    h = (n * 97) & 0xFFFFFFFF
    if n <= 1024:
        h = (h + fnv1a(value)) & 0xFFFFFFFF
    else:
        h = (h + fnv1a(value[:512])) & 0xFFFFFFFF
        h = (h * 97) & 0xFFFFFFFF
        h = (h + fnv1a(value[n - 512:])) & 0xFFFFFFFF
    return h & 0xFFFF


def replay(data: bytes, start: int = 0, max_key=MAX_KEY_LEN, body_max=BODY_MAX):
    """buildHintFromData (store/bucket.go:89-117) minus the hint/htree writes:
    per record (offset, sizeBroken, key, ver, flag_after, value_after, vhash)."""
    recs, err = stream_all(data, start, max_key, body_max)
    rows = []
    for r in recs:
        flag, body = r.flag, r.body
        if flag & FLAG_COMPRESS:
            # CDecompressSafe (quicklz/cquicklz.go:84-101): size check, then decode
            st, out = O.decompress(body)
            if st == O.OK:
                flag, body = flag - FLAG_COMPRESS, out
        rows.append((r.offset, r.size_broken, r.key, r.ver, flag, body, getvhash(body)))
    return rows, err


def make_record(key: bytes, body: bytes, flag: int = 0, ver: int = 0, ts: int = 0) -> bytes:
    """WriteRecord.append with padding (store/datafile.go:78-88,307-330)."""
    tail = struct.pack("<IIiII", ts, flag, ver, len(key), len(body))
    crc = O.record_crc(tail, key, body)
    rec = struct.pack("<I", crc) + tail + key + body
    pad = (-len(rec)) % PADDING
    return rec + bytes(pad)
