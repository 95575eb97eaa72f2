"""CPU restatement of the GC rewrite of one .data chunk -- TEST INFRASTRUCTURE ONLY.

Follows the reference loop record by record (pure Python, small fixtures):

  GCMgr.gc record loop           store/gc.go:268-353 (liveness = the caller's keep list;
                                 the HTree / hint / collision lookups that decide it are out of scope)
  wrapRecord                     store/datafile.go:38-45 (RecSize = Record.Sizes padded size)
  rotation at DataFileMax        store/gc.go:320-332 (recsize + writingHead > DataFileMax)
  beginGCWriting                 store/datachunk.go:185-199 (rewrite from 0, or append at size)
  dataChunk.AppendRecordGC       store/datachunk.go:56-79
  WriteRecord.append             store/datafile.go:307-330 (encodeHeader + getCRC, zero padding)

Only tests/ import this module; the product path is gobeansdb_amd/gc.py.
"""
from __future__ import annotations

import struct

from . import oracle as O
from .replay import HDR, PADDING, stream_all


def append(rec) -> bytes:
    """WriteRecord.append(wbuf, dopadding=true) of a record read back by the stream reader."""
    tail = struct.pack("<IIiII", rec.ts, rec.flag, rec.ver, len(rec.key), len(rec.body))  # encodeHeader
    crc = O.record_crc(tail, rec.key, rec.body)                                           # getCRC
    out = struct.pack("<I", crc) + tail + rec.key + rec.body
    return out + bytes((-len(out)) % PADDING)


def gc_rewrite(data: bytes, keep, data_file_max: int, dst_head: int = 0, next_heads=()):
    """Kept records of `data` (keep[i] for the i-th record the reader returns), rewritten in
    order: returns (chunks, positions) with chunks[j] = the bytes written into the j-th
    destination chunk and positions[i] = (chunk index, offset) of each kept record.  The first
    destination chunk starts at dst_head, destination chunk j >= 1 at next_heads[j - 1]
    (0 past the list): beginGCWriting appends at the chunk's size unless it rewrites the
    source chunk itself (store/datachunk.go:185-193)."""
    recs, _ = stream_all(data)
    chunks = [bytearray()]
    head = dst_head
    pos = []
    for r, k in zip(recs, keep):
        if not k:
            continue                                      # gc.go:310-313 (not isNewest)
        recsize = (HDR + len(r.key) + len(r.body) + 255) >> 8 << 8
        if recsize + head > data_file_max:                # gc.go:320: next destination chunk
            chunks.append(bytearray())
            j = len(chunks) - 1
            head = next_heads[j - 1] if j - 1 < len(next_heads) else 0
        b = append(r)
        pos.append((len(chunks) - 1, head))
        chunks[-1] += b
        head += recsize
    return [bytes(c) for c in chunks], pos
