"""GC rewrite of a .data chunk on the GPU.

Host mirror of the data movement of GCMgr.gc (store/gc.go:268-353) for one source
chunk resident in device memory: the records the stream reader returns (their offsets
come from qlzx_replay_index, gobeansdb_amd/replay.py) are filtered by the caller's
liveness mask -- the HTree / hint / collision lookups that decide isNewest are out of
scope -- and every kept record is appended to the destination in order, as
dataChunk.AppendRecordGC -> WriteRecord.append (store/datachunk.go:56-79,
store/datafile.go:307-330) does: header re-encoded with its CRC recomputed over
header[4:24] ‖ key ‖ value (store/datafile.go:66-88), zero padding to 256 B, and a new
destination chunk whenever recsize + writingHead > DataFileMax (store/gc.go:320-332).

The destination offsets are an exclusive scan of the kept records' padded sizes with
those rotations (host, one pass over the sizes); the copies (qlzx_copy_batch) and the
CRCs (qlzx_crc32_batch over the copied records) run in libqlzx.so.  The rewritten
CRC must equal the stored one (the reader verified it); `crc_mismatch` counts the
records where it does not, which would mean a corrupted copy.
"""
from __future__ import annotations

from dataclasses import dataclass

import numpy as np
import torch

from . import _lib, batch
from .record import _copy, _dev_u32, _dev_u64
from .replay import HDR

DATA_FILE_MAX = 4000 << 20   # store/config_default.go:39


@dataclass
class GCResult:
    chunks: list[torch.Tensor]   # destination chunk bytes (device), each from its starting head on
    chunk: np.ndarray            # int32 [kept] destination chunk index of each kept record
    offset: np.ndarray           # uint64 [kept] offset in that chunk (absolute, from the chunk's start)
    crc: np.ndarray              # uint32 [kept] recomputed record CRCs
    crc_mismatch: int            # kept records whose recomputed CRC differs from the stored one


def chunk_head(c: int, dst_head: int, next_heads) -> int:
    """Starting writingHead of destination chunk c: dst_head for the first, next_heads[c - 1]
    for later ones (0 past the list).  beginGCWriting starts a destination at its current size
    unless it is the source chunk being rewritten (store/datachunk.go:185-193)."""
    if c == 0:
        return int(dst_head)
    return int(next_heads[c - 1]) if c - 1 < len(next_heads) else 0


def plan(recsize: np.ndarray, dst_head: int = 0, data_file_max: int = DATA_FILE_MAX, next_heads=()):
    """Destination (chunk, offset) of records of padded size `recsize` appended in order from
    dst_head, rotating when recsize + head > data_file_max (store/gc.go:320); destination
    chunk c >= 1 starts at chunk_head(c)."""
    n = len(recsize)
    chunk = np.zeros(n, np.int32)
    off = np.zeros(n, np.uint64)
    i, c, head = 0, 0, int(dst_head)
    rs = recsize.astype(np.int64)
    while i < n:
        # the longest run from i that fits without rotating, by a cumulative sum
        cs = np.cumsum(rs[i:]) + head
        fit = int(np.searchsorted(cs, data_file_max, side="right"))
        if fit == 0:          # this record starts a new chunk
            c += 1
            head = chunk_head(c, dst_head, next_heads)
            cs = np.cumsum(rs[i:]) + head
            fit = max(1, int(np.searchsorted(cs, data_file_max, side="right")))
        chunk[i:i + fit] = c
        off[i:i + fit] = (cs[:fit] - rs[i:i + fit]).astype(np.uint64)
        head = int(cs[fit - 1])
        i += fit
    return chunk, off


def rewrite(data: torch.Tensor, rec_off: torch.Tensor, keep: torch.Tensor, dst_head: int = 0,
            data_file_max: int = DATA_FILE_MAX, stream=None, next_heads=()) -> GCResult:
    """Rewrite the kept records of the chunk `data` (record offsets `rec_off` in reader order,
    bool mask `keep`) into destination chunks: the first starts at dst_head, chunk c >= 1 at
    next_heads[c - 1] (0 past the list).  chunks[c] holds the bytes written from that head on."""
    dev = data.device
    ko = rec_off[keep].to(torch.int64)
    n = int(ko.numel())
    if n == 0:
        return GCResult([torch.zeros(0, dtype=torch.uint8, device=dev)], np.zeros(0, np.int32),
                        np.zeros(0, np.uint64), np.zeros(0, np.uint32), 0)
    hidx = ko.unsqueeze(1) + torch.arange(HDR, device=dev).unsqueeze(0)
    hdr = data[hidx.reshape(-1)].reshape(n, HDR).contiguous().view(torch.int32).cpu().numpy().view(np.uint32)
    stored_crc, ksz, vsz = hdr[:, 0], hdr[:, 4].astype(np.int64), hdr[:, 5].astype(np.int64)
    size = HDR + ksz + vsz                                    # Record.Sizes (store/item.go:219-222)
    recsize = (size + 255) // 256 * 256
    chunk, off = plan(recsize, dst_head, data_file_max, next_heads)
    src_off = ko.cpu().numpy().view(np.uint64)
    chunks = []
    for c in range(int(chunk[-1]) + 1):
        sel = np.nonzero(chunk == c)[0]
        base = chunk_head(c, dst_head, next_heads)
        end = int(off[sel[-1]] + recsize[sel[-1]]) if len(sel) else base
        buf = torch.zeros(max(end - base, 1), dtype=torch.uint8, device=dev)[: end - base]
        if len(sel):   # record bytes; the zero padding is the fresh buffer's (datafile.go:322-327)
            _copy(data, src_off[sel], size[sel].astype(np.uint32), buf, off[sel] - np.uint64(base), stream)
        chunks.append(buf)
    # encodeHeader/getCRC over each rewritten record, written into its header
    crc = np.zeros(n, np.uint32)
    for c, buf in enumerate(chunks):
        sel = np.nonzero(chunk == c)[0]
        if not len(sel):
            continue
        local = off[sel] - np.uint64(chunk_head(c, dst_head, next_heads))
        got = batch.crc32(batch.BlockBatch(buf, _dev_u64(local + np.uint64(4), dev),
                                           _dev_u32((size[sel] - 4).astype(np.uint32), dev)), stream=stream)
        buf.view(torch.int32)[torch.from_numpy((local // 4).astype(np.int64)).to(dev)] = got
        crc[sel] = got.cpu().numpy().view(np.uint32)
    return GCResult(chunks, chunk, off, crc, int((crc != stored_crc).sum()))
