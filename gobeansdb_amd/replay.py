"""Batched replay of a .data chunk on the GPU (SURVEY §8 f1 + f2).

Host mirror of buildHintFromData (store/bucket.go:89-117) over a chunk file
resident in device memory: record discovery with DataStreamReader's nextValid
resync and CRC verify (store/datafile.go:114-277, qlzx_replay_index), value
decompress of FLAG_COMPRESS records (Payload.Decompress, store/item.go:163-176,
errors swallowed as in the reference: the body stays compressed) and the value
hash Getvhash (store/item.go:89-100, qlzx_vhash_batch).  torch tensors are the
device memory; every byte of work runs in libqlzx.so.
"""
from __future__ import annotations

import ctypes
from dataclasses import dataclass

import numpy as np
import torch

from . import _lib, batch

HDR = 24
FLAG_COMPRESS = 0x00010000
MAX_KEY_LEN = 250          # config/mc_config.go:6
BODY_MAX = 50 << 20        # config/mc_config.go:7 ("50M")


@dataclass
class ReplayResult:
    offset: torch.Tensor       # int64 [n] record offsets in the chunk
    size_broken: torch.Tensor  # int32 [n] bytes skipped by the nextValid resync before each record
    header: torch.Tensor       # int32 [n, 6]: crc, ts, flag, ver, ksz, vsz (as stored)
    flag: torch.Tensor         # int32 [n] flag after Payload.Decompress
    value_len: torch.Tensor    # int32 [n] value length after decompress
    vhash: torch.Tensor        # int32 [n] Getvhash of the value (uint16)
    # The FLAG_COMPRESS records only, in record order: their decoder outputs in one packed buffer
    # (lengths = the QuickLZ header dsize, meaningless for a record whose decode failed).  Read a
    # record's value through in_out / val_off (or value(j)), not by position in here.
    values: batch.BlockBatch
    end_error: bool            # the reader stopped on an unexpected EOF after these records
    n_candidates: int
    n_valid: int
    in_out: torch.Tensor       # uint8 [n]: 1 = value in values.data at val_off, 0 = in the chunk at val_off
    val_off: torch.Tensor      # int64 [n] value offset (decoded buffer or chunk, per in_out)
    data: torch.Tensor         # the chunk replayed (val_off's base where in_out is 0)

    @property
    def n(self) -> int:
        return int(self.offset.numel())

    def value(self, j: int) -> bytes:
        """Record j's value after Payload.Decompress (store/item.go:163-176): the decoded bytes, or
        the raw body where the record is not compressed or its decode failed."""
        o, n = int(self.val_off[j]), int(self.value_len[j])
        src = self.values.data if int(self.in_out[j]) else self.data
        return src[o:o + n].cpu().numpy().tobytes()

    def value_crcs(self, stream=None) -> torch.Tensor:
        """crc32 (store/crc32.go get) of every record's value after Payload.Decompress, on the
        device (int32 [n]); an XOR of them is the parity digest of a replay."""
        out = torch.zeros(self.n, dtype=torch.int32, device=self.offset.device)
        for where, src in ((1, self.values.data), (0, self.data)):
            m = torch.nonzero(self.in_out == where).flatten()
            if m.numel():
                out[m] = batch.crc32(batch.BlockBatch(src, self.val_off[m], self.value_len[m]), stream=stream)
        return out


def index(data: torch.Tensor, start: int = 0, max_key: int = MAX_KEY_LEN, body_max: int = BODY_MAX,
          workspace: batch.Workspace | None = None, stream=None):
    """Records DataStreamReader.Next would return from `start`: (offsets, sizeBroken, end_error, ncand, nvalid)."""
    L = _lib.lib()
    dev = data.device
    size = int(data.numel())
    cap = size // 256 + 1
    rec_off = torch.empty(cap, dtype=torch.int64, device=dev)
    rec_broken = torch.empty(cap, dtype=torch.int32, device=dev)
    result = torch.zeros(4, dtype=torch.int32, device=dev)
    ws_bytes = L.qlzx_replay_workspace_size(size)
    ws = (workspace or batch.Workspace(dev)).get(ws_bytes)
    rc = L.qlzx_replay_index(data.data_ptr() if size else None, size, start, max_key, body_max,
                             rec_off.data_ptr(), rec_broken.data_ptr(), result.data_ptr(), ws.data_ptr(),
                             ws_bytes, batch._stream(stream))
    _lib.check(rc, "qlzx_replay_index")
    r = result.cpu().numpy()
    n = int(r[0])
    return rec_off[:n], rec_broken[:n], bool(r[1]), int(r[2]), int(r[3])


def replay(data: torch.Tensor, start: int = 0, max_key: int = MAX_KEY_LEN, body_max: int = BODY_MAX,
           workspace: batch.Workspace | None = None, stream=None) -> ReplayResult:
    """Index, plan, decompress, finish: every per-record step runs on the device
    (qlzx_replay_index / qlzx_replay_plan / qlzx_decompress_batch / qlzx_replay_finish); the
    host reads back five numbers once (record and compressed counts, the largest dsize and the
    output size), which size the output buffer and the decoder launch."""
    L = _lib.lib()
    dev = data.device
    ws = workspace or batch.Workspace(dev)
    size = int(data.numel())
    cap = size // 256 + 1
    st_ = batch._stream(stream)
    rec_off = torch.empty(cap, dtype=torch.int64, device=dev)
    rec_broken = torch.empty(cap, dtype=torch.int32, device=dev)
    result = torch.zeros(4, dtype=torch.int32, device=dev)
    ws_bytes = L.qlzx_replay_workspace_size(size)
    w = ws.get(ws_bytes)
    _lib.check(L.qlzx_replay_index(data.data_ptr() if size else None, size, start, max_key, body_max,
                                   rec_off.data_ptr(), rec_broken.data_ptr(), result.data_ptr(), w.data_ptr(),
                                   ws_bytes, st_), "qlzx_replay_index")
    hdr = torch.empty(cap * 6, dtype=torch.int32, device=dev)
    comp_idx = torch.empty(cap, dtype=torch.int32, device=dev)
    comp_off = torch.empty(cap, dtype=torch.int64, device=dev)
    comp_len = torch.empty(cap, dtype=torch.int32, device=dev)
    comp_dsize = torch.empty(cap, dtype=torch.int32, device=dev)
    comp_dst = torch.empty(cap, dtype=torch.int64, device=dev)
    totals = torch.zeros(5, dtype=torch.int32, device=dev)
    pws = torch.empty(L.qlzx_replay_plan_workspace_size(cap), dtype=torch.uint8, device=dev)
    _lib.check(L.qlzx_replay_plan(data.data_ptr() if size else None, rec_off.data_ptr(), result.data_ptr(), cap,
                                  hdr.data_ptr(), comp_idx.data_ptr(), comp_off.data_ptr(), comp_len.data_ptr(),
                                  comp_dsize.data_ptr(), comp_dst.data_ptr(), totals.data_ptr(), pws.data_ptr(),
                                  pws.numel(), st_), "qlzx_replay_plan")
    # the one read-back: it sizes the output buffer and the decoder launch
    with torch.cuda.stream(stream) if stream is not None else _nullctx():
        t = totals.cpu().numpy().view(np.uint32)
        r = result.cpu().numpy()
    n, ncomp, maxd = int(t[0]), int(t[1]), int(t[2])
    out_bytes = int(t[3]) | (int(t[4]) << 32)
    out = torch.empty(out_bytes + 64, dtype=torch.uint8, device=dev)
    cst = torch.zeros(max(ncomp, 1), dtype=torch.int32, device=dev)
    cds = torch.zeros(max(ncomp, 1), dtype=torch.int32, device=dev)
    values = batch.BlockBatch(out, comp_dst[:ncomp], comp_dsize[:ncomp])
    if ncomp:
        csrc = batch.BlockBatch(data, comp_off[:ncomp], comp_len[:ncomp])
        cds, cst, _ = batch.decompress(csrc, values, dst_cap=comp_dsize[:ncomp], max_dsize=maxd, workspace=ws,
                                       stream=stream)
    flag = torch.empty(cap, dtype=torch.int32, device=dev)
    value_len = torch.empty(cap, dtype=torch.int32, device=dev)
    in_out = torch.empty(cap, dtype=torch.uint8, device=dev)
    val_off = torch.empty(cap, dtype=torch.int64, device=dev)
    vh16 = torch.empty(cap, dtype=torch.int16, device=dev)
    _lib.check(L.qlzx_replay_finish(data.data_ptr() if size else None, rec_off.data_ptr(), result.data_ptr(),
                                    totals.data_ptr(), comp_idx.data_ptr(), cst.data_ptr(), cds.data_ptr(),
                                    comp_dst.data_ptr(), out.data_ptr(), cap, flag.data_ptr(), value_len.data_ptr(),
                                    in_out.data_ptr(), val_off.data_ptr(), vh16.data_ptr(), st_),
               "qlzx_replay_finish")
    vh = vh16[:n].to(torch.int32) & 0xFFFF
    return ReplayResult(rec_off[:n], rec_broken[:n], hdr[: 6 * n].view(n, 6), flag[:n], value_len[:n], vh, values,
                        bool(r[1]), int(r[2]), int(r[3]), in_out[:n], val_off[:n], data)


class _nullctx:
    def __enter__(self):
        return self

    def __exit__(self, *a):
        return False


def _headers_dsize(data: torch.Tensor, off: np.ndarray, length: np.ndarray) -> np.ndarray:
    """Decompressed sizes from the QuickLZ headers (host parse of 9 bytes per block, quicklz.go:32-44);
    0 where the body is too short to hold a header (the decoder reports it)."""
    n = len(off)
    if n == 0:
        return np.zeros(0, np.uint32)
    idx = torch.from_numpy(off.view(np.int64)).to(data.device).unsqueeze(1) + torch.arange(9, device=data.device)
    idx = torch.clamp(idx, max=data.numel() - 1)
    h = data[idx.reshape(-1)].reshape(n, 9).cpu().numpy()
    big = (h[:, 0] & 2) != 0
    d9 = h[:, 5].astype(np.uint32) | (h[:, 6].astype(np.uint32) << 8) | (h[:, 7].astype(np.uint32) << 16) | \
        (h[:, 8].astype(np.uint32) << 24)
    d3 = h[:, 2].astype(np.uint32)
    d = np.where(big, d9, d3).astype(np.uint32)
    d[length < np.where(big, 9, 3)] = 0
    return np.minimum(d, BODY_MAX).astype(np.uint32)


def _vhash(src: torch.Tensor, off: torch.Tensor, length: torch.Tensor, out16: torch.Tensor, where: torch.Tensor,
           stream=None):
    L = _lib.lib()
    n = int(off.numel())
    o = off.to(torch.int64).contiguous()
    ln = length.to(torch.int32).contiguous()
    tmp = torch.zeros(n, dtype=torch.int16, device=src.device)
    rc = L.qlzx_vhash_batch(src.data_ptr(), o.data_ptr(), ln.data_ptr(), n, tmp.data_ptr(), batch._stream(stream))
    _lib.check(rc, "qlzx_vhash_batch")
    out16[where] = tmp


@dataclass
class HostReplayPart:
    """What the pipelined replay of one part leaves in host (pinned) memory.

    want="values": the per-record fields a reader of the values needs (offset, stored header,
    flag and length after Payload.Decompress, in_out / val_off, vhash) and the decoder's output
    buffer; a value with in_out 0 is the part's own bytes at val_off (the host already holds them).
    want="hints": buildHintFromData's fields only (store/bucket.go:89-117: the decompressed body
    only feeds Getvhash and is freed): offset, stored header, vhash."""
    n: int
    end_error: bool
    offset: torch.Tensor
    header: torch.Tensor
    vhash: torch.Tensor
    flag: torch.Tensor | None = None
    value_len: torch.Tensor | None = None
    in_out: torch.Tensor | None = None
    val_off: torch.Tensor | None = None
    values: torch.Tensor | None = None

    def value(self, part: torch.Tensor | np.ndarray, j: int) -> memoryview:
        """Record j's value after Payload.Decompress, from host memory (the decoder output copied
        back, or the part itself)."""
        o, n = int(self.val_off[j]), int(self.value_len[j])
        src = self.values if int(self.in_out[j]) else part
        a = src.numpy() if isinstance(src, torch.Tensor) else src
        return memoryview(a)[o:o + n]


class ReplayPipeline:
    """Replay of .data streams held in pinned host memory (chunk files read from disk),
    pipelined over three streams: pinned H2D of part i+1 || replay of part i || pinned D2H of
    part i-1's results (PCIe is full duplex), two device slots for the parts.  The streams, slots
    and host buffers are made once, here, for parts of at most `part_cap` bytes; run() then moves
    no allocation into the copy/replay loop (a host buffer only grows when a part needs more).

    want="values": the decompressed values and their per-record fields go back into two pinned
    host slots (`values_cap` bytes of decoder output each to start with), reused every other part.
    want="hints": buildHintFromData's fields only, into `nparts` per-part pinned buffers."""

    def __init__(self, part_cap: int, want: str = "values", device=None, workspace: batch.Workspace | None = None,
                 values_cap: int = 0, nparts: int = 0):
        if want not in ("values", "hints"):
            raise ValueError("want is 'values' or 'hints'")
        self.want = want
        self.dev = torch.device(device) if device is not None else torch.device("cuda", torch.cuda.current_device())
        self.ws = workspace or batch.Workspace(self.dev)
        self.part_cap = max(int(part_cap), 1)
        self.s_h2d, self.s_cmp, self.s_d2h = (torch.cuda.Stream(self.dev) for _ in range(3))
        self.dslot = [torch.empty(self.part_cap, dtype=torch.uint8, device=self.dev) for _ in range(2)]
        self.ev_in = [torch.cuda.Event(), torch.cuda.Event()]      # part landed in its device slot
        self.ev_used = [torch.cuda.Event(), torch.cuda.Event()]    # replay done with the device slot
        self.ev_out = [torch.cuda.Event(), torch.cuda.Event()]     # D2H into the host slot done
        rec_cap = self.part_cap // 256 + 1                         # records are 256-B aligned
        if want == "values":
            self.host = [self._values_slot(rec_cap, values_cap) for _ in range(2)]
        else:
            self.host = [self._hint_slot(rec_cap) for _ in range(max(nparts, 0))]

    @staticmethod
    def _pinned(n, dtype, shape=None):
        return torch.empty(shape if shape is not None else max(n, 1), dtype=dtype).pin_memory()

    def _values_slot(self, recs, nbytes):
        p = self._pinned
        return dict(cap=recs, values=p(nbytes, torch.uint8), off=p(recs, torch.int64),
                    hdr=p(0, torch.int32, (recs, 6)), vh=p(recs, torch.int32), flag=p(recs, torch.int32),
                    vlen=p(recs, torch.int32), io=p(recs, torch.uint8), voff=p(recs, torch.int64))

    def _hint_slot(self, recs):
        p = self._pinned
        return dict(cap=recs, off=p(recs, torch.int64), hdr=p(0, torch.int32, (recs, 6)), vh=p(recs, torch.int32))

    def run(self, parts: list[torch.Tensor], sink=None) -> list["HostReplayPart | None"]:
        """Replay every part (each a whole .data stream cut at record starts, in pinned memory).
        want="values": `sink(i, HostReplayPart)` (optional) runs once part i's copy has landed and
        before its host slot is reused (the host waits for it: a checking pass); without a sink
        nothing waits, and only the last two parts' results are left valid in the returned list
        (the others are None).  want="hints": every part's result is returned (and passed to
        `sink` at the end if given)."""
        np_ = len(parts)
        out: list[HostReplayPart | None] = [None] * np_
        if np_ == 0:
            return out
        if any(int(q.numel()) > self.part_cap for q in parts):
            raise ValueError("a part is larger than the pipeline's part_cap")
        if self.want == "hints":
            while len(self.host) < np_:
                self.host.append(self._hint_slot(self.part_cap // 256 + 1))
        s_h2d, s_cmp, s_d2h = self.s_h2d, self.s_cmp, self.s_d2h
        dslot, ev_in, ev_used, ev_out = self.dslot, self.ev_in, self.ev_used, self.ev_out
        pend: list[int | None] = [None, None]   # part whose results a host slot holds (sink not run yet)

        def h2d(i):
            dslot[i & 1][: parts[i].numel()].copy_(parts[i], non_blocking=True)
            ev_in[i & 1].record(s_h2d)

        def flush(j):
            i = pend[j]
            if i is not None:
                ev_out[j].synchronize()
                sink(i, out[i])
                pend[j] = None

        with torch.cuda.stream(s_h2d):
            h2d(0)
        for i in range(np_):
            j = i & 1
            if i + 1 < np_:   # prefetch the next part while this one replays
                with torch.cuda.stream(s_h2d):
                    if i >= 1:
                        s_h2d.wait_event(ev_used[j ^ 1])
                    h2d(i + 1)
            with torch.cuda.stream(s_cmp):
                s_cmp.wait_event(ev_in[j])
                r = replay(dslot[j][: parts[i].numel()], workspace=self.ws, stream=s_cmp)
                ev_used[j].record(s_cmp)
            n = r.n
            if self.want == "hints":
                h = self.host[i]
                hp = HostReplayPart(n, r.end_error, h["off"][:n], h["hdr"][:n], h["vh"][:n])
            else:
                if sink is not None:
                    flush(j)
                nb = int(r.values.data.numel())
                h = self.host[j]
                if h["cap"] < n or h["values"].numel() < nb:   # grow (a copy may still target the old one)
                    ev_out[j].synchronize()
                    h = self.host[j] = self._values_slot(max(n, h["cap"]), max(nb, h["values"].numel()))
                hp = HostReplayPart(n, r.end_error, h["off"][:n], h["hdr"][:n], h["vh"][:n], h["flag"][:n],
                                    h["vlen"][:n], h["io"][:n], h["voff"][:n], h["values"][:nb])
                if i >= 2 and sink is None:
                    out[i - 2] = None   # its host slot is reused now
            with torch.cuda.stream(s_d2h):
                s_d2h.wait_event(ev_used[j])
                if i >= 2:
                    s_d2h.wait_event(ev_out[j])
                srcs = [(hp.offset, r.offset), (hp.header, r.header), (hp.vhash, r.vhash)]
                if self.want == "values":
                    srcs += [(hp.flag, r.flag), (hp.value_len, r.value_len), (hp.in_out, r.in_out),
                             (hp.val_off, r.val_off), (hp.values, r.values.data)]
                for dst, src in srcs:
                    if src.numel():
                        dst.copy_(src, non_blocking=True)
                        src.record_stream(s_d2h)
                ev_out[j].record(s_d2h)
            out[i] = hp
            if self.want == "values" and sink is not None:
                pend[j] = i
        if self.want == "values" and sink is not None:
            for j in (((np_ - 2) & 1, (np_ - 1) & 1) if np_ >= 2 else (0,)):
                flush(j)
        for e in ev_out:
            e.synchronize()
        if self.want == "hints" and sink is not None:
            for i, hp in enumerate(out):
                sink(i, hp)
        return out


def replay_pipelined(parts: list[torch.Tensor], want: str = "values", device=None,
                     workspace: batch.Workspace | None = None, sink=None) -> list["HostReplayPart | None"]:
    """One-shot ReplayPipeline(max part size, want).run(parts, sink)."""
    cap = max([int(q.numel()) for q in parts], default=1)
    return ReplayPipeline(cap, want, device, workspace, nparts=len(parts)).run(parts, sink)


def host_value_digest(hp: HostReplayPart, part, key_base: int = 0, file_id: int = 0, threads: int = 16) -> int:
    """XOR over the part's records of crc32 (zlib's = store/crc32.go's) of each value as it sits
    in HOST memory after the pipelined replay, keyed by the record's place like the device-only
    digest: crc ^ ((key_base + offset) * 0x85EBCA77 + (file_id + 1) * 0x9E3779B1) mod 2^32."""
    import zlib
    from concurrent.futures import ThreadPoolExecutor
    n = hp.n
    if n == 0:
        return 0
    off = hp.offset.numpy()
    voff = hp.val_off.numpy()
    vlen = hp.value_len.numpy()
    io = hp.in_out.numpy()
    pa = part.numpy() if isinstance(part, torch.Tensor) else np.asarray(part)
    vals = memoryview(hp.values.numpy())
    raw = memoryview(pa)
    keys = ((key_base + off.astype(np.int64)) * 0x85EBCA77 + (file_id + 1) * 0x9E3779B1) & 0xFFFFFFFF

    def run(lo, hi):
        d = 0
        for j in range(lo, hi):
            o = int(voff[j])
            src = vals if io[j] else raw
            d ^= zlib.crc32(src[o:o + int(vlen[j])]) ^ int(keys[j])
        return d

    t = max(1, min(threads, n // 256 + 1))
    cuts = [n * k // t for k in range(t + 1)]
    with ThreadPoolExecutor(t) as ex:
        parts_ = list(ex.map(lambda k: run(cuts[k], cuts[k + 1]), range(t)))
    d = 0
    for x in parts_:
        d ^= x
    return d


def hint_digest(offset, header, vhash, key_base: int = 0, file_id: int = 0) -> int:
    """XOR over records of a keyed mix of the hint fields (offset, stored header, vhash): the
    parity digest of buildHintFromData's output; torch tensors (host or device) or arrays."""
    def a(x):
        return x.cpu().numpy() if isinstance(x, torch.Tensor) else np.asarray(x)
    off = a(offset).astype(np.int64) + key_base
    hdr = a(header).astype(np.int64).reshape(-1, 6) & 0xFFFFFFFF
    vh = a(vhash).astype(np.int64) & 0xFFFF
    if off.size == 0:
        return 0
    m = (off * 0x85EBCA77 + (file_id + 1) * 0x9E3779B1) & 0xFFFFFFFF
    for c in range(6):
        m = (m * 0x01000193 ^ hdr[:, c]) & 0xFFFFFFFF
    m = (m * 0x01000193 ^ vh) & 0xFFFFFFFF
    return int(np.bitwise_xor.reduce(m))


def read_record(rec: bytes) -> tuple[int, bytes] | None:
    """One record as a GET reads it: readRecordAt's CRC check (store/datafile.go:161-168) and
    Payload.Decompress (store/item.go:163-176) -- header[4:24] and the key through crc32_write
    (the library folds such short slices on the host), then the value's CRC and its decode in ONE
    request (qlzx_read_record1).  Returns (flag after Payload.Decompress, value), or None when the
    record CRC does not match (readRecordAt's error).  As in the reference, a value that fails to
    decode stays compressed with its flag unchanged."""
    import struct
    L = _lib.lib()
    crc, _ts, flag, _ver, ksz, vsz = struct.unpack_from("<IIIiII", rec, 0)
    key = rec[HDR:HDR + ksz]
    val = bytes(rec[HDR + ksz:HDR + ksz + vsz])
    st = L.crc32_write(0xFFFFFFFF, bytes(rec[4:HDR]), 20)
    if ksz:
        st = L.crc32_write(st, bytes(key), ksz)
    comp = bool(flag & FLAG_COMPRESS)
    cap = 0
    if comp and len(val) >= (9 if (val and val[0] & 2) else 3):
        cap = int.from_bytes(val[5:9], "little") if val[0] & 2 else val[2]
    dst = ctypes.create_string_buffer(max(cap, 1))
    out = ctypes.c_size_t(0)
    status = ctypes.c_int32(0)
    _lib.check(L.qlzx_read_record1(val, len(val), st, crc, int(comp), dst, cap, ctypes.byref(out),
                                   ctypes.byref(status)), "qlzx_read_record1")
    if status.value == _lib.E_CRC:
        return None
    if comp and status.value == _lib.OK:
        return flag - FLAG_COMPRESS, dst.raw[:out.value]
    return flag, val
