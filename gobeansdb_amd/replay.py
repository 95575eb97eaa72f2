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
