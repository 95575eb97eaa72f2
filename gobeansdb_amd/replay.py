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
    values: batch.BlockBatch   # decompressed values (compressed records) / raw bodies (others)
    end_error: bool            # the reader stopped on an unexpected EOF after these records
    n_candidates: int
    n_valid: int

    @property
    def n(self) -> int:
        return int(self.offset.numel())


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
    L = _lib.lib()
    dev = data.device
    ws = workspace or batch.Workspace(dev)
    off, broken, end_err, ncand, nvalid = index(data, start, max_key, body_max, ws, stream)
    n = int(off.numel())
    # 24-B headers of the records (gathered on device)
    hidx = off.unsqueeze(1) + torch.arange(HDR, device=dev).unsqueeze(0)
    hdr = data[hidx.reshape(-1)].reshape(n, HDR).contiguous().view(torch.int32) if n else \
        torch.zeros((0, 6), dtype=torch.int32, device=dev)
    flag = hdr[:, 2].clone()
    ksz = hdr[:, 4].to(torch.int64)
    vsz = hdr[:, 5].to(torch.int64)
    body_off = off + HDR + ksz
    comp = (flag & FLAG_COMPRESS) != 0
    ci = torch.nonzero(comp).flatten()
    # values: compressed ones decompressed into a fresh buffer, the others referenced in place
    value_len = vsz.to(torch.int32).clone()
    src_base = data
    val_off = body_off.clone()
    out = None
    if ci.numel():
        csrc = batch.BlockBatch(data, body_off[ci].contiguous(), vsz[ci].to(torch.int32).contiguous())
        # dsize from each header; Payload.Decompress needs >= 9 B to read it
        clen = csrc.length.cpu().numpy().view(np.uint32)
        coff = csrc.off.cpu().numpy().view(np.uint64)
        host = _headers_dsize(data, coff, clen)
        out = batch.BlockBatch.empty_for(host, device=dev)
        dsz, st, _ = batch.decompress(csrc, out, dst_cap=torch.from_numpy(host.view(np.int32)).to(dev),
                                      max_dsize=int(host.max()) if len(host) else 0, workspace=ws,
                                      stream=stream)
        ok = st == 0
        # successful records: value = decompressed, flag -= FLAG_COMPRESS (store/item.go:172-174)
        flag[ci[ok]] -= FLAG_COMPRESS
        value_len[ci[ok]] = dsz[ok]
    # Getvhash over the final values: gather into one view per source
    vh = torch.zeros(n, dtype=torch.int32, device=dev)
    vh16 = torch.zeros(n, dtype=torch.int16, device=dev)
    plain_i = torch.nonzero(~comp).flatten()
    if ci.numel():
        okm = (st == 0)
        good = ci[okm]
        bad = ci[~okm]
        plain_i = torch.cat([plain_i, bad])
        if good.numel():
            _vhash(out.data, out.off[okm], value_len[good], vh16, good, stream)
    if plain_i.numel():
        _vhash(src_base, val_off[plain_i], value_len[plain_i], vh16, plain_i, stream)
    vh = vh16.to(torch.int32) & 0xFFFF
    values = out if out is not None else batch.BlockBatch(data, val_off, value_len)
    return ReplayResult(off, broken, hdr, flag, value_len, vh, values, end_err, ncand, nvalid)


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
