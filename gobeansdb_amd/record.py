"""Write-side record encode on the GPU.

Host mirror of the set path between a value arriving and its bytes reaching a
.data chunk:

  Record.TryCompress     store/item.go:120-161  (policy: ver >= 0, no client /
                         compress flag, padded record > 256 B, MIME sniff, a
                         10 KiB trial compress kept when float32(c)/float32(t) <= 0.7,
                         then the whole body)
  NeedCompress           store/item.go:114-118 + NotCompress defaults
                         (store/config_default.go:46-49: audio/wave, audio/mpeg)
  WriteRecord.encodeHeader / getCRC / append   store/datafile.go:66-88, 307-330

The compress runs in qlzx_compress_batch with the value CRC fused (raw state 0),
and the header+key prefix is folded in with qlzx_crc32_combine, because the
header carries the compressed size.  Records come out 256-B padded and laid
out back to back, ready to append.
"""
from __future__ import annotations

import struct
from dataclasses import dataclass

import numpy as np
import torch

from . import _lib, batch

FLAG_COMPRESS = 0x00010000
FLAG_CLIENT_COMPRESS = 0x00000010
TRY_COMPRESS_SIZE = 10 * 1024
COMPRESS_RATIO_LIMIT = np.float32(0.7)
PADDING = 256
HDR = 24
NOT_COMPRESS = frozenset({"audio/wave", "audio/mpeg"})


# conf/global.yaml:29-33 (the shipped hstore.data.not_compress); the defaults of
# store/config_default.go:46-49 are NOT_COMPRESS.
NOT_COMPRESS_SHIPPED = frozenset({"audio/mpeg", "audio/wave", "audio/ogg", "audio/midi"})

# The audio/video rows of Go 1.13's http.DetectContentType table (net/http/sniff.go, go.mod:
# go 1.13), in table order: (mask, pattern, answer).  Every row before them needs a
# different first byte ('<' after optional whitespace for HTML/XML, '%', a BOM, or an image
# signature: \x00\x00\x01/\x02\x00, "BM", "GIF8", "RIFF....WEBPVP", \x89PNG, \xFF\xD8\xFF), and
# "RIFF....WEBPVP" differs from the RIFF rows here at offset 8, so none shadows these.
_AV_SIGS = (
    (b"\xFF\xFF\xFF\xFF", b".snd", "audio/basic"),
    (b"\xFF\xFF\xFF\xFF\x00\x00\x00\x00\xFF\xFF\xFF\xFF", b"FORM\x00\x00\x00\x00AIFF", "audio/aiff"),
    (b"\xFF\xFF\xFF", b"ID3", "audio/mpeg"),
    (b"\xFF\xFF\xFF\xFF\xFF", b"OggS\x00", "application/ogg"),   # never "audio/ogg"
    (b"\xFF\xFF\xFF\xFF\xFF\xFF\xFF\xFF", b"MThd\x00\x00\x00\x06", "audio/midi"),
    (b"\xFF\xFF\xFF\xFF\x00\x00\x00\x00\xFF\xFF\xFF\xFF", b"RIFF\x00\x00\x00\x00AVI ", "video/avi"),
    (b"\xFF\xFF\xFF\xFF\x00\x00\x00\x00\xFF\xFF\xFF\xFF", b"RIFF\x00\x00\x00\x00WAVE", "audio/wave"),
)


def sniff(prefix: bytes) -> str | None:
    """The http.DetectContentType answers a NotCompress set of audio types can act on
    (store/item.go:114-118): the masked audio/video signatures of Go 1.13's sniff table.
    None = some other answer (text, HTML, images, archives, octet-stream), which no audio
    entry of NotCompress matches.  Go answers "application/ogg" for Ogg data, so the
    shipped "audio/ogg" entry never fires (store/item_test.go:19 expects exactly that)."""
    p = prefix[:512]
    for mask, pat, ct in _AV_SIGS:
        if len(p) >= len(pat) and all((p[k] & mask[k]) == pat[k] for k in range(len(pat))):
            return ct
    return None


def need_compress(prefix: bytes, not_compress=NOT_COMPRESS) -> bool:
    """store/item.go:114-118."""
    return sniff(prefix) not in not_compress


@dataclass
class Encoded:
    data: torch.Tensor        # uint8 device buffer: the records, back to back
    offset: np.ndarray        # uint64 record offsets
    flag: np.ndarray          # uint32 flags as written (FLAG_COMPRESS added where kept)
    vsz: np.ndarray           # uint32 stored value sizes
    crc: np.ndarray           # uint32 record CRCs


def _dev_u64(a, dev):
    return torch.from_numpy(np.ascontiguousarray(a, dtype=np.uint64).view(np.int64)).to(dev)


def _dev_u32(a, dev):
    return torch.from_numpy(np.ascontiguousarray(a, dtype=np.uint32).view(np.int32)).to(dev)


def sniff_many(heads: np.ndarray, lens: np.ndarray, not_compress=NOT_COMPRESS) -> np.ndarray:
    """need_compress for many values at once: heads = the first bytes of each value (uint8
    [n, >= 12]), lens = the value lengths.  Same rows, order and masks as sniff()."""
    n = len(lens)
    undecided = np.ones(n, bool)
    skip = np.zeros(n, bool)
    for mask, pat, name in _AV_SIGS:   # the first matching row decides, as in sniff()
        k = len(pat)
        m = np.frombuffer(mask, np.uint8)[None, :]
        hit = undecided & (lens >= k) & np.all((heads[:, :k] & m) == np.frombuffer(pat, np.uint8)[None, :], axis=1)
        if name in not_compress:
            skip |= hit
        undecided &= ~hit
    if None in not_compress:   # "some other answer" listed: every value without an audio/video row
        skip |= undecided
    return ~skip


def encode(keys: list[bytes], values: batch.BlockBatch, flags=None, vers=None, ts=None,
           not_compress=NOT_COMPRESS, workspace: batch.Workspace | None = None, stream=None) -> Encoded:
    """TryCompress + encodeHeader + padding for n records whose values live on the device.
    Every per-record step is a device batch or a numpy array operation (no per-record host loop)."""
    L = _lib.lib()
    dev = values.data.device
    n = values.n
    ws = workspace or batch.Workspace(dev)
    flags = np.zeros(n, np.uint32) if flags is None else np.asarray(flags, np.uint32).copy()
    vers = np.zeros(n, np.int32) if vers is None else np.asarray(vers, np.int32)
    ts = np.zeros(n, np.uint32) if ts is None else np.asarray(ts, np.uint32)
    vlen = values.length.cpu().numpy().view(np.uint32).astype(np.int64)
    voff = values.off.cpu().numpy().view(np.uint64)
    klen = np.fromiter(map(len, keys), np.int64, count=n)

    # ---- TryCompress candidates (store/item.go:121-137) ----
    padded = (HDR + klen + vlen + 255) // 256 * 256
    cand = (vers >= 0) & ((flags & (FLAG_CLIENT_COMPRESS | FLAG_COMPRESS)) == 0) & (padded > PADDING)
    ci = np.nonzero(cand)[0]
    if len(ci):
        # MIME sniff (item.go:114-118) on the first bytes of each candidate, gathered from the device
        ok = sniff_many(_gather_heads(values, ci, 16), vlen[ci], not_compress)
        ci = ci[ok]
    is_comp = np.zeros(n, bool)
    c_src = np.zeros(n, np.int8)      # 0: the trial's output buffer, 1: the full compress's
    c_off = np.zeros(n, np.uint64)
    c_len = np.zeros(n, np.int64)
    c_crc = np.zeros(n, np.uint32)    # raw CRC (state 0) of the compressed value
    bufs = [None, None]
    if len(ci):
        tlen = np.minimum(vlen[ci], TRY_COMPRESS_SIZE)
        trial = batch.BlockBatch(values.data, _dev_u64(voff[ci], dev), _dev_u32(tlen, dev))
        crc0 = torch.zeros(len(ci), dtype=torch.int32, device=dev)
        tdst, tcs, tst, tcrc = batch.compress(trial, crc_state=crc0, max_len=int(tlen.max()), workspace=ws,
                                             stream=stream)
        tcs_h = tcs.cpu().numpy().view(np.uint32).astype(np.int64)
        if int((tst != 0).sum()):
            raise _lib.QlzxError("trial compress failed on the device")
        keep = (tcs_h.astype(np.float32) / tlen.astype(np.float32)) <= COMPRESS_RATIO_LIMIT   # :145
        full = keep & (vlen[ci] > tlen)      # :149-156: recompress the whole body
        kt = keep & ~full
        bufs[0] = tdst.data
        r = ci[kt]
        is_comp[r] = True
        c_off[r] = tdst.off.cpu().numpy().view(np.uint64)[kt]
        c_len[r] = tcs_h[kt]
        c_crc[r] = tcrc.cpu().numpy().view(np.uint32)[kt] ^ np.uint32(0xFFFFFFFF)
        fi = ci[full]
        if len(fi):
            fsrc = batch.BlockBatch(values.data, _dev_u64(voff[fi], dev), _dev_u32(vlen[fi], dev))
            fcrc0 = torch.zeros(len(fi), dtype=torch.int32, device=dev)
            fdst, fcs, fst, fcrc = batch.compress(fsrc, crc_state=fcrc0, max_len=int(vlen[fi].max()),
                                                 workspace=ws, stream=stream)
            if int((fst != 0).sum()):
                raise _lib.QlzxError("compress failed on the device")
            bufs[1] = fdst.data
            is_comp[fi] = True
            c_src[fi] = 1
            c_off[fi] = fdst.off.cpu().numpy().view(np.uint64)
            c_len[fi] = fcs.cpu().numpy().view(np.uint32).astype(np.int64)
            c_crc[fi] = fcrc.cpu().numpy().view(np.uint32) ^ np.uint32(0xFFFFFFFF)
    # ---- stored value sizes / flags ----
    vsz = np.where(is_comp, c_len, vlen)
    flags = flags + np.where(is_comp, np.uint32(FLAG_COMPRESS), np.uint32(0)).astype(np.uint32)   # :159
    # ---- raw CRC (from state 0) of every stored value ----
    raw_v = c_crc.copy()
    plain = np.nonzero(~is_comp)[0]
    if len(plain):
        c = batch.crc32(batch.BlockBatch(values.data, _dev_u64(voff[plain], dev), _dev_u32(vlen[plain], dev)),
                        init=torch.zeros(len(plain), dtype=torch.int32, device=dev), final_xor=0, stream=stream)
        raw_v[plain] = c.cpu().numpy().view(np.uint32)
    # ---- header[4:24] || key prefixes (16-B aligned staging), their raw CRC state from ~0, and
    # the combine with the value's raw CRC (datafile.go:66-76) ----
    pre_len = (20 + klen).astype(np.int64)
    pre_step = (pre_len + 15) // 16 * 16
    pre_off = np.zeros(n, np.int64)
    if n:
        pre_off[1:] = np.cumsum(pre_step)[:-1]
    pre = np.zeros(int(pre_step.sum()) if n else 0, np.uint8)
    tail = np.zeros(n, dtype=[("ts", "<u4"), ("flag", "<u4"), ("ver", "<i4"), ("ksz", "<u4"), ("vsz", "<u4")])
    tail["ts"], tail["flag"], tail["ver"], tail["ksz"], tail["vsz"] = ts, flags, vers, klen, vsz
    if n:
        pre[(pre_off[:, None] + np.arange(20)[None, :]).reshape(-1)] = tail.view(np.uint8).reshape(n, 20).reshape(-1)
        kall = np.frombuffer(b"".join(keys), np.uint8)
        if kall.size:
            kstart = np.zeros(n, np.int64)
            kstart[1:] = np.cumsum(klen)[:-1]
            pre[np.repeat(pre_off + 20 - kstart, klen) + np.arange(kall.size)] = kall
    pre_d = torch.from_numpy(pre).to(dev)
    s_hk = batch.crc32(batch.BlockBatch(pre_d, _dev_u64(pre_off.astype(np.uint64), dev),
                                        _dev_u32(pre_len.astype(np.uint32), dev)), final_xor=0, stream=stream)
    crc_d = torch.zeros(n, dtype=torch.int32, device=dev)
    rv = _dev_u32(raw_v, dev)
    lv = _dev_u32(vsz, dev)
    _lib.check(L.qlzx_crc32_combine(s_hk.data_ptr(), rv.data_ptr(), lv.data_ptr(), n, 0xFFFFFFFF,
                                    crc_d.data_ptr(), batch._stream(stream)), "qlzx_crc32_combine")
    crc = crc_d.cpu().numpy().view(np.uint32).copy()
    # ---- assemble: crc || header tail || key || value, zero padding to 256 (datafile.go:307-330) ----
    rsize = (HDR + klen + vsz + 255) // 256 * 256
    roff = np.zeros(n, np.uint64)
    if n:
        roff[1:] = np.cumsum(rsize)[:-1]
    total = int(rsize.sum())
    out = torch.zeros(max(total, 1), dtype=torch.uint8, device=dev)
    # header tail + key (from the prefix staging) at off + 4
    _copy(pre_d, pre_off.astype(np.uint64), pre_len.astype(np.uint32), out, roff + 4, stream)
    # values: raw ones from the value buffer, compressed ones from their compress buffers
    if len(plain):
        _copy(values.data, voff[plain], vlen[plain].astype(np.uint32), out,
              roff[plain] + HDR + klen[plain].astype(np.uint64), stream)
    for b in (0, 1):
        rs = np.nonzero(is_comp & (c_src == b))[0]
        if len(rs):
            _copy(bufs[b], c_off[rs], c_len[rs].astype(np.uint32), out, roff[rs] + HDR + klen[rs].astype(np.uint64),
                  stream)
    # crc field (records are 256-B aligned, so int32 words)
    out.view(torch.int32)[torch.from_numpy((roff // 4).astype(np.int64)).to(dev)] = crc_d
    return Encoded(out[:total], roff, flags, vsz.astype(np.uint32), crc)


def _copy(src: torch.Tensor, src_off, length, dst: torch.Tensor, dst_off, stream=None):
    L = _lib.lib()
    n = len(src_off)
    if n == 0:
        return
    dev = dst.device
    so, ln, do = _dev_u64(src_off, dev), _dev_u32(length, dev), _dev_u64(dst_off, dev)
    _lib.check(L.qlzx_copy_batch(src.data_ptr(), so.data_ptr(), ln.data_ptr(), dst.data_ptr(), do.data_ptr(), n,
                                 batch._stream(stream)), "qlzx_copy_batch")


def _gather_heads(values: batch.BlockBatch, idx: np.ndarray, k: int) -> np.ndarray:
    """The first k bytes of each selected value (zeros past its end), uint8 [len(idx), k]."""
    dev = values.data.device
    sel = torch.from_numpy(idx).to(dev)
    off = values.off[sel]
    ln = values.length[sel].to(torch.int64)
    ar = torch.arange(k, device=dev)
    pos = torch.minimum(off.unsqueeze(1) + ar.unsqueeze(0), torch.tensor(values.data.numel() - 1, device=dev))
    h = values.data[pos.reshape(-1)].reshape(len(idx), k)
    return torch.where(ar.unsqueeze(0) < ln.unsqueeze(1), h, torch.zeros_like(h)).cpu().numpy()


def _gather_prefix(values: batch.BlockBatch, idx: np.ndarray, k: int) -> list[bytes]:
    dev = values.data.device
    off = values.off[torch.from_numpy(idx).to(dev)]
    ln = values.length[torch.from_numpy(idx).to(dev)].to(torch.int64)
    ar = torch.arange(k, device=dev)
    pos = off.unsqueeze(1) + ar.unsqueeze(0)
    pos = torch.minimum(pos, torch.tensor(values.data.numel() - 1, device=dev))
    h = values.data[pos.reshape(-1)].reshape(len(idx), k).cpu().numpy()
    lh = np.minimum(ln.cpu().numpy(), k)
    return [h[j, : lh[j]].tobytes() for j in range(len(idx))]
