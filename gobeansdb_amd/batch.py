"""Batch device API over libqlzx.so, with torch tensors as device memory.

torch is plumbing here (allocation, streams, host<->device copies); the codec
is the HIP code behind include/qlzx.h.

A ``BlockBatch`` is one packed buffer plus per-block offsets/lengths, laid out
for HBM: block i lives at ``data[off[i] : off[i] + len[i]]`` and offsets are
aligned to ``ALIGN`` bytes so every block starts on a 256-B boundary (the
.data record alignment of store/item.go:20, and a whole number of 128-B lines).
"""
from __future__ import annotations

import ctypes
from dataclasses import dataclass

import numpy as np
import torch

from . import _lib

ALIGN = 256


def _ptr(t: torch.Tensor | None) -> int | None:
    return None if t is None else t.data_ptr()


def _stream(stream=None) -> int:
    s = stream if stream is not None else torch.cuda.current_stream()
    return s.cuda_stream


def pack_offsets(lengths, align: int = ALIGN, pad: int = 0) -> tuple[np.ndarray, int]:
    """Aligned offsets for blocks of the given lengths (+pad each); returns (off, total)."""
    ln = np.asarray(lengths, dtype=np.int64) + pad
    sz = (ln + align - 1) // align * align
    off = np.zeros(len(ln), dtype=np.uint64)
    if len(ln):
        off[1:] = np.cumsum(sz)[:-1]
    return off, int(sz.sum())


@dataclass
class BlockBatch:
    data: torch.Tensor      # uint8, device
    off: torch.Tensor       # uint64 (stored as int64), device
    length: torch.Tensor    # uint32 (stored as int32), device

    @property
    def n(self) -> int:
        return int(self.off.numel())

    @staticmethod
    def from_bytes(blocks: list[bytes], device="cuda", pad: int = 0) -> "BlockBatch":
        off, total = pack_offsets([len(b) for b in blocks], pad=pad)
        host = np.zeros(max(total, 1), dtype=np.uint8)
        for o, b in zip(off, blocks):
            host[int(o): int(o) + len(b)] = np.frombuffer(b, dtype=np.uint8)
        return BlockBatch(torch.from_numpy(host).to(device),
                          torch.from_numpy(off.view(np.int64)).to(device),
                          torch.from_numpy(np.asarray([len(b) for b in blocks], dtype=np.uint32).view(np.int32)).to(device))

    @staticmethod
    def empty_for(lengths, device="cuda", pad: int = 0) -> "BlockBatch":
        off, total = pack_offsets(lengths, pad=pad)
        return BlockBatch(torch.zeros(max(total, 1), dtype=torch.uint8, device=device),
                          torch.from_numpy(off.view(np.int64)).to(device),
                          torch.from_numpy(np.asarray(lengths, dtype=np.uint32).view(np.int32)).to(device))

    def to_bytes(self, lengths=None) -> list[bytes]:
        host = self.data.cpu().numpy()
        off = self.off.cpu().numpy().view(np.uint64)
        ln = (self.length.cpu().numpy().view(np.uint32) if lengths is None
              else np.asarray(lengths.cpu().numpy() if isinstance(lengths, torch.Tensor) else lengths).view(np.uint32))
        return [host[int(o): int(o) + int(l)].tobytes() for o, l in zip(off, ln)]


def _blocks(src: BlockBatch, dst_data: torch.Tensor, dst_off: torch.Tensor) -> _lib.Blocks:
    return _lib.Blocks(src.data.data_ptr(), src.off.data_ptr(), src.length.data_ptr(),
                       dst_data.data_ptr(), dst_off.data_ptr(), src.n)


class Workspace:
    """Grow-only device workspace (allocated outside the launch path)."""

    def __init__(self, device="cuda"):
        self.device = device
        self.buf = torch.empty(0, dtype=torch.uint8, device=device)

    def get(self, nbytes: int) -> torch.Tensor:
        if self.buf.numel() < nbytes:
            self.buf = torch.empty(max(nbytes, 1), dtype=torch.uint8, device=self.device)
        return self.buf


def decompress(src: BlockBatch, dst: BlockBatch, *, dst_cap: torch.Tensor | None = None,
               crc_state: torch.Tensor | None = None, crc_expect: torch.Tensor | None = None,
               want_crc: bool = False, max_dsize: int | None = None,
               workspace: Workspace | None = None, stream=None, general: bool = False):
    """Batch CDecompressSafe.  Returns (dsize u32, status i32, crc_out u32|None) device tensors.
    general=True passes no workspace, which routes every block to the general lane-per-block
    kernel (the path of values over 64 KiB); used by the parity tests of that kernel."""
    L = _lib.lib()
    n = src.n
    dev = src.data.device
    dsize = torch.zeros(n, dtype=torch.int32, device=dev)
    status = torch.full((n,), -1, dtype=torch.int32, device=dev)
    crc_out = torch.zeros(n, dtype=torch.int32, device=dev) if (want_crc or crc_expect is not None) else None
    if max_dsize is None:
        max_dsize = 0xFFFFFFFF
    ws_bytes = 0 if general else L.qlzx_decompress_workspace_size(n, max_dsize)
    ws_ptr = None if general else (workspace or Workspace(dev)).get(ws_bytes).data_ptr()
    b = _blocks(src, dst.data, dst.off)
    rc = L.qlzx_decompress_batch(ctypes.byref(b), _ptr(dst_cap), dsize.data_ptr(), status.data_ptr(),
                                 _ptr(crc_state), _ptr(crc_expect), _ptr(crc_out), max_dsize,
                                 ws_ptr, ws_bytes, _stream(stream))
    _lib.check(rc, "qlzx_decompress_batch")
    return dsize, status, crc_out


def compress(src: BlockBatch, dst: BlockBatch | None = None, *, crc_state: torch.Tensor | None = None,
             want_crc: bool = False, go_compat: bool = False, max_len: int | None = None,
             workspace: Workspace | None = None, stream=None):
    """Batch CCompress.  Returns (dst BlockBatch, csize i32, status i32, crc_out|None)."""
    L = _lib.lib()
    n = src.n
    dev = src.data.device
    if dst is None:
        lengths = src.length.cpu().numpy().view(np.uint32)
        dst = BlockBatch.empty_for(lengths, device=dev, pad=400)
    csize = torch.zeros(n, dtype=torch.int32, device=dev)
    status = torch.full((n,), -1, dtype=torch.int32, device=dev)
    crc_out = None
    if want_crc or crc_state is not None:
        crc_out = torch.zeros(n, dtype=torch.int32, device=dev)
        if crc_state is None:
            crc_state = torch.full((n,), -1, dtype=torch.int32, device=dev)
    if max_len is None:
        max_len = int(src.length.max().item()) if n else 0
    ws_bytes = L.qlzx_compress_workspace_size(n, max_len)
    ws = (workspace or Workspace(dev)).get(ws_bytes)
    b = _blocks(src, dst.data, dst.off)
    rc = L.qlzx_compress_batch(ctypes.byref(b), csize.data_ptr(), status.data_ptr(), _ptr(crc_state),
                               _ptr(crc_out), max_len, _lib.F_GO_COMPAT if go_compat else 0,
                               ws.data_ptr(), ws_bytes, _stream(stream))
    _lib.check(rc, "qlzx_compress_batch")
    return dst, csize, status, crc_out


def go_l1_compress(src: BlockBatch, dst: BlockBatch | None = None, workspace: Workspace | None = None,
                   stream=None):
    """Batch Go quicklz.Compress(src, 1) (quicklz.go:80-191), one lane per block.
    Returns (dst BlockBatch, csize i32, status i32)."""
    L = _lib.lib()
    n = src.n
    dev = src.data.device
    if dst is None:
        dst = BlockBatch.empty_for(src.length.cpu().numpy().view(np.uint32), device=dev, pad=400)
    csize = torch.zeros(n, dtype=torch.int32, device=dev)
    status = torch.full((n,), -1, dtype=torch.int32, device=dev)
    ws_bytes = L.qlzx_go_l1_workspace_size(n)
    ws = (workspace or Workspace(dev)).get(ws_bytes)
    b = _blocks(src, dst.data, dst.off)
    rc = L.qlzx_go_l1_compress_batch(ctypes.byref(b), csize.data_ptr(), status.data_ptr(), ws.data_ptr(),
                                     ws_bytes, _stream(stream))
    _lib.check(rc, "qlzx_go_l1_compress_batch")
    return dst, csize, status


def go_decompress(src: BlockBatch, dst: BlockBatch, *, dst_cap: torch.Tensor | None = None,
                  workspace: Workspace | None = None, stream=None):
    """Batch Go quicklz.Decompress of stored and level-1 streams (quicklz.go:291-431),
    one lane per block.  Returns (dsize i32, status i32)."""
    L = _lib.lib()
    n = src.n
    dev = src.data.device
    dsize = torch.zeros(n, dtype=torch.int32, device=dev)
    status = torch.full((n,), -1, dtype=torch.int32, device=dev)
    ws_bytes = L.qlzx_go_decompress_workspace_size(n)
    ws = (workspace or Workspace(dev)).get(ws_bytes)
    b = _blocks(src, dst.data, dst.off)
    rc = L.qlzx_go_decompress_batch(ctypes.byref(b), _ptr(dst_cap), dsize.data_ptr(), status.data_ptr(),
                                    ws.data_ptr(), ws_bytes, _stream(stream))
    _lib.check(rc, "qlzx_go_decompress_batch")
    return dsize, status


def crc32(src: BlockBatch, init: torch.Tensor | None = None, final_xor: int = 0xFFFFFFFF, stream=None):
    """out[i] = crc32_write(init[i] or ~0, block i) ^ final_xor (store/crc32.go:61-88)."""
    L = _lib.lib()
    out = torch.zeros(src.n, dtype=torch.int32, device=src.data.device)
    rc = L.qlzx_crc32_batch(src.data.data_ptr(), src.off.data_ptr(), src.length.data_ptr(), src.n,
                            _ptr(init), final_xor & 0xFFFFFFFF, out.data_ptr(), _stream(stream))
    _lib.check(rc, "qlzx_crc32_batch")
    return out


_TABLES_DEV = {}


def synth(kind: str, seed: int, lengths, first_id: int = 0, device="cuda", stream=None,
          out: BlockBatch | None = None) -> BlockBatch:
    """Deterministic synthetic blocks generated on the GPU: block i is
    gen(seed, first_id + i), written into `out` (its offsets and lengths) when given."""
    from . import synth as S
    L = _lib.lib()
    key = str(device)
    if key not in _TABLES_DEV:
        v, o, c = S.tables()
        _TABLES_DEV[key] = (torch.from_numpy(v).to(device), torch.from_numpy(o.view(np.int32)).to(device),
                            torch.from_numpy(c.view(np.int32)).to(device))
    v, o, c = _TABLES_DEV[key]
    if out is None:
        out = BlockBatch.empty_for(lengths, device=device)
    rc = L.qlzx_synth_batch(0 if kind == "text" else 1, seed, first_id, out.data.data_ptr(), out.off.data_ptr(),
                            out.length.data_ptr(), out.n, v.data_ptr(), o.data_ptr(), c.data_ptr(), c.numel(),
                            _stream(stream))
    _lib.check(rc, "qlzx_synth_batch")
    return out
