"""Mirror of gobeansdb's ``quicklz`` Go package (quicklz/quicklz.go, quicklz/cquicklz.go).

Same names, argument meaning and error behaviour, so the parity tests read
like ``quicklz/quicklz_test.go``.  Go's ``(value, error)`` pairs are returned
as tuples; Go panics are raised.  Every codec call runs on the GPU through
libqlzx.so (include/qlzx.h); there is no CPU codec here.

    Go                                   here
    SizeCompressed(src) int              SizeCompressed(src) -> int      quicklz.go:46
    SizeDecompressed(src) int            SizeDecompressed(src) -> int    quicklz.go:39
    CCompress(src) (CArray, bool)        CCompress(src) -> (CArray, bool) cquicklz.go:23
    CDecompress(src, sizeD) (CArray, err) CDecompress(src, n) -> (CArray, err) cquicklz.go:44
    CDecompressSafe(src) (CArray, err)   CDecompressSafe(src)            cquicklz.go:84
    DecompressSafe(src) ([]byte, err)    DecompressSafe(src)             cquicklz.go:62
    Compress(src, level) []byte          Compress(src, level)            quicklz.go:80
    Decompress(src) []byte               Decompress(src)                 quicklz.go:291
"""
from __future__ import annotations

import ctypes

from . import _lib

CompressBufferSize = 528400   # cquicklz.go:19
DecompressBufferSize = 16     # cquicklz.go:20
BodyInC = 4096                # config/mc_config.go:9 (cmem.CArray: Go heap below, C heap above)


class QuicklzError(Exception):
    pass


class CArray:
    """cmem.CArray (cmem/cmem.go): Body plus the allocation size Cap."""

    __slots__ = ("Body", "Cap")

    def __init__(self, body: bytes = b"", cap: int = 0):
        self.Body = body
        self.Cap = cap

    def Free(self) -> None:  # cmem.go:96-104
        self.Body = b""
        self.Cap = 0


def _as_bytes(src) -> bytes:
    return bytes(src)


def SizeDecompressed(source) -> int:
    """quicklz.go:39-44 (header parse; reads byte 0 and the size field)."""
    s = _as_bytes(source)
    if s[0] & 2:
        return int.from_bytes(s[5:9], "little")
    return s[2]


def SizeCompressed(source) -> int:
    """quicklz.go:46-51."""
    s = _as_bytes(source)
    if s[0] & 2:
        return int.from_bytes(s[1:5], "little")
    return s[1]


def CCompress(src) -> tuple[CArray, bool]:
    """cquicklz.go:23-42: C-library level-3 compress into a len+400 CArray.

    ``&src[0]`` panics on an empty slice (cquicklz.go:36): IndexError here."""
    s = _as_bytes(src)
    if len(s) == 0:
        raise IndexError("index out of range [0] with length 0")
    dst = ctypes.create_string_buffer(len(s) + 400)
    n = _lib.lib().qlz_compress(s, dst, len(s), None)
    if n == 0:
        raise _lib.QlzxError("qlz_compress failed: " + _lib.lib().qlzx_last_error().decode())
    return CArray(dst.raw[:n], len(s) + 400), True


def CDecompress(src, sizeD: int) -> tuple[CArray, QuicklzError | None]:
    """cquicklz.go:44-60."""
    s = _as_bytes(src)
    dst = ctypes.create_string_buffer(max(sizeD, 1))
    size = _lib.lib().qlz_decompress(s, dst, None)
    if size != sizeD:
        return CArray(), QuicklzError(f"fail to alloc for decompress, size {sizeD} != {size}")
    return CArray(dst.raw[:size], sizeD), None


def CDecompressSafe(src) -> tuple[CArray, QuicklzError | None]:
    """cquicklz.go:84-101: size-checked CDecompress."""
    s = _as_bytes(src)
    try:
        sizeC = SizeCompressed(s)
    except IndexError as e:  # recover() in the Go wrapper
        return CArray(), QuicklzError(f"CDecompressSafe panic({e!r})")
    if len(s) != sizeC:
        return CArray(), QuicklzError(f"bad sizeCompressed, expect {sizeC}, got {len(s)}")
    return CDecompress(s, SizeDecompressed(s))


def Compress(source, level: int) -> bytes | None:
    """quicklz.go:80-289: Go encoder.  Level 3 differs from CCompress in three
    ways (always a 9-byte header, earlier bail-out, nil on empty), reproduced
    by the GPU encoder's GO_COMPAT mode; level 1 (quicklz.go:120-191) is the
    lane-per-block k_enc_go_l1 (qlzx_level1.hip)."""
    if level not in (1, 3):
        raise QuicklzError("Go version only supports level 1 and 3")   # quicklz.go:94-96
    s = _as_bytes(source)
    if len(s) == 0:
        return None   # quicklz.go:109-111
    dst = ctypes.create_string_buffer(len(s) + 400)
    flags = _lib.F_LEVEL1 if level == 1 else _lib.F_GO_COMPAT
    n = _lib.lib().qlzx_compress1(s, dst, len(s), flags)
    if n == 0:
        raise _lib.QlzxError("qlzx_compress1 failed: " + _lib.lib().qlzx_last_error().decode())
    return dst.raw[:n]


def Decompress(source) -> bytes:
    """quicklz.go:291-431.  Compressed level-3 streams take the level-3 decoder
    (K1/K2); stored streams of either level and compressed level-1 streams take
    k_dec_go_l1 (Go's copy() semantics for a short stored body, zero-filled).
    Where Go panics (level not 1/3, an index out of range on a corrupt stream)
    this raises QuicklzError."""
    s = _as_bytes(source)
    if len(s) == 0 or len(s) < (9 if s[0] & 2 else 3):
        # SizeDecompressed indexes the size field: Go panics on a short header
        raise QuicklzError(f"truncated quicklz header ({len(s)} bytes)")
    level = (s[0] >> 2) & 3
    if level not in (1, 3):
        raise QuicklzError("Go version only supports level 1 and 3")
    n = SizeDecompressed(s)
    dst = ctypes.create_string_buffer(max(n, 1))
    L = _lib.lib()
    if level == 3 and (s[0] & 1):
        # qlz_decompress reads SizeCompressed(s) bytes (quicklz.c:777-836 trusts the header);
        # Go never reads that field: it decodes any stream whose tokens fit in len(source) and
        # panics on the first index past it (quicklz.go:291-431).  A header csize that differs
        # from len(s), above or below, is therefore rewritten to len(s): the decoder is bounded
        # by the bytes Go may index.  Known difference: Go ignores bytes after the item that
        # completes dsize, while check C5 rejects a stream with such trailing bytes.
        if len(s) != SizeCompressed(s):
            b = bytearray(s)
            if s[0] & 2:
                b[1:5] = len(s).to_bytes(4, "little")
            else:
                b[1] = len(s)
            s = bytes(b)
        size = L.qlz_decompress(s, dst, None)
        bad = size != n or L.qlzx_last_status() != _lib.OK
    else:
        # QLZX_GO_ERROR is the error channel: a dsize-0 stream the kernel rejects must raise too
        size = L.qlzx_go_decompress1(s, len(s), dst, n)
        bad = size == _lib.GO_ERROR or size != n
    if bad:
        st = L.qlzx_last_status()
        name = _lib.STATUS_NAMES[st] if 0 <= st < len(_lib.STATUS_NAMES) else str(st)
        raise QuicklzError(f"corrupt quicklz stream (status {name}: {L.qlzx_last_error().decode()})")
    return dst.raw[:n]


def DecompressSafe(src) -> tuple[bytes | None, QuicklzError | None]:
    """cquicklz.go:62-82."""
    s = _as_bytes(src)
    try:
        sizeC = SizeCompressed(s)
        if len(s) != sizeC:
            return None, QuicklzError(f"bad sizeCompressed, expect {sizeC}, got {len(s)}")
        sizeD = SizeDecompressed(s)
        dst = Decompress(s)
    except (QuicklzError, IndexError) as e:
        return None, QuicklzError(f"decompress panic with non-error: {e!r}")
    if len(dst) != sizeD:
        return None, QuicklzError(f"bad sizeDecompressed, expect {sizeD}, got {len(dst)}")
    return dst, None
