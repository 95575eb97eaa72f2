"""ctypes view of the CPU oracle -- TEST INFRASTRUCTURE ONLY.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg import
this module.  `ref()` additionally exposes the reference quicklz.c /
crc32_write compiled from /root/reference (oracle/_ref, container only).
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
_lib = None
_ref = None

OK, E_SIZE_COMPRESSED, E_CORRUPT, E_LEVEL, E_DST_CAP, E_HEADER = 0, 1, 2, 3, 4, 6
_u8p = ctypes.POINTER(ctypes.c_uint8)


def build():
    subprocess.run(["make", "-s", "-C", HERE], check=True)


def lib():
    global _lib
    if _lib is None:
        path = os.path.join(HERE, "liboracle.so")
        if not os.path.exists(path):
            build()
        L = ctypes.CDLL(path)
        vp, sz = ctypes.c_void_p, ctypes.c_size_t
        L.orc_compress.argtypes = [vp, sz, vp]
        L.orc_compress.restype = sz
        L.orc_compress_go.argtypes = [vp, sz, vp]
        L.orc_compress_go.restype = sz
        L.orc_decompress.argtypes = [vp, sz, vp, sz, ctypes.POINTER(sz)]
        L.orc_decompress.restype = ctypes.c_int
        L.orc_compress_go_l1.argtypes = [vp, sz, vp]
        L.orc_compress_go_l1.restype = sz
        L.orc_decompress_go_l1.argtypes = [vp, sz, vp, sz, ctypes.POINTER(sz)]
        L.orc_decompress_go_l1.restype = ctypes.c_int
        L.orc_crc32_write.argtypes = [ctypes.c_uint32, vp, sz]
        L.orc_crc32_write.restype = ctypes.c_uint32
        L.orc_size_compressed.argtypes = [vp]
        L.orc_size_compressed.restype = sz
        L.orc_size_decompressed.argtypes = [vp]
        L.orc_size_decompressed.restype = sz
        L.orc_block_seed.argtypes = [ctypes.c_uint64, ctypes.c_uint64]
        L.orc_block_seed.restype = ctypes.c_uint64
        for fn in (L.orc_gen_text, L.orc_gen_image):
            fn.argtypes = [ctypes.c_uint64, vp, vp, vp, ctypes.c_uint32, vp, sz]
            fn.restype = None
        for fn in (L.orc_bench_decompress, L.orc_bench_compress):
            fn.argtypes = [vp, vp, vp, vp, vp, ctypes.c_uint32, ctypes.c_int, ctypes.c_int]
            fn.restype = ctypes.c_double
        _lib = L
    return _lib


def _buf(b):
    a = np.frombuffer(bytes(b), dtype=np.uint8) if not isinstance(b, np.ndarray) else b
    return np.ascontiguousarray(a), a.ctypes.data


def compress(data: bytes) -> bytes:
    src = np.frombuffer(data, dtype=np.uint8) if len(data) else np.zeros(1, np.uint8)
    dst = np.zeros(len(data) + 400, dtype=np.uint8)
    r = lib().orc_compress(src.ctypes.data, len(data), dst.ctypes.data)
    return dst[:r].tobytes()


def compress_go(data: bytes) -> bytes:
    src = np.frombuffer(data, dtype=np.uint8) if len(data) else np.zeros(1, np.uint8)
    dst = np.zeros(len(data) + 400, dtype=np.uint8)
    r = lib().orc_compress_go(src.ctypes.data, len(data), dst.ctypes.data)
    return dst[:r].tobytes()


def decompress(data: bytes, cap: int | None = None):
    """Return (status, bytes)."""
    src = np.frombuffer(data, dtype=np.uint8) if len(data) else np.zeros(1, np.uint8)
    if cap is None:
        cap = lib().orc_size_decompressed(src.ctypes.data) if len(data) >= 9 else 256
    dst = np.zeros(max(cap, 1), dtype=np.uint8)
    out = ctypes.c_size_t(0)
    st = lib().orc_decompress(src.ctypes.data, len(data), dst.ctypes.data, cap, ctypes.byref(out))
    return st, dst[: out.value].tobytes()


def compress_go_l1(data: bytes) -> bytes | None:
    """Go quicklz.Compress(data, 1) (quicklz.go:80-191); None for empty input (Go nil)."""
    if not data:
        return None
    src = np.frombuffer(data, dtype=np.uint8)
    dst = np.zeros(len(data) + 400, dtype=np.uint8)
    r = lib().orc_compress_go_l1(src.ctypes.data, len(data), dst.ctypes.data)
    return dst[:r].tobytes()


def decompress_go_l1(data: bytes, cap: int | None = None):
    """Go quicklz.Decompress of a level-1 or stored stream: (status, bytes)."""
    src = np.frombuffer(data, dtype=np.uint8) if len(data) else np.zeros(1, np.uint8)
    if cap is None:
        cap = lib().orc_size_decompressed(src.ctypes.data) if len(data) >= 9 else 256
    dst = np.zeros(max(cap, 1), dtype=np.uint8)
    out = ctypes.c_size_t(0)
    st = lib().orc_decompress_go_l1(src.ctypes.data, len(data), dst.ctypes.data, cap, ctypes.byref(out))
    return st, dst[: out.value].tobytes()


def crc32_write(crc: int, data: bytes) -> int:
    src = np.frombuffer(data, dtype=np.uint8) if len(data) else np.zeros(1, np.uint8)
    return lib().orc_crc32_write(crc, src.ctypes.data, len(data))


def record_crc(header_tail20: bytes, key: bytes, value: bytes) -> int:
    """store/datafile.go:66-76: ~crc32_write(~0, header[4:] ‖ key ‖ value)."""
    c = 0xFFFFFFFF
    for part in (header_tail20, key, value):
        if part:
            c = crc32_write(c, part)
    return c ^ 0xFFFFFFFF


def gen_text(seed: int, block_id: int, n: int) -> bytes:
    from gobeansdb_amd import synth
    v, o, cdf = synth.tables()
    out = np.zeros(n, dtype=np.uint8)
    L = lib()
    L.orc_gen_text(L.orc_block_seed(seed, block_id), v.ctypes.data, o.ctypes.data,
                   cdf.ctypes.data, len(cdf), out.ctypes.data, n)
    return out.tobytes()


def gen_image(seed: int, block_id: int, n: int) -> bytes:
    from gobeansdb_amd import synth
    v, o, cdf = synth.tables()
    out = np.zeros(n, dtype=np.uint8)
    L = lib()
    L.orc_gen_image(L.orc_block_seed(seed, block_id), v.ctypes.data, o.ctypes.data,
                    cdf.ctypes.data, len(cdf), out.ctypes.data, n)
    return out.tobytes()


# ---- reference codec (container only: /root/reference) ----
def ref():
    """The reference quicklz.c + crc32_write, compiled by oracle/Makefile."""
    global _ref
    if _ref is None:
        q = os.path.join(HERE, "_ref", "libqlzref.so")
        c = os.path.join(HERE, "_ref", "libcrc32ref.so")
        if not (os.path.exists(q) and os.path.exists(c)):
            build()
        if not (os.path.exists(q) and os.path.exists(c)):
            return None
        Q, C = ctypes.CDLL(q), ctypes.CDLL(c)
        vp, sz = ctypes.c_void_p, ctypes.c_size_t
        Q.qlz_compress.argtypes = [vp, vp, sz, vp]
        Q.qlz_compress.restype = sz
        Q.qlz_decompress.argtypes = [vp, vp, vp]
        Q.qlz_decompress.restype = sz
        Q.qlz_get_setting.argtypes = [ctypes.c_int]
        Q.qlz_get_setting.restype = ctypes.c_int
        C.crc32_write.argtypes = [ctypes.c_uint32, vp, ctypes.c_int]
        C.crc32_write.restype = ctypes.c_uint32
        _ref = (Q, C)
    return _ref


def ref_if_built():
    """The compiled reference codec if oracle/_ref holds it (never builds: the GPU box
    has no /root/reference, only the .so built here); None otherwise."""
    q = os.path.join(HERE, "_ref", "libqlzref.so")
    if not os.path.exists(q):
        return None
    Q = ctypes.CDLL(q)
    L = lib()
    L.orc_bench_ref.argtypes = [ctypes.c_void_p] * 6 + [ctypes.c_uint32, ctypes.c_int, ctypes.c_int]
    L.orc_bench_ref.restype = ctypes.c_double
    L.orc_bench_replay.argtypes = [ctypes.c_void_p] * 4 + [ctypes.c_int, ctypes.c_int, ctypes.c_void_p]
    L.orc_bench_replay.restype = ctypes.c_double
    return Q


def crc_ref_if_built():
    """The compiled reference crc32_write (oracle/_ref/libcrc32ref.so) if present."""
    c = os.path.join(HERE, "_ref", "libcrc32ref.so")
    return ctypes.CDLL(c) if os.path.exists(c) else None


def ref_compress(data: bytes) -> bytes:
    Q, _ = ref()
    src = np.frombuffer(data, dtype=np.uint8) if len(data) else np.zeros(1, np.uint8)
    dst = np.zeros(len(data) + 400, dtype=np.uint8)   # zero-filled
    scratch = np.zeros(528400, dtype=np.uint8)
    r = Q.qlz_compress(src.ctypes.data, dst.ctypes.data, len(data), scratch.ctypes.data)
    return dst[:r].tobytes()


def ref_decompress(data: bytes) -> bytes:
    Q, _ = ref()
    src = np.frombuffer(data, dtype=np.uint8)
    n = lib().orc_size_decompressed(src.ctypes.data)
    dst = np.zeros(n + 8, dtype=np.uint8)
    scratch = np.zeros(16, dtype=np.uint8)
    r = Q.qlz_decompress(src.ctypes.data, dst.ctypes.data, scratch.ctypes.data)
    return dst[:r].tobytes()


def ref_crc32_write(crc: int, data: bytes) -> int:
    _, C = ref()
    src = np.frombuffer(data, dtype=np.uint8)
    return C.crc32_write(crc, src.ctypes.data, len(data))


_ref_l1 = None


def ref_l1():
    """The reference quicklz.c compiled at QuickLZ level 1 (oracle/_ref/libqlzref_l1.so,
    container only); None when it is not built."""
    global _ref_l1
    if _ref_l1 is None:
        q = os.path.join(HERE, "_ref", "libqlzref_l1.so")
        if not os.path.exists(q):
            build()
        if not os.path.exists(q):
            return None
        Q = ctypes.CDLL(q)
        vp, sz = ctypes.c_void_p, ctypes.c_size_t
        Q.qlz_compress.argtypes = [vp, vp, sz, vp]
        Q.qlz_compress.restype = sz
        Q.qlz_decompress.argtypes = [vp, vp, vp]
        Q.qlz_decompress.restype = sz
        Q.qlz_get_setting.argtypes = [ctypes.c_int]
        Q.qlz_get_setting.restype = ctypes.c_int
        _ref_l1 = Q
    return _ref_l1


def ref_l1_compress(data: bytes) -> bytes:
    Q = ref_l1()
    src = np.frombuffer(data, dtype=np.uint8) if len(data) else np.zeros(1, np.uint8)
    dst = np.zeros(len(data) + 400, dtype=np.uint8)
    scratch = np.zeros(max(Q.qlz_get_setting(1), 1) + 64, dtype=np.uint8)   # QLZ_SCRATCH_COMPRESS
    r = Q.qlz_compress(src.ctypes.data, dst.ctypes.data, len(data), scratch.ctypes.data)
    return dst[:r].tobytes()


def ref_l1_decompress(data: bytes) -> bytes:
    Q = ref_l1()
    src = np.frombuffer(data, dtype=np.uint8)
    n = lib().orc_size_decompressed(src.ctypes.data)
    dst = np.zeros(n + 8, dtype=np.uint8)
    scratch = np.zeros(max(Q.qlz_get_setting(2), 1) + 64, dtype=np.uint8)   # QLZ_SCRATCH_DECOMPRESS
    r = Q.qlz_decompress(src.ctypes.data, dst.ctypes.data, scratch.ctypes.data)
    return dst[:r].tobytes()
