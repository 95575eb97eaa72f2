"""Loader for libqlzx.so (the HIP product library) and its C ABI (include/qlzx.h).

The library is built in-tree by ``gobeansdb_amd.build`` (hipcc, gfx950).  There
is no CPU codec behind this module: if the shared object is missing the
import of any codec entry point raises, and on a host without a GPU the
compute calls fail loudly (``QlzxError``).
"""
from __future__ import annotations

import ctypes
import os
import re

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
LIB_PATH = os.environ.get("QLZX_LIB", os.path.join(HERE, "libqlzx.so"))
HEADER = os.path.join(ROOT, "include", "qlzx.h")

# enum qlzx_status
OK, E_SIZE_COMPRESSED, E_CORRUPT, E_LEVEL, E_DST_CAP, E_CRC, E_HEADER, E_EMPTY, E_TOO_LARGE, E_MAX_DSIZE, E_RUNTIME = range(11)
STATUS_NAMES = ["OK", "E_SIZE_COMPRESSED", "E_CORRUPT", "E_LEVEL", "E_DST_CAP", "E_CRC",
                "E_HEADER", "E_EMPTY", "E_TOO_LARGE", "E_MAX_DSIZE", "E_RUNTIME"]


F_GO_COMPAT = 1
F_LEVEL1 = 2
GO_ERROR = (1 << (8 * ctypes.sizeof(ctypes.c_size_t))) - 1   # QLZX_GO_ERROR, (size_t)-1


class QlzxError(RuntimeError):
    pass


class Blocks(ctypes.Structure):
    _fields_ = [("src", ctypes.c_void_p), ("src_off", ctypes.c_void_p),
                ("src_len", ctypes.c_void_p), ("dst", ctypes.c_void_p),
                ("dst_off", ctypes.c_void_p), ("n", ctypes.c_uint32)]


_lib = None


def header_functions() -> list[str]:
    """Every function declared in include/qlzx.h."""
    text = open(HEADER).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    text = re.sub(r"^\s*#.*$", "", text, flags=re.M)   # preprocessor lines (#define X (...))
    return sorted(set(re.findall(r"\b([A-Za-z_][A-Za-z0-9_]*)\s*\([^;{]*\)\s*;", text)))


def lib() -> ctypes.CDLL:
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise QlzxError(f"{LIB_PATH} is missing: run gobeansdb_amd.build.build() (hipcc, gfx950)")
    L = ctypes.CDLL(LIB_PATH)
    vp, sz, u32, i32, u64 = ctypes.c_void_p, ctypes.c_size_t, ctypes.c_uint32, ctypes.c_int32, ctypes.c_uint64
    L.qlz_size_decompressed.argtypes = [vp]
    L.qlz_size_decompressed.restype = sz
    L.qlz_size_compressed.argtypes = [vp]
    L.qlz_size_compressed.restype = sz
    L.qlz_decompress.argtypes = [vp, vp, vp]
    L.qlz_decompress.restype = sz
    L.qlz_compress.argtypes = [vp, vp, sz, vp]
    L.qlz_compress.restype = sz
    L.qlz_get_setting.argtypes = [ctypes.c_int]
    L.qlz_get_setting.restype = ctypes.c_int
    L.crc32_write.argtypes = [u32, vp, ctypes.c_int]
    L.crc32_write.restype = u32
    BP = ctypes.POINTER(Blocks)
    L.qlzx_decompress_workspace_size.argtypes = [u32, u32]
    L.qlzx_decompress_workspace_size.restype = sz
    L.qlzx_decompress_batch.argtypes = [BP, vp, vp, vp, vp, vp, vp, u32, vp, sz, vp]
    L.qlzx_decompress_batch.restype = ctypes.c_int
    L.qlzx_compress_workspace_size.argtypes = [u32, u32]
    L.qlzx_compress_workspace_size.restype = sz
    L.qlzx_compress_batch.argtypes = [BP, vp, vp, vp, vp, u32, u32, vp, sz, vp]
    L.qlzx_compress_batch.restype = ctypes.c_int
    L.qlzx_compress1.argtypes = [vp, vp, sz, u32]
    L.qlzx_compress1.restype = sz
    L.qlzx_go_l1_workspace_size.argtypes = [u32]
    L.qlzx_go_l1_workspace_size.restype = sz
    L.qlzx_go_decompress_workspace_size.argtypes = [u32]
    L.qlzx_go_decompress_workspace_size.restype = sz
    L.qlzx_go_l1_compress_batch.argtypes = [BP, vp, vp, vp, sz, vp]
    L.qlzx_go_l1_compress_batch.restype = ctypes.c_int
    L.qlzx_go_decompress_batch.argtypes = [BP, vp, vp, vp, vp, sz, vp]
    L.qlzx_go_decompress_batch.restype = ctypes.c_int
    L.qlzx_go_decompress1.argtypes = [vp, sz, vp, sz]
    L.qlzx_go_decompress1.restype = sz
    L.qlzx_crc32_batch.argtypes = [vp, vp, vp, u32, vp, u32, vp, vp]
    L.qlzx_crc32_batch.restype = ctypes.c_int
    L.qlzx_synth_batch.argtypes = [ctypes.c_int, u64, u64, vp, vp, vp, u32, vp, vp, vp, u32, vp]
    L.qlzx_synth_batch.restype = ctypes.c_int
    L.qlzx_crc32_combine.argtypes = [vp, vp, vp, u32, u32, vp, vp]
    L.qlzx_crc32_combine.restype = ctypes.c_int
    L.qlzx_copy_batch.argtypes = [vp, vp, vp, vp, vp, u32, vp]
    L.qlzx_copy_batch.restype = ctypes.c_int
    L.qlzx_replay_workspace_size.argtypes = [u64]
    L.qlzx_replay_workspace_size.restype = sz
    L.qlzx_replay_index.argtypes = [vp, u64, u64, u32, u64, vp, vp, vp, vp, sz, vp]
    L.qlzx_replay_index.restype = ctypes.c_int
    L.qlzx_replay_plan_workspace_size.argtypes = [u32]
    L.qlzx_replay_plan_workspace_size.restype = sz
    L.qlzx_replay_plan.argtypes = [vp, vp, vp, u32, vp, vp, vp, vp, vp, vp, vp, vp, sz, vp]
    L.qlzx_replay_plan.restype = ctypes.c_int
    L.qlzx_replay_finish.argtypes = [vp, vp, vp, vp, vp, vp, vp, vp, vp, u32, vp, vp, vp, vp, vp, vp]
    L.qlzx_replay_finish.restype = ctypes.c_int
    L.qlzx_vhash_batch.argtypes = [vp, vp, vp, u32, vp, vp]
    L.qlzx_vhash_batch.restype = ctypes.c_int
    L.qlzx_last_status.argtypes = []
    L.qlzx_last_status.restype = ctypes.c_int
    L.qlzx_last_error.argtypes = []
    L.qlzx_last_error.restype = ctypes.c_char_p
    L.qlzx_info.argtypes = [ctypes.c_char_p, sz]
    L.qlzx_info.restype = ctypes.c_int
    L.qlzx_read_record1.argtypes = [vp, sz, u32, u32, ctypes.c_int, vp, sz, ctypes.POINTER(sz),
                                    ctypes.POINTER(ctypes.c_int32)]
    L.qlzx_read_record1.restype = ctypes.c_int
    L.qlzx_service_test_fault.argtypes = [ctypes.c_int]
    L.qlzx_service_test_fault.restype = ctypes.c_int
    _lib = L
    return L


def check(rc: int, what: str) -> None:
    if rc != 0:
        msg = lib().qlzx_last_error().decode(errors="replace")
        raise QlzxError(f"{what} failed ({rc}): {msg}")


def info() -> str:
    buf = ctypes.create_string_buffer(512)
    lib().qlzx_info(buf, 512)
    return buf.value.decode()
