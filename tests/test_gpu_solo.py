"""GPU parity of the single-call latency path (csrc/qlzx_decode_solo.hip): qlz_decompress on one
block (dsize <= 64 KiB, csize <= 64 KiB) runs the workgroup-parallel parse and decode.  Bytes and
statuses must equal the oracle's (oracle/qlz_oracle.c, pinned to quicklz.c by the golden
vectors) on valid, corrupted and truncated streams."""
import ctypes

import numpy as np
import pytest

from oracle import oracle as O

pytestmark = pytest.mark.gpu

SOLO_MAX_CSIZE = 65536


def _hdr_sizes(c: bytes):
    if c[0] & 2:
        return int.from_bytes(c[1:5], "little"), int.from_bytes(c[5:9], "little")
    return c[1], c[2]


def _solo(L, c: bytes):
    """qlz_decompress(c) -> (status, bytes); the header's csize is what the call reads."""
    csize, dsize = _hdr_sizes(c)
    src = ctypes.create_string_buffer(bytes(c) + bytes(max(0, csize - len(c)) + 16))
    out = ctypes.create_string_buffer(max(dsize, 1))
    n = L.qlz_decompress(src, out, None)
    st = L.qlzx_last_status()
    return st, out.raw[:n]


def _all_literal_stream(data: bytes) -> bytes:
    """A level-3 stream of literals only (31 per control word), long header: valid for
    quicklz.c's decoder though its encoder would store such a block raw."""
    body = bytearray()
    for i in range(0, len(data), 31):
        body += (0x80000000).to_bytes(4, "little") + data[i:i + 31]
    csize = 9 + len(body)
    return bytes([0x4F]) + csize.to_bytes(4, "little") + len(data).to_bytes(4, "little") + bytes(body)


def _cases():
    rng = np.random.default_rng(11)
    out = []
    for n in (1, 2, 9, 10, 11, 12, 31, 32, 35, 36, 100, 255, 256, 257, 1000, 4095, 4096, 4097, 16383,
              16384, 16385, 20000, 32767, 32768, 32769, 40000, 65535, 65536):
        out.append(O.gen_text(0x501, n, n))
    for n in (17000, 17400, 17500):  # stored / compressed around the small path's 17 KiB stream bound
        out.append(O.gen_image(0x504, n, n))
    for n in (64, 4096, 30000, 65536):
        out.append(b"a" * n)
        out.append((b"abc" * n)[:n])
        out.append(bytes(rng.integers(0, 4, n, dtype=np.uint8)))
        out.append(O.gen_image(0x502, n, n))
    return out


def test_solo_round_trips(cuda):
    from gobeansdb_amd import _lib
    L = _lib.lib()
    for x in _cases():
        c = O.compress(x)
        assert len(c) <= SOLO_MAX_CSIZE
        st, y = _solo(L, c)
        assert st == 0 and y == x, (len(x), st)


def test_solo_golden(cuda, golden):
    from gobeansdb_amd import _lib
    L = _lib.lib()
    for v in golden.vectors:
        c, x = golden.get(v["c_out"]), golden.get(v["input"])
        st, y = _solo(L, c)
        assert st == 0 and y == x, v["name"]


@pytest.mark.parametrize("n", [15400, 15420, 58000, 65536])
def test_solo_all_literal_stream(cuda, n):
    """Literal-only streams: the largest the small LDS path takes (15400 B -> csize 17397 <= 17408)
    and one past it (15420 B -> 17421), the largest the latency path takes (58000 B -> csize 65493)
    and one past it (64 KiB -> csize 74005, the batch decoder)."""
    from gobeansdb_amd import _lib
    L = _lib.lib()
    x = O.gen_image(0x503, n, n)
    c = _all_literal_stream(x)
    assert (len(c) <= SOLO_MAX_CSIZE) == (n != 65536)
    assert (len(c) <= 17408) == (n == 15400)
    ost, od = O.decompress(c)
    assert ost == 0 and od == x
    st, y = _solo(L, c)
    assert st == 0 and y == x


def test_solo_dsize_zero_streams(cuda):
    """Compressed streams that declare dsize 0: OK with nothing written iff csize is the header
    alone or header + 9 (the oracle's C5 rule, oracle/qlz_oracle.c:197,228), else corrupt."""
    from gobeansdb_amd import _lib
    L = _lib.lib()
    cases = []
    for body in (b"", bytes(9), bytes(5), b"\xff" * 9, (0x80000000).to_bytes(4, "little") + b"abc"):
        cases.append(bytes([0x4D, 3 + len(body), 0]) + body)
        cs = 9 + len(body)
        cases.append(bytes([0x4F]) + cs.to_bytes(4, "little") + bytes(4) + body)
    for c in cases:
        ost, od = O.decompress(c)
        st, y = _solo(L, c)
        assert st == ost and y == b"", (c.hex(), st, ost)


@pytest.mark.parametrize("n", [300, 16384, 30000, 65536])
def test_solo_corrupt_matches_oracle(cuda, n):
    """Byte flips after the header and truncations (csize field rewritten): status and bytes
    == the oracle's; the batch decoder (K1 + K2b) agrees on the same streams."""
    from gobeansdb_amd import _lib
    L = _lib.lib()
    rng = np.random.default_rng(n)
    base = [O.compress(O.gen_text(0x600 + j, n, n)) for j in range(4)]
    base.append(O.compress((b"xyz" * n)[:n]))
    cases = []
    for c in base:
        hdr = 9 if c[0] & 2 else 3
        for _ in range(40 if n < 60000 else 16):
            b = bytearray(c)
            for _ in range(int(rng.integers(1, 4))):
                b[int(rng.integers(hdr, len(b)))] = int(rng.integers(0, 256))
            cases.append(bytes(b))
        for _ in range(4):
            cut = int(rng.integers(hdr + 1, len(c)))
            b = bytearray(c[:cut])
            if b[0] & 2:
                b[1:5] = cut.to_bytes(4, "little")
            else:
                b[1] = cut
            cases.append(bytes(b))
    bad = 0
    for c in cases:
        ost, od = O.decompress(c)
        st, y = _solo(L, c)
        assert st == ost, (len(c), st, ost)
        if st == 0:
            assert y == od
        bad += st != 0
    assert bad > len(cases) // 4   # the corruptions were exercised, not all benign
    # the batch path on the same streams
    from test_gpu_codec import _gpu_decompress
    outs, sts, _ = _gpu_decompress(cases)
    for c, o, s in zip(cases, outs, sts):
        st, y = _solo(L, c)
        assert s == st
        if s == 0:
            assert o == y
