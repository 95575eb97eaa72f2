"""The GF(2) CRC shift/combine identities the kernels rely on (no GPU)."""
import random
import zlib

POLY = 0xEDB88320


def mulmod(a, b):
    p = 0
    for _ in range(32):
        if a & 0x80000000:
            p ^= b
        a = (a << 1) & 0xFFFFFFFF
        b = (b >> 1) ^ POLY if b & 1 else b >> 1
    return p


def pow8():
    x = 0x40000000
    for _ in range(3):
        x = mulmod(x, x)
    out = []
    for _ in range(64):
        out.append(x)
        x = mulmod(x, x)
    return out


P8 = pow8()


def shift(s, n):
    k = 0
    while n:
        if n & 1:
            s = mulmod(P8[k], s)
        n >>= 1
        k += 1
    return s


def raw(data, s=0):
    # store/crc32.go:61-68 without the ~ of the Go wrapper
    return zlib.crc32(data, s ^ 0xFFFFFFFF) ^ 0xFFFFFFFF


def test_shift_is_zero_byte_advance():
    rng = random.Random(3)
    for n in [0, 1, 2, 3, 7, 64, 1000, 4096, 65537]:
        s = rng.getrandbits(32)
        assert shift(s, n) == raw(bytes(n), s)


def test_split_combine():
    rng = random.Random(4)
    for _ in range(50):
        a = bytes(rng.getrandbits(8) for _ in range(rng.randrange(0, 300)))
        b = bytes(rng.getrandbits(8) for _ in range(rng.randrange(0, 300)))
        s = rng.getrandbits(32)
        assert raw(a + b, s) == shift(raw(a, s), len(b)) ^ raw(b, 0)
        assert raw(b, s) == raw(b, 0) ^ shift(s, len(b))
