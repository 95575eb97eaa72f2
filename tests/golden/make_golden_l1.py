"""Generate the level-1 golden fixtures from the *reference* code.

Run in the build container (needs /root/reference):  python tests/golden/make_golden_l1.py

The Go API's level 1 (quicklz/quicklz.go, a QuickLZ.java 1.5.0 translation) is pinned
through the reference quicklz.c compiled at QuickLZ level 1 (oracle/Makefile ->
oracle/_ref/libqlzref_l1.so; the same sources, -DQLZ_COMPRESSION_LEVEL=1).  For every
input the fixture holds the input bytes and the reference level-1 stream `ref`.  The
tests check that (a) the oracle and the GPU decode `ref` to the input (the formats are
one), and (b) the oracle's and the GPU's Go Compress(src, 1) bytes equal `ref` after the
header, except where the Go encoder differs by construction: the 9-byte header always
(C uses 3 bytes below 256 B), no 9-byte core minimum, and a bail-out that counts the
header (`go_quirk` marks those cases, whose output is then checked by round trip through
the reference decoder here and the oracle/GPU decoders in the tests).

Only data is written (inputs and expected outputs); no reference source.
"""
from __future__ import annotations

import json
import os
import random
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)

from oracle import oracle as O  # noqa: E402

SIZES = [1, 2, 4, 5, 9, 10, 11, 12, 13, 20, 31, 32, 33, 100, 255, 256, 300, 1000, 4096, 4097, 16384, 65536]


def inputs(rng: random.Random):
    out = []
    for n in SIZES:
        out.append(("zeros", n, bytes(n)))
        out.append(("rand", n, bytes(rng.getrandbits(8) for _ in range(n))))
        out.append(("ab", n, (b"ab" * (n // 2 + 1))[:n]))
        out.append(("text", n, O.gen_text(17, n, n)))
        out.append(("image", n, O.gen_image(19, n, n)))
        runs = bytearray()
        while len(runs) < n:
            runs += bytes([rng.getrandbits(2)]) * rng.randint(1, 40)
        out.append(("runs", n, bytes(runs[:n])))
    return out


def main():
    if O.ref_l1() is None:
        sys.exit("oracle/_ref/libqlzref_l1.so is not built (needs /root/reference)")
    rng = random.Random(20261016)
    blob = bytearray()
    vecs = []

    def put(b: bytes):
        off = len(blob)
        blob.extend(b)
        return [off, len(b)]

    for kind, n, data in inputs(rng):
        ref = O.ref_l1_compress(data)
        assert O.ref_l1_decompress(ref) == data
        go = O.compress_go_l1(data)
        hdr = 9 if ref[0] & 2 else 3
        quirk = go[9:] != ref[hdr:]
        if quirk:   # the Go encoder's own output must still be a reference level-1 stream
            assert O.ref_l1_decompress(go) == data, (kind, n)
        vecs.append({"name": f"{kind}_{n}", "input": put(data), "ref": put(ref), "go_quirk": quirk})
    with open(os.path.join(HERE, "qlz_l1_vectors.bin"), "wb") as f:
        f.write(blob)
    with open(os.path.join(HERE, "golden_l1.json"), "w") as f:
        json.dump({"generator": "tests/golden/make_golden_l1.py",
                   "reference": "quicklz/quicklz.c at QLZ_COMPRESSION_LEVEL 1 (oracle/_ref/libqlzref_l1.so)",
                   "vectors": vecs}, f, indent=0)
    print(f"{len(vecs)} level-1 vectors, {len(blob)} bytes, "
          f"{sum(v['go_quirk'] for v in vecs)} with Go-encoder quirks")


if __name__ == "__main__":
    main()
