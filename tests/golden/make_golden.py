"""Generate the committed golden fixtures from the *reference* code.

Run in the build container (needs /root/reference):  python tests/golden/make_golden.py

- codec vectors: inputs of several classes/sizes and the output of the reference
  qlz_compress (quicklz/quicklz.c compiled unchanged by oracle/Makefile into
  oracle/_ref/libqlzref.so; destination zero-filled), plus the
  reference crc32_write (store/crc32.go preamble, oracle/_ref/libcrc32ref.so).
- records.data: a small .data chunk in the store/datafile.go layout (24-B header,
  key, value, 256-B padding) whose values went through the TryCompress policy of
  store/item.go:120-161 using the reference codec, and whose CRCs come from the
  reference crc32_write.

Only data is written (inputs and expected outputs); no reference source.
"""
from __future__ import annotations

import json
import os
import random
import struct
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)

from oracle import oracle as O  # noqa: E402

KAT = (b"LZ compression is based on finding repeated strings: Five, six, seven, eight, nine, "
       b"fifteen, sixteen, seventeen, fifteen, sixteen, seventeen.")   # quicklz_test.go:9

SIZES = [1, 2, 3, 4, 5, 8, 9, 10, 11, 12, 13, 20, 31, 32, 33, 62, 63, 100, 215, 216, 217, 255,
         256, 300, 1000, 4096, 4097, 16384]
BIG = [65536]


def inputs(rng: random.Random):
    out = []
    for n in SIZES + BIG:
        out.append(("zeros", n, bytes(n)))
        out.append(("rand", n, bytes(rng.getrandbits(8) for _ in range(n))))
        out.append(("ab", n, (b"ab" * (n // 2 + 1))[:n]))
        out.append(("text", n, O.gen_text(7, n, n)))
        out.append(("image", n, O.gen_image(9, n, n)))
        t = bytearray(O.gen_text(3, n, n))
        for j in range(n):
            if rng.random() < 0.42:
                t[j] = rng.getrandbits(8)
        out.append(("noisy", n, bytes(t)))
    out.append(("kat", len(KAT), KAT))
    # long runs: maximum match length (255) and overlapping offset-3 copies
    out.append(("runs", 5000, (b"abc" * 300 + bytes(1000) + b"xyz" * 700 + bytes(900))[:5000]))
    # offset limit: a 2 KiB random chunk repeated 140,000 B later (> 131071) and 100,000 B later
    chunk = bytes(rng.getrandbits(8) for _ in range(2048))
    filler = O.gen_text(5, 1, 150000)
    far = bytearray(filler)
    far[0:2048] = chunk
    far[100000:102048] = chunk
    far[142000:144048] = chunk
    out.append(("far", len(far), bytes(far)))
    return out


def main():
    if O.ref() is None:
        sys.exit("reference not available (needs /root/reference)")
    rng = random.Random(20261015)
    blob = bytearray()
    entries = []

    def put(b: bytes):
        off = len(blob)
        blob.extend(b)
        while len(blob) % 16:
            blob.append(0)
        return [off, len(b)]

    for cls, n, data in inputs(rng):
        n = len(data)
        c = O.ref_compress(data)
        crc = O.ref_crc32_write(0xFFFFFFFF, data) ^ 0xFFFFFFFF if data else 0
        crc_c = O.ref_crc32_write(0xFFFFFFFF, c) ^ 0xFFFFFFFF
        e = {"name": f"{cls}_{n}", "cls": cls, "n": n, "input": put(data), "c_out": put(c),
             "crc_in": crc, "crc_c_out": crc_c}
        if cls == "kat":
            e["go_len"] = 116   # quicklz_test.go:13 (Go Compress, 9-byte header)
        entries.append(e)

    with open(os.path.join(HERE, "qlz_vectors.bin"), "wb") as f:
        f.write(blob)
    # ---- records.data (store/datafile.go layout) ----
    recs = []
    data = bytearray()
    values = [
        (b"key", b"value"), (b"key", b"v" * 255), (b"key", bytes(rng.getrandbits(8) for _ in range(400))),
        (b"k" * 200, bytes(rng.getrandbits(8) for _ in range(512))),
    ]
    for i in range(12):
        values.append((b"key_%016x" % i, O.gen_text(21, i, [300, 4096, 16384, 12000, 65536, 777][i % 6])))
    values.append((b"img_key", O.gen_image(4, 0, 8192)))
    values.append((b"img_key2", O.gen_image(4, 3, 8192)))
    values.append((b"big", O.gen_text(22, 0, 200000)))
    for i, (key, value) in enumerate(values):
        flag = 0
        body = value
        recsize = 24 + len(key) + len(value)
        if (recsize + 255) // 256 * 256 > 256:               # store/item.go:129
            trial = value[:10240]                             # item.go:133-136
            cc = O.ref_compress(trial)
            if len(cc) / len(trial) <= 0.7:                   # item.go:145 (float32 compare)
                body = O.ref_compress(value) if len(value) > len(trial) else cc
                flag |= 0x10000                               # item.go:159
        ts, ver = 1700000000 + i, i + 1
        head = struct.pack("<IIiII", ts, flag, ver, len(key), len(body))
        crc = O.ref_crc32_write(0xFFFFFFFF, head)
        crc = O.ref_crc32_write(crc, key)
        crc = O.ref_crc32_write(crc, body) ^ 0xFFFFFFFF
        rec = struct.pack("<I", crc) + head + key + body
        off = len(data)
        data.extend(rec)
        pad = (-len(rec)) % 256
        data.extend(bytes(pad))
        recs.append({"offset": off, "key": key.decode(), "flag": flag, "ver": ver, "ts": ts,
                     "vsz": len(body), "crc": crc, "value": put(value)})
    with open(os.path.join(HERE, "records.data"), "wb") as f:
        f.write(data)
    with open(os.path.join(HERE, "qlz_vectors.bin"), "wb") as f:
        f.write(blob)
    manifest = {
        "generator": "tests/golden/make_golden.py",
        "reference": "douban/gobeansdb quicklz/quicklz.c (1.4.1, level 3) + store/crc32.go crc32_write",
        "settings": {str(k): O.ref()[0].qlz_get_setting(k) for k in range(10)},
        "vectors": entries,
        "records": recs,
    }
    with open(os.path.join(HERE, "golden.json"), "w") as f:
        json.dump(manifest, f, indent=0)
    print(f"{len(entries)} vectors, {len(recs)} records, blob {len(blob)} B, data {len(data)} B")


if __name__ == "__main__":
    main()
