"""Model of the K2 decode schedule on synthetic blocks (tools only, not product code).

Parses level-3 streams from the oracle compressor into items (literal / match with
offset and length) and counts, for a match-batch formulation (literals placed by an
item phase, matches copied 64 per batch), the copy sub-rounds each batch needs under
three readiness rules:
  exact  a match waits for the in-batch matches whose output overlaps its source;
  starts a match waits for the in-batch matches from the last match start at or before
         its source start to the last one before its source end (conservative);
  prefix a match waits for every in-batch match that starts before its source end.
usage: python tools/model_k2.py [--blocks N] [--size 16384] [--batch 64]
"""
from __future__ import annotations

import argparse
import os
import struct
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from oracle import oracle as O  # noqa: E402


def parse_items(c: bytes):
    hdr = 9 if c[0] & 2 else 3
    dsize = struct.unpack_from("<I", c, 5)[0] if hdr == 9 else c[2]
    if not c[0] & 1:
        return dsize, []
    src, dst, cw = hdr, 0, 1
    items = []  # (d, len, off)  off = 0 for literals
    last_matchstart = dsize - 10 - 1  # quicklz.c:503: dst <= last_destination_byte - 10
    cb = c + b"\0" * 8
    while dst < dsize:
        if cw == 1:
            cw = struct.unpack_from("<I", cb, src)[0]
            src += 4
        if dst <= last_matchstart and (cw & 1):
            f = struct.unpack_from("<I", cb, src)[0]
            cw >>= 1
            if (f & 3) == 0:
                off, ml, tl = (f & 0xff) >> 2, 3, 1
            elif (f & 2) == 0:
                off, ml, tl = (f & 0xffff) >> 2, 3, 2
            elif (f & 1) == 0:
                off, ml, tl = (f & 0xffff) >> 6, ((f >> 2) & 15) + 3, 2
            elif (f & 127) != 3:
                off, ml, tl = (f >> 7) & 0x1ffff, ((f >> 2) & 0x1f) + 2, 3
            else:
                off, ml, tl = f >> 15, ((f >> 7) & 255) + 3, 4
            items.append((dst, ml, off))
            src += tl
            dst += ml
        else:
            items.append((dst, 1, 0))
            src += 1
            dst += 1
            cw >>= 1
    return dsize, items


def subrounds(batch, rule):
    n = len(batch)
    starts = [d for d, _, _ in batch]
    ends = [d + l for d, l, _ in batch]
    need = []
    for j, (d, l, off) in enumerate(batch):
        s = d - off
        se = min(s + l, d)
        deps = set()
        if rule == "exact":
            deps = {i for i in range(j) if starts[i] < se and ends[i] > s}
        elif rule == "prefix":
            deps = {i for i in range(j) if starts[i] < se}
        else:
            la = max([i for i in range(j) if starts[i] <= s], default=0 if s < starts[0] else None)
            lb = max([i for i in range(j) if starts[i] < se], default=None)
            if lb is not None and se > starts[0]:
                la = la if la is not None else 0
                deps = set(range(la, lb + 1))
        need.append(deps)
    done = [False] * n
    r = 0
    while not all(done):
        r += 1
        ready = [j for j in range(n) if not done[j] and all(done[i] for i in need[j])]
        for j in ready:
            done[j] = True
    return r


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--blocks", type=int, default=40)
    ap.add_argument("--size", type=int, default=16384)
    ap.add_argument("--batch", type=int, default=64)
    a = ap.parse_args()
    tot_items = tot_match = tot_lit = 0
    sr = {"exact": 0, "starts": 0, "prefix": 0}
    nbat = 0
    long16 = overl = 0
    far = {2048: 0, 4096: 0, 8192: 0}
    for b in range(a.blocks):
        p = O.gen_text(0x5EED2026, b, a.size)
        c = O.compress(p)
        dsize, items = parse_items(c)
        tot_items += len(items)
        ms = [it for it in items if it[2]]
        tot_match += len(ms)
        tot_lit += len(items) - len(ms)
        for d, l, off in ms:
            long16 += l > 16
            overl += off < l
            for w in far:
                far[w] += off > w // 2
        for k in range(0, len(ms), a.batch):
            bt = ms[k:k + a.batch]
            nbat += 1
            for rule in sr:
                sr[rule] += subrounds(bt, rule)
    nb = a.blocks
    print(f"per block: items {tot_items / nb:.0f}, matches {tot_match / nb:.0f}, literals {tot_lit / nb:.0f}, "
          f"ratio {len(c) / a.size:.3f}")
    print(f"match batches/block {nbat / nb:.1f}; sub-rounds per batch: " +
          ", ".join(f"{k} {v / nbat:.2f}" for k, v in sr.items()))
    print(f"matches >16 B {long16 / tot_match:.3f}, overlapping {overl / tot_match:.3f}, "
          f"offset > W/2: " + ", ".join(f"W={w}: {v / tot_match:.3f}" for w, v in far.items()))


if __name__ == "__main__":
    main()
