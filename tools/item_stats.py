"""Item statistics of level-3 streams (tools only, host): what a span-based K2 would save.

Walks the token streams of oracle-compressed synthetic blocks (quicklz.c:513-671 restated as a
token walk: 4-byte control words, a match token's length from its first byte) and reports per
block the control-word groups, literal items, literal runs, matches and match bytes, the match
length distribution and how far back matches reach.
usage: python tools/item_stats.py [kind=text|image] [block_size=16384] [blocks=64]
"""
import os
import struct
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from oracle import oracle as O  # noqa: E402


def walk(c: bytes) -> dict:
    hdr = 9 if c[0] & 2 else 3
    dsize = struct.unpack_from("<I", c, 5)[0] if hdr == 9 else c[2]
    if not c[0] & 1:  # stored
        return dict(groups=0, lits=dsize, runs=1, matches=0, mbytes=0, mlens=[], offs=[])
    cp = c + bytes(4)
    ip, op, cw, prev_lit = hdr, 0, 1, False
    st = dict(groups=0, lits=0, runs=0, matches=0, mbytes=0, mlens=[], offs=[])
    while op < dsize:
        if cw == 1:
            cw = struct.unpack_from("<I", cp, ip)[0]
            ip += 4
            st["groups"] += 1
            prev_lit = False
        if cw & 1:
            t = struct.unpack_from("<I", cp, ip)[0]
            k = t & 3
            if k == 0:
                ml, off, n = 3, (t >> 2) & 63, 1
            elif k == 1:
                ml, off, n = 3, (t >> 2) & 16383, 2
            elif k == 2:
                ml, off, n = ((t >> 2) & 15) + 3, (t >> 6) & 1023, 2
            elif (t >> 2) & 31:
                ml, off, n = ((t >> 2) & 31) + 2, (t >> 7) & 0x1FFFF, 3
            else:
                ml, off, n = ((t >> 7) & 255) + 3, t >> 15, 4
            ip, op = ip + n, op + ml
            st["matches"] += 1
            st["mbytes"] += ml
            st["mlens"].append(ml)
            st["offs"].append(off)
            prev_lit = False
        else:
            st["runs"] += 0 if prev_lit else 1
            prev_lit = True
            ip, op = ip + 1, op + 1
            st["lits"] += 1
        cw >>= 1
    return st


def main():
    kind = sys.argv[1] if len(sys.argv) > 1 else "text"
    bs = int(sys.argv[2]) if len(sys.argv) > 2 else 16384
    nb = int(sys.argv[3]) if len(sys.argv) > 3 else 64
    gen = O.gen_text if kind == "text" else O.gen_image
    tot, ml, of = {}, [], []
    for i in range(nb):
        s = walk(O.compress(gen(7, i, bs)))
        for k in ("groups", "lits", "runs", "matches", "mbytes"):
            tot[k] = tot.get(k, 0) + s[k]
        ml += s["mlens"]
        of += s["offs"]
    per = {k: round(v / nb, 1) for k, v in tot.items()}
    print(f"{kind} {bs} B x {nb}: per block {per}")
    print(f"  items {per['lits'] + per['matches']:.0f}, spans (literal runs + matches) {per['runs'] + per['matches']:.0f}")
    if ml:
        ml, of = np.array(ml), np.array(of)
        print(f"  match length mean {ml.mean():.2f} median {np.median(ml):.0f} p90 {np.percentile(ml, 90):.0f}; "
              f"offset < 256: {(of < 256).mean():.3f}, < 1024: {(of < 1024).mean():.3f}, < 4096: {(of < 4096).mean():.3f}")


if __name__ == "__main__":
    main()
