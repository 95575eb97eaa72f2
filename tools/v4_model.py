"""CPU model of the round-4 decoder pair (qlzx_decode_v4.hip), lane for lane (tools only).

K1 (k_dec_parse4): one lane's step loop over a whole stream (no ring: every byte is "landed").
K2 (k_dec_chunk4): the wave's batches (64 items) and chunks (256 B) with the u32 key ring, the
max-scan fill, pointer jumping over the chunk's own slots and the window/HBM gather.
Checked against oracle.decompress on golden-like inputs: python tools/v4_model.py
"""
from __future__ import annotations

import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from oracle import oracle as O  # noqa: E402

M32 = 0xFFFFFFFF


def ctz(x):
    return (x & -x).bit_length() - 1


def clz(x):
    return 32 - x.bit_length()


def code(b0):
    ty = (b0 & 3) + (1 if (b0 & 127) == 3 else 0)
    return (0x32110 >> (4 * ty)) & 15


def k1(src):
    hdr = 9 if src[0] & 2 else 3
    csize = len(src)
    ip, g, cwr, cwg, ra, rb, rec_ip = hdr, 0, 1, 0, 0, 0, 0
    recs = []
    st = 0
    while True:
        gb = cwr == 1
        rem = csize - ip
        run = min(ctz(cwr), rem)
        q = ip + run
        rest = cwr >> run
        hasm = (not gb) and rest != 1 and (rest & 1) and q < csize
        end = ip + (4 if gb else 1) > csize
        if end:
            break
        w = int.from_bytes(bytes(src[q:q + 4]).ljust(4, b"\0"), "little")
        e = code(w & 0xFF)
        bad = (gb and ((w >> 31) == 0)) or (hasm and q + e + 1 > csize)
        if gb and g > 0:
            recs.append((rec_ip, cwg, ra, rb))
        if bad:
            st = 2
            break
        kb = (1 << (clz(cwr) + run)) if hasm else 0
        if gb:
            rec_ip, cwg, g = ip, w, g + 1
            ip, cwr, ra, rb = ip + 4, w, 0, 0
        else:
            ip = q + (e + 1 if hasm else 0)
            cwr = rest >> 1 if hasm else rest
            ra |= kb if e & 1 else 0
            rb |= kb if e & 2 else 0
    if st == 0 and g > 0:
        recs.append((rec_ip, cwg, ra, rb))
    if st == 0 and g == 0:
        st = 2
    nitems = (g - 1) * 31 + clz(cwr) if g else 0
    return st, recs, nitems


def decode_tok(t):
    ty = (t & 3) + (1 if (t & 127) == 3 else 0)
    if ty == 0:
        return (t & 0xFF) >> 2, 3, 1
    if ty == 1:
        return (t & 0xFFFF) >> 2, 3, 2
    if ty == 2:
        return (t & 0xFFFF) >> 6, ((t >> 2) & 15) + 3, 2
    if ty == 3:
        return (t >> 7) & 0x1FFFF, ((t >> 2) & 0x1F) + 2, 3
    return t >> 15, ((t >> 7) & 255) + 3, 4


def k2(src, recs, nitems, dsize, W=4096, MR=512, CH=256):
    csize = len(src)
    hdr = 9 if src[0] & 2 else 3
    tail_from = dsize - 11 if dsize > 10 else 0
    win = bytearray(W)
    mk = [0] * MR
    dst = bytearray(dsize)
    D = bt = c = cin = 0
    tail = complete = False
    pend = []  # (d, key, lit)
    nb = (nitems + 63) // 64

    def batch():
        nonlocal D, bt, tail, complete, pend
        for (d, key, lit) in pend:  # flush: every pending item starts below c + CH <= c + MR
            assert d < c + MR
            mk[d & (MR - 1)] = key
            if lit is not None:
                win[d & (W - 1)] = lit
        pend = []
        items = []
        for lane in range(64):
            I = bt * 64 + lane
            v = I < nitems
            if not v:
                items.append((False, False, 0, 0, 0, 0, 0))
                continue
            g, k = divmod(I, 31)
            ip, m, a, b = recs[g]
            low = (1 << k) - 1
            pos = ip + 4 + k + bin(a & low).count("1") + 2 * bin(b & low).count("1")
            ism = (m >> k) & 1
            t = int.from_bytes(bytes(src[pos:pos + 4]).ljust(4, b"\0"), "little")
            off, mlen, tl = decode_tok(t)
            ln = mlen if ism else 1
            items.append((True, bool(ism), off, ln, tl if ism else 1, pos, t & 0xFF))
        incl = 0
        ds = []
        for it in items:
            ds.append(D + incl)
            incl += it[3]
        total = incl
        bad = False
        lasts = []
        if tail or D + total > tail_from:
            tail_lane = 64
            if not tail:
                for lane, it in enumerate(items):
                    if it[0] and ds[lane] < dsize and not it[1] and ds[lane] >= tail_from:
                        tail_lane = lane
                        break
            else:
                tail_lane = 0
            tail = tail or tail_lane < 64 or any(it[0] and ds[ln] < dsize and not it[1] and ds[ln] >= tail_from
                                                  for ln, it in enumerate(items))
            for lane, it in enumerate(items):
                v, ism, off, ln, tl, pos, lit = it
                d = ds[lane]
                live = v and d < dsize
                mok = off >= 3 and off <= d and d + ln + 4 <= dsize and lane < tail_lane
                last = live and d + ln == dsize
                ip_end = pos + tl
                eok = ip_end == csize or (ip_end < hdr + 9 and csize == hdr + 9)
                if live and ((ism and not mok) or (last and not eok)):
                    bad = True
                lasts.append(last)
        else:
            for lane, it in enumerate(items):
                if it[1] and (it[2] < 3 or it[2] > ds[lane]):
                    bad = True
        if bad:
            return False
        complete = any(lasts)
        pend = []
        for lane, it in enumerate(items):
            v, ism, off, ln, tl, pos, lit = it
            d = ds[lane]
            if not (v and d < dsize):
                continue
            key = (d << 16) | (off if ism else 0)
            if d < c + MR:
                assert mk[d & (MR - 1)] == 0, "marker slot in use"
                mk[d & (MR - 1)] = key
                if not ism:
                    win[d & (W - 1)] = lit
            else:
                pend.append((d, key, None if ism else lit))
        D += total
        bt += 1
        return True

    def chunks():
        nonlocal c, cin, pend
        while c < dsize and (complete or D >= c + CH):
            keep = []
            for (d, key, lit) in pend:
                if d < c + MR:
                    mk[d & (MR - 1)] = key
                    if lit is not None:
                        win[d & (W - 1)] = lit
                else:
                    keep.append((d, key, lit))
            pend = keep
            base = c & (MR - 1)
            m = mk[base:base + CH]
            f = []
            run = cin
            for j in range(CH):
                run = max(run, m[j])
                f.append(run)
            cin = max(cin, max(m))
            s = [c + j - (f[j] & 0xFFFF) for j in range(CH)]
            # pointer jumping over the chunk's slots
            sp = list(s)
            q = [(s[j] - c) & M32 < j for j in range(CH)]
            while any(q):
                t = [sp[(s[j] if q[j] else c + j) - c] for j in range(CH)]
                q = [((t[j] - c) & M32) < ((s[j] - c) & M32) for j in range(CH)]
                s = t
                sp = list(s)
            lo = c + MR - W if c + MR > W else 0
            out = bytes((win[x & (W - 1)] if x >= lo else dst[x]) for x in s)
            for j in range(CH):
                win[(c + j) & (W - 1)] = out[j]
                if c + j < dsize:
                    dst[c + j] = out[j]
            for j in range(CH):
                mk[base + j] = 0
            c += CH
        return c >= dsize

    while True:
        if bt >= nb:
            return 2, None
        if not batch():
            return 2, None
        if chunks():
            break
    return 0, bytes(dst)


def decode(src, ch=256):
    src = bytes(src)
    hdr = 9 if src[0] & 2 else 3
    dsize = O.size_decompressed(src) if hasattr(O, "size_decompressed") else (
        int.from_bytes(src[5:9], "little") if src[0] & 2 else src[2])
    if not src[0] & 1:
        return 0, src[hdr:hdr + dsize]
    st, recs, nitems = k1(src)
    if st:
        return st, None
    return k2(src, recs, nitems, dsize, CH=ch)


def main():
    import numpy as np
    rng = np.random.default_rng(5)
    cases = [O.gen_text(3, k, n) for k, n in enumerate((1, 5, 13, 64, 255, 256, 257, 1000, 4097, 16384, 30000))]
    cases += [bytes(5000), b"ab" * 3000 + b"c", np.resize(rng.integers(0, 256, 7, dtype=np.uint8), 9000).tobytes()]
    cases += [O.gen_image(4, k, 16384) for k in range(3)]
    for ch in (256, 512):
        for k, p in enumerate(cases):
            comp = O.compress(p)
            st, out = decode(comp, ch)
            assert st == 0 and out == p, (ch, k, len(p), st)
    print("v4 model ok on", len(cases), "cases, chunks of 256 and 512 B")


if __name__ == "__main__":
    main()
